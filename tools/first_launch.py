"""Where the first imitation launch's ~25 ms goes: the bench's full-env reset
(mode 2) right after the motion tables are loaded, timed with HIP events; then the same reset again,
a plain step, and a reset after the tables are reloaded. Writes JSON to stdout.

  python tools/first_launch.py [--config imitation]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from humanoid_amd.model import load_default_model
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="imitation")
    a = ap.parse_args()
    args = argparse.Namespace(config=a.config, num_envs=4096, clips=128, seed=0, max_contacts=40)
    model = load_default_model()
    out = {}

    def timed(name, fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        out[name] = round(s.elapsed_time(e), 4)

    import time
    t0 = time.perf_counter()
    ro = bench.Rollout(args, model, 0, 0)  # loads the tables, then the full reset (the first launch)
    torch.cuda.synchronize()
    out["rollout_init_s"] = round(time.perf_counter() - t0, 3)
    n = args.num_envs
    ids = torch.arange(n, dtype=torch.int32, device=ro.eng.device)
    ph = torch.as_tensor(np.random.default_rng(1).uniform(0, 1, n).astype(np.float32), device=ro.eng.device)
    reset = lambda: ro.eng.reset_envs(ro.p, ro.em, ids, ph, ro.obs, ro.reset, ro.term)  # noqa: E731
    timed("second_full_reset_ms", reset)
    timed("third_full_reset_ms", reset)
    timed("step_ms", ro.step)
    tables, _, _ = bench.build_workload(args, model, 0)
    ro.eng.load_motions(tables)
    timed("full_reset_after_reload_ms", reset)
    timed("full_reset_again_ms", reset)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
