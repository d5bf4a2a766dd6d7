"""Which first-launch effect makes the setup's first full-env reset (imitation kernel, mode 2) take
16-30 ms on the GPU (rocprofv3 kernel traces profiles/r04/first_launch_trace.json)?
The bench's Rollout setup runs with its reset deferred; then, in a fresh process per mode, HIP
events time:
  plain      the full reset first (as the bench does)
  one_env    a reset of env 0 alone first (the kernel's first dispatch, negligible work), then the full reset
  warm_mem   a 256 MB device copy first (memory / fabric clocks busy), then the full reset
  physics    one physics launch first (another of the engine's kernels), then the full reset
  python tools/first_launch2.py MODE   -> one JSON line
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse
    import numpy as np
    import torch
    import bench
    from humanoid_amd.engine import Engine
    from humanoid_amd.model import load_default_model
    mode = sys.argv[1]
    args = argparse.Namespace(config="imitation", num_envs=4096, clips=128, seed=0, max_contacts=40, fused=False)
    model = load_default_model()
    deferred = []
    real = Engine.reset_envs
    Engine.reset_envs = lambda self, *a: deferred.append(a)
    t0 = time.perf_counter()
    ro = bench.Rollout(args, model, 0, 0)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    Engine.reset_envs = real
    p, em, ids, phases, obs, reset, term = deferred[0]

    def timed(fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        w = time.perf_counter()
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        return round(s.elapsed_time(e), 4), round((time.perf_counter() - w) * 1e3, 4)

    out = {"mode": mode, "setup_s": round(setup_s, 3)}
    if mode == "one_env":
        out["pre_ms"] = timed(lambda: ro.eng.reset_envs(p, em, ids[:1], phases[:1], obs, reset, term))
    elif mode == "warm_mem":
        a = torch.empty(64 * 1024 * 1024, device="cuda")
        b = torch.empty_like(a)
        out["pre_ms"] = timed(lambda: b.copy_(a))
    elif mode == "physics":
        out["pre_ms"] = timed(lambda: ro.eng.simulate(2))
    out["full_reset_ms"] = timed(lambda: ro.eng.reset_envs(p, em, ids, phases, obs, reset, term))
    out["full_reset_again_ms"] = timed(lambda: ro.eng.reset_envs(p, em, ids, phases, obs, reset, term))
    out["first_step_ms"] = timed(ro.step)
    out["second_step_ms"] = timed(ro.step)
    out["definition"] = "(event ms, host wall ms) per launch"
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
