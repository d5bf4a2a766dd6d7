"""Eval-path cost at 4096 envs on the imitation workload (configs[2]).

Device: the imitation launch with and without eval recording attached (HIP events, same stream).
Reference flow (host): the per-step D2H copies of body_pos / body_pos_gt (humanoid_phc.py:167-168)
and, per batch, the restated compute_metrics_lite over 4096 motions of 149 frames (the smpl_sim
call at phc_train.py:188; here oracle/eval_metrics.py, numpy).

Usage: python tests/diag/eval_bench.py [--out profiles/r01/eval_bench.json]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from humanoid_amd.eval import EvalRecorder  # noqa: E402
from humanoid_amd.model import load_default_model  # noqa: E402
from oracle import eval_metrics as EM  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--host-motions", type=int, default=512, help="motions in the timed host sample")
    a = ap.parse_args()
    model = load_default_model()
    bargs = bench.parse(["--config", "imitation", "--no-cpu-baseline", "--no-puffer-level"])
    ro = bench.Rollout(bargs, model, 0, 0)
    eng, n = ro.eng, bargs.num_envs
    rec = EvalRecorder(eng, n, eng.device)
    rec.set_num_steps(torch.full((n,), 150, dtype=torch.int32))
    stream = torch.cuda.current_stream(eng.device)

    def imit(with_eval):
        if with_eval:
            rec.attach()
            rec.frame = (rec.frame + 1) % 140
        else:
            rec.detach()
        eng.imitation_step(ro.p, ro.em, ro.obs, ro.rew, ro.raw, ro.reset, ro.term)

    res = {"num_envs": n}
    for key, we in (("imitation_ms", False), ("imitation_with_eval_ms", True)):
        imit(we)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(a.reps):
            imit(we)
        e1.record(stream)
        torch.cuda.synchronize()
        res[key] = round(e0.elapsed_time(e1) / a.reps, 5)
    res["eval_recording_overhead_ms"] = round(res["imitation_with_eval_ms"] - res["imitation_ms"], 5)
    # reference flow: per-step host copies ...
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        rec.body_pos.cpu().numpy()
        rec.body_pos_gt.cpu().numpy()
    res["host_copy_per_step_ms"] = round((time.perf_counter() - t0) / 20 * 1e3, 4)
    # ... and compute_metrics_lite at batch end (sampled, scaled to 4096 motions)
    rng = np.random.default_rng(0)
    m, T = a.host_motions, 149
    gt = [rng.standard_normal((T, 24, 3)).astype(np.float32) for _ in range(m)]
    pr = [g + 0.01 * rng.standard_normal(g.shape).astype(np.float32) for g in gt]
    t0 = time.perf_counter()
    EM.compute_metrics_lite(pr, gt)
    dt = time.perf_counter() - t0
    res["host_metrics_per_batch_ms"] = round(dt / m * n * 1e3, 1)
    res["host_metrics_sample"] = f"{m} motions x {T} frames timed, scaled to {n}"
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
