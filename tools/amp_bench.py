"""AMP observation path cost at 4096 envs on the imitation workload (configs[2]).

Device: the policy step (physics + imitation + device resets) with and without the AMP buffers
attached (HIP events on the engine's stream); under rocprofv3 the amp_kernel row gives the launch
alone. Algorithmic HBM bytes of the AMP launch per env
(step update): history shift 2 * 9 * 784 B, row 0 write 784 B, rb rows of the root and 4 key
bodies plus 19 joints' dof state read (5 * 52 + 19 * 24 B) = 15,330 B.

Also probes what this torch does for the reference's un-indexed history assignment
(humanoid_phc.py:1341-1347) on the device: raise (-> the reference's .clone() fallback, a shift)
or an in-place overlapping copy.

Usage: python tools/amp_bench.py [--out profiles/r01/amp_bench.json]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from humanoid_amd.model import load_default_model  # noqa: E402

AMP_BYTES_PER_ENV = 2 * 9 * 784 + 784 + 5 * 52 + 19 * 24


def overlap_probe():
    b = torch.arange(2 * 10 * 196, dtype=torch.float32, device="cuda:0").view(2, 10, 196)
    want = b.clone()
    want[:, 1:] = b[:, :-1].clone()
    try:
        b[:, 1:] = b[:, 0:9]
    except RuntimeError as e:
        return f"raises ({str(e)[:60]}...): the reference falls back to clone(), a shift"
    torch.cuda.synchronize()
    if torch.equal(b, want):
        return "no raise; result equals the shift"
    smeared = all(torch.equal(b[:, k], want[:, 1]) for k in range(1, 10))
    return "no raise; row 0 smeared over the history" if smeared else "no raise; overlapping copy, mixed rows"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    model = load_default_model()
    bargs = bench.parse(["--config", "imitation", "--no-cpu-baseline", "--no-puffer-level"])
    ro = bench.Rollout(bargs, model, 0, 0)
    eng, n = ro.eng, bargs.num_envs
    stream = torch.cuda.current_stream(eng.device)
    buf = torch.zeros(n, 10, 196, device=eng.device)
    demo = torch.zeros_like(buf)

    # the full policy step (physics + imitation + device resets), with and without AMP attached
    res = {"num_envs": n, "num_amp_obs_steps": 10}
    for key, amp in (("env_step_ms", False), ("env_step_with_amp_ms", True)):
        eng.set_amp(buf, demo) if amp else eng.set_amp(None)
        for _ in range(20):
            ro.step()
        torch.cuda.synchronize()
        resets = torch.zeros((), device=eng.device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(a.reps):
            ro.step()
        e1.record(stream)
        torch.cuda.synchronize()
        res[key] = round(e0.elapsed_time(e1) / a.reps, 5)
        for _ in range(50):
            ro.step()
            resets += ro.reset.float().sum()
        res["reset_fraction"] = round(float(resets) / (50 * n), 4)
    ms = res["env_step_with_amp_ms"] - res["env_step_ms"]
    res["amp_overhead_ms"] = round(ms, 5)
    res["amp_algorithmic_bytes_per_env"] = AMP_BYTES_PER_ENV
    res["amp_achieved_GBps"] = round(AMP_BYTES_PER_ENV * n / (ms * 1e-3) / 1e9, 1) if ms > 0 else None
    res["torch_overlapping_history_assignment"] = overlap_probe()
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
