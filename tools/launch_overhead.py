"""Step-loop overheads at 4096 envs (configs[1]): the bench's timed loop with per-step HIP events,
the same loop without events, and the steps replayed from a captured HIP graph.

Usage: python tools/launch_overhead.py [--steps 200]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from humanoid_amd.model import load_default_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--config", default="standstill")
    a = ap.parse_args()
    model = load_default_model()
    ro = bench.Rollout(bench.parse(["--config", a.config, "--no-cpu-baseline", "--no-puffer-level"]), model, 0, 0)
    for _ in range(20):
        ro.step()
    torch.cuda.synchronize()
    res = {}

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e3

    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(a.steps)]
    res["loop_with_events_ms"] = timed(lambda: [ro.step(evs[k]) for k in range(a.steps)])
    res["loop_no_events_ms"] = timed(lambda: [ro.step() for _ in range(a.steps)])
    # graph: capture a block of steps (each step index baked in), replay
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    block = 50
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(block):
                ro.step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    reps = max(1, a.steps // block)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    res["graph_replay_ms"] = (time.perf_counter() - t0) / (reps * block) * 1e3
    res = {k: round(v, 4) for k, v in res.items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
