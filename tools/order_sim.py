"""Dispatch-order study (DESIGN §4.1 "Dispatch order"): per-env wave cycles of real physics launches
(the engine's cost buffer, HE_BUF_PHYS_COST) on the bench workloads, and the launch makespan that
greedy dispatch over 2048 wave slots (1024 SIMDs x 2 waves; the hardware hands out workgroups in
order as slots free) gives under several orders: workgroup id = env, the shipped heavy-first
partition, a three-class partition (heavy, middle, light last) and the full longest-first sort.
Prints one JSON object.

  python tools/order_sim.py [LAUNCHES]
  python tools/order_sim.py --offline DIR   (the cycles dumped by HE_ORDER_SIM_DUMP=DIR, replayed with
                                             stale orders: profiles/r06/order_costs/)
"""
import argparse
import heapq
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SLOTS = 2048


def makespan(cost, order):
    h = [0] * SLOTS
    heapq.heapify(h)
    end = 0
    for e in order:
        t = heapq.heappop(h) + int(cost[e])
        end = max(end, t)
        heapq.heappush(h, t)
    return end


def orders(cost):
    n = len(cost)
    mean = cost.mean()
    ids = np.arange(n)
    heavy = cost > mean + mean / 16
    out = {"env order": ids, "heavy first (shipped)": np.concatenate([ids[heavy], ids[~heavy]])}
    for frac in (8, 4):
        light = cost < mean - mean / frac
        mid = ~heavy & ~light
        out[f"heavy, middle, light (light < mean - mean/{frac})"] = np.concatenate([ids[heavy], ids[mid], ids[light]])
    out["longest first (sorted)"] = np.argsort(-cost, kind="stable")
    return out


def classes32(c):
    """The shipped round-6 order: 32 classes floor(32 c / mean) - 16 clamped to [0, 31], costliest first."""
    n = len(c)
    ids = np.arange(n)
    k = np.clip((32 * c.astype(np.int64) * n // int(c.sum())) - 16, 0, 31)
    return np.concatenate([ids[k == j] for j in range(31, -1, -1)])


def offline(d):
    """The cycles dumped by a GPU run (HE_ORDER_SIM_DUMP), replayed: each order built from the first
    launch's cycles and kept for the next ones (as the engine keeps it for 8 launches), the makespan
    averaged over those launches, against the shipped order of round 5 (heavy first)."""
    res = {}
    for f in sorted(os.listdir(d)):
        if not f.endswith(".npy"):
            continue
        C = np.load(os.path.join(d, f))
        c0 = C[0]
        n = len(c0)
        ids = np.arange(n)
        cand = orders(c0)
        cand["32 classes, costliest first (round 6)"] = classes32(c0)
        spans = {name: [makespan(C[i], o) for i in range(1, C.shape[0])] for name, o in cand.items()}
        # the same 32-class order rebuilt before every launch from the previous launch's cycles (what a
        # per-launch rebuild could do), and from the launch's own cycles (unattainable: the bound of
        # any cost-ordered dispatch)
        spans["32 classes, rebuilt every launch from the previous one"] = [
            makespan(C[i], classes32(C[i - 1])) for i in range(1, C.shape[0])]
        spans["32 classes from the launch's own cycles (unattainable)"] = [
            makespan(C[i], classes32(C[i])) for i in range(1, C.shape[0])]
        base = np.mean(spans["heavy first (shipped)"])
        res[f[:-4]] = {"launches_replayed": C.shape[0] - 1,
                       "vs_round5_heavy_first": {name: round(float(np.mean(v)) / base, 4) for name, v in spans.items()},
                       "lag1_cost_correlation": [round(float(np.corrcoef(C[i], C[i - 1])[0, 1]), 3)
                                                 for i in range(1, C.shape[0])],
                       "lower_bound_vs_round5": round(float(np.mean([max(C[i].sum() / SLOTS, C[i].max())
                                                                     for i in range(1, C.shape[0])])) / base, 4)}
    print(json.dumps(res, indent=1))


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--offline":
        return offline(sys.argv[2])
    import torch
    import bench
    from humanoid_amd.model import load_default_model
    ap = argparse.ArgumentParser()
    ap.add_argument("launches", nargs="?", type=int, default=8)
    a = ap.parse_args()
    model = load_default_model()
    res = {}
    for name, cfg, track in (("configs[1] standstill", "standstill", False), ("configs[2] tracking", "imitation", True),
                             ("configs[2] fixed action", "imitation", False), ("configs[4] dr", "dr", False)):
        args = argparse.Namespace(config=cfg, num_envs=4096, clips=128, seed=0, max_contacts=40)
        ro = bench.Rollout(args, model, 0, 0)
        for _ in range(10):
            if track:
                ro.tracking_actions()
            ro.step()
        spans = {}
        stats = []
        raw = []
        for _ in range(a.launches):
            if track:
                ro.tracking_actions()
            ro.step()
            torch.cuda.synchronize()
            cost = ro.eng.physics_cost.cpu().numpy().view(np.uint32).astype(np.int64)
            raw.append(cost.copy())
            stats.append((cost.mean(), np.percentile(cost, 50), np.percentile(cost, 98), cost.max(), cost.min()))
            for k, o in orders(cost).items():
                spans.setdefault(k, []).append(makespan(cost, o))
        if os.environ.get("HE_ORDER_SIM_DUMP"):  # the per-env cycles themselves, for offline study
            np.save(os.path.join(os.environ["HE_ORDER_SIM_DUMP"], cfg + ("_track" if track else "") + ".npy"),
                    np.stack(raw))
        base = np.mean(spans["heavy first (shipped)"])
        res[name] = {"per_env_cycles": dict(zip(("mean", "p50", "p98", "max", "min"),
                                                 (float(x) for x in np.mean(stats, axis=0)))),
                     "makespan_cycles": {k: float(np.mean(v)) for k, v in spans.items()},
                     "vs_shipped": {k: round(float(np.mean(v)) / base, 4) for k, v in spans.items()},
                     "lower_bound_sum_over_slots": float(np.mean([s[0] for s in stats]) * 4096 / SLOTS)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
