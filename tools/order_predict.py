"""Can an env's next physics launch cost be predicted from the state the launch starts from? (DESIGN
§4.1 "Dispatch order": the shipped order uses the previous launch's cycles, lag-1 correlation
0.6-0.8 on configs[2] tracking and configs[4].) Dumps, per launch and env, the launch's wave cycles
(HE_BUF_PHYS_COST) and what the state after it holds: the last solve's row count (warm-start cache
word 7), its row keys (bodies of every row: the leg / full support class), the contact slots and the
reset flags; then, offline, the correlation of each predictor with the next launch's cycles and the
makespan of greedy dispatch over 2048 slots under orders built from them (tools/order_sim.py).

  python tools/order_predict.py dump DIR [LAUNCHES]      (GPU)
  python tools/order_predict.py --offline DIR           (CPU)
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from order_sim import SLOTS, classes32, makespan  # noqa: E402

CACHE_KEYS, CACHE_NR = 8, 7  # include/humanoid_engine.h cache layout


def dump(d, launches):
    import torch
    import bench
    from humanoid_amd.model import load_default_model
    os.makedirs(d, exist_ok=True)
    model = load_default_model()
    for name, cfg in (("tracking", "tracking"), ("imitation", "imitation"), ("dr", "dr")):
        args = argparse.Namespace(config=cfg, num_envs=4096, clips=128, seed=0, max_contacts=40)
        ro = bench.Rollout(args, model, 0, 0)
        for _ in range(10):
            ro.step()
        rec = {k: [] for k in ("cost", "nr", "keys", "slots", "reset")}
        for _ in range(launches):
            ro.step()
            torch.cuda.synchronize()
            cache = ro.eng.contact_cache.clone().cpu().numpy()
            rec["cost"].append(ro.eng.physics_cost.cpu().numpy().view(np.uint32).astype(np.int64))
            rec["nr"].append(cache[:, CACHE_NR].view(np.int32).copy())
            rec["keys"].append(cache[:, CACHE_KEYS:CACHE_KEYS + 32].view(np.uint32).copy())
            rec["slots"].append(ro.eng.num_contacts.clone().cpu().numpy())
            rec["reset"].append(ro.reset.cpu().numpy().astype(np.int8))
        np.savez_compressed(os.path.join(d, name + ".npz"), **{k: np.stack(v) for k, v in rec.items()})
        print(name, "dumped", flush=True)


def support_all(keys, nr):
    """Per env: whether some row of the last solve reaches a body past the legs (bodies 9-23), from
    its 16-bit keys (b0 bits 0-4, b1 + 2 bits 5-9)."""
    n = keys.shape[0]
    k = np.stack([keys & 0xFFFF, keys >> 16], axis=2).reshape(n, 64)[:, :63]
    live = np.arange(63)[None, :] < nr[:, None]
    b0 = k & 31
    b1 = ((k >> 5) & 31).astype(np.int64) - 2
    far = (b0 > 8) | (b1 > 8)
    return (far & live).any(axis=1)


def offline(d):
    out = {}
    for f in sorted(os.listdir(d)):
        if not f.endswith(".npz"):
            continue
        z = np.load(os.path.join(d, f))
        C, NR, K, S, R = z["cost"], z["nr"], z["keys"], z["slots"], z["reset"]
        L = C.shape[0]
        feats = {}
        for i in range(1, L):
            full = support_all(K[i - 1], NR[i - 1])
            X = np.stack([np.ones(C.shape[1]), NR[i - 1], NR[i - 1] > 32, full, S[i - 1], R[i - 1],
                          C[i - 1] / C[i - 1].mean()], axis=1).astype(np.float64)
            feats.setdefault("X", []).append(X)
            feats.setdefault("y", []).append(C[i].astype(np.float64))
        Xs, ys = feats["X"], feats["y"]
        # fit on the first half of the launches, evaluate on the second
        h = len(Xs) // 2
        A = np.concatenate(Xs[:h])
        b = np.concatenate(ys[:h])
        coef, *_ = np.linalg.lstsq(A, b, rcond=None)
        res = {"launches": L, "fit_on": h, "coef[1, nr, nr>32, full, slots, reset, prev/mean]": [round(float(c), 1) for c in coef]}
        corr = {"previous launch's cycles": [], "state predictor": [], "state + previous": []}
        spans = {"32 classes, every 8 launches (shipped)": [], "32 classes from the previous launch": [],
                 "32 classes from the state predictor": [], "launch's own cycles (unattainable)": []}
        coef_s, *_ = np.linalg.lstsq(A[:, :6], b, rcond=None)
        for j in range(h, len(Xs)):
            i = j + 1
            c = C[i]
            pred_sp = Xs[j] @ coef
            pred_s = Xs[j][:, :6] @ coef_s
            corr["previous launch's cycles"].append(np.corrcoef(C[i - 1], c)[0, 1])
            corr["state predictor"].append(np.corrcoef(pred_s, c)[0, 1])
            corr["state + previous"].append(np.corrcoef(pred_sp, c)[0, 1])
            stale = C[8 * ((i - 1) // 8)] if i > 8 * ((i - 1) // 8) else C[i - 1]
            spans["32 classes, every 8 launches (shipped)"].append(makespan(c, classes32(stale)))
            spans["32 classes from the previous launch"].append(makespan(c, classes32(C[i - 1])))
            spans["32 classes from the state predictor"].append(makespan(c, classes32(np.maximum(pred_sp, 1).astype(np.int64))))
            spans["launch's own cycles (unattainable)"].append(makespan(c, classes32(c)))
        base = np.mean(spans["32 classes, every 8 launches (shipped)"])
        res["correlation_with_next_launch"] = {k: round(float(np.mean(v)), 3) for k, v in corr.items()}
        res["makespan_vs_shipped"] = {k: round(float(np.mean(v)) / base, 4) for k, v in spans.items()}
        res["lower_bound_vs_shipped"] = round(float(np.mean([max(C[j + 1].sum() / SLOTS, C[j + 1].max())
                                                             for j in range(h, len(Xs))])) / base, 4)
        out[f[:-4]] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "--offline":
        offline(sys.argv[2])
    else:
        dump(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 32)
