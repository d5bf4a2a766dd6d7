"""Offline study (DESIGN §11 "Load balance"): the physics launch with envs handed between waves at
physics-step boundaries -- four tasks per env, a free wave slot takes the ready env with the most
remaining work, every task paying a state round trip of `ovh` of its cost -- against the shipped
dispatch order (32 classes from the first launch's cycles, kept), on the committed per-env cycles
(profiles/r06/order_costs/). An upper bound: the remaining work is taken as known.

  python tools/order_chain_sim.py
"""
import heapq
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from order_sim import SLOTS, classes32, makespan  # noqa: E402


def chain_makespan(cost, steps=4, ovh=0.0):
    per = cost * (1.0 + ovh) / steps
    rem = np.full(len(cost), steps)
    ready = [(-float(cost[e]), e) for e in range(len(cost))]
    heapq.heapify(ready)
    slots = [(0.0, w) for w in range(SLOTS)]
    heapq.heapify(slots)
    last = [-1] * SLOTS
    end = 0.0
    while slots:
        t, w = heapq.heappop(slots)
        e = last[w]
        if e >= 0 and rem[e] > 0:  # the step this slot ran leaves its env ready for any slot
            heapq.heappush(ready, (-float(per[e] * rem[e]), e))
        if not ready:
            continue
        _, e = heapq.heappop(ready)
        rem[e] -= 1
        last[w] = e
        heapq.heappush(slots, (t + per[e], w))
        end = max(end, t + per[e])
    return end


def main():
    out = {}
    for name in ("standstill", "imitation_track", "dr"):
        C = np.load(os.path.join(os.path.dirname(HERE), "profiles", "r06", "order_costs", name + ".npy")).astype(np.float64)
        shipped = classes32(C[0].astype(np.int64))
        base = np.mean([makespan(C[i].astype(np.int64), shipped) for i in range(1, C.shape[0])])
        res = {f"step tasks, round trip {ovh:.0%} of a task": round(float(np.mean(
            [chain_makespan(C[i], ovh=ovh) for i in range(1, C.shape[0])])) / base, 4) for ovh in (0.0, 0.03, 0.05)}
        res["lower bound"] = round(float(np.mean([max(C[i].sum() / SLOTS, C[i].max())
                                                  for i in range(1, C.shape[0])])) / base, 4)
        out[name] = {"makespan_vs_shipped": res}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
