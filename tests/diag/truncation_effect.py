"""The contact-capacity truncation made visible on the oracle: the same
fallen / tumbling bodies stepped with the engine's capacity (40 slots / 63 solver rows,
deepest-first row-budgeted reduction) and with the oracle's own 64-slot capacity (no row budget),
and the difference reported:
penetration (lowest contact-candidate gap), CoM trajectory, contacts dropped.

  python tests/diag/truncation_effect.py [--envs 128] [--steps 60] > profiles/r03/truncation_effect.json
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "..", "tests"))

import cases  # noqa: E402
from humanoid_amd import _abi  # noqa: E402
from humanoid_amd.model import load_default_model, pd_action_offset_scale  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(hm, model, root, dof, targets, cap, steps):
    sp = _abi.default_sim_params(max_contacts=cap)
    r, d = root.copy(), dof.copy()
    cache = O.new_cache(r.shape[0])
    gaps, coms, dropped, slots = [], [], [], []
    for t in range(steps):
        out = O.physics_step(hm, sp, r, d, targets, 2, cache=cache)
        gaps.append(cases.ground_gaps(model, out["rb_state"]).min(1))
        coms.append(cases.center_of_mass(model, out["rb_state"]))
        dropped.append(out["dropped"].copy())
        slots.append(out["num_contacts"].copy())
    return np.array(gaps), np.array(coms), np.array(dropped), np.array(slots)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=128)
    ap.add_argument("--steps", type=int, default=60)
    args = ap.parse_args()
    model = load_default_model()
    hm = _abi.make_model(model)
    off, _ = pd_action_offset_scale(model)
    res = {}
    for name, on_floor in (("lying_on_floor", True), ("lying_tumbling", False)):
        rng = np.random.default_rng(11)
        root, dof = cases.lying_state(args.envs, rng, on_floor=on_floor, model=model)
        targets = np.broadcast_to(off, (args.envs, 69)).astype(np.float32).copy()
        g40, c40, d40, s40 = run(hm, model, root, dof, targets, _abi.MAX_CONTACTS, args.steps)
        g64, c64, d64, s64 = run(hm, model, root, dof, targets, 64, args.steps)
        com_diff = np.linalg.norm(c40 - c64, axis=-1)
        res[name] = {
            "envs": args.envs, "steps": args.steps,
            "cap40": {"envs_dropping_any_step": int((d40 > 0).any(0).sum()), "dropped_mean": float(d40.mean()),
                      "dropped_max": int(d40.max()), "slots_mean": float(s40.mean()),
                      "min_gap_m": float(g40.min()), "min_gap_p01_m": float(np.percentile(g40.min(0), 1))},
            "cap64": {"dropped_max": int(d64.max()), "slots_mean": float(s64.mean()), "slots_max": int(s64.max()),
                      "min_gap_m": float(g64.min()), "min_gap_p01_m": float(np.percentile(g64.min(0), 1))},
            "com_diff_m": {"mean_final": float(com_diff[-1].mean()), "p90_final": float(np.percentile(com_diff[-1], 90)),
                           "max_final": float(com_diff[-1].max())},
        }
    res["definition"] = ("oracle (fp64) lying_state seed 11, PD targets at the action offset (actions 0), 2 substeps; "
                         "cap40 = the engine's capacity (40 slots, 63 rows) with the deepest-first reduction, cap64 = "
                         "the oracle's own capacity (64 slots, no row budget; its warm start covers the first 63 rows "
                         "the cache holds); min_gap over every body's contact candidates and steps")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
