"""Contact-slot histograms on the GPU: how many contact slots envs use and how
many contacts the engine capacity (he_sim_params.max_contacts slots, 63 solver rows) drops, for lying bodies (cases.lying_state: limbs start inside the
plane, the overflow case) and for configs[4] (mass / friction randomisation + plane / 10 deg slope /
box steps, the divergent contact-set stress config). Writes JSON to stdout."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def hist(x, width=33):
    return np.bincount(np.asarray(x).ravel(), minlength=width)[:width].tolist()


def main():
    import torch
    import bench
    import cases
    from humanoid_amd import _abi
    from humanoid_amd.engine import Engine
    from humanoid_amd.model import load_default_model
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-envs", type=int, default=4096)
    a = ap.parse_args()
    model = load_default_model()
    out = {}
    n = a.num_envs
    rng = np.random.default_rng(0)
    root, dof = cases.lying_state(n, rng)
    eng = Engine(model, n, device=0, sim_params=_abi.default_sim_params())
    eng.root_states.copy_(torch.as_tensor(root, device="cuda:0"))
    eng.dof_state.copy_(torch.as_tensor(dof.reshape(n * 69, 2), device="cuda:0"))
    eng.dof_targets.zero_()
    lying = {}
    for step in range(1, 121):
        eng.simulate(2)
        if step in (1, 10, 30, 60, 120):
            nc = eng.num_contacts.cpu().numpy()
            dr = eng.dropped_contacts.cpu().numpy()
            lying[f"step{step}"] = {"slots_hist": hist(nc), "generated_hist": hist(nc + dr, 48),
                                    "envs_dropping": int((dr > 0).sum()), "dropped_mean": float(dr.mean()),
                                    "dropped_max": int(dr.max())}
    out["lying_state"] = lying
    args = bench.parse(["--config", "dr"])
    ro = bench.Rollout(args, model, 0, 0)
    dr_hist = {}
    for step in range(1, 101):
        ro.step()
        if step in (1, 50, 100):
            nc = ro.eng.num_contacts.cpu().numpy()
            dr = ro.eng.dropped_contacts.cpu().numpy()
            tk = np.arange(n) % 3
            dr_hist[f"step{step}"] = {
                kind: {"slots_hist": hist(nc[tk == k]), "envs_dropping": int((dr[tk == k] > 0).sum()),
                       "dropped_mean": float(dr[tk == k].mean())}
                for k, kind in enumerate(("plane", "slope10", "steps"))}
    out["configs4_dr"] = dr_hist
    out["capacity"] = {"slots": int(_abi.default_sim_params().max_contacts), "rows": int(_abi.MAX_ROWS)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
