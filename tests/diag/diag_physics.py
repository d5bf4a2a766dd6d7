"""Diagnostic: GPU physics vs the fp64 oracle on the parity-test cases, printing error percentiles
per quantity (used when tuning tolerances; not part of the product path)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import cases
    from humanoid_amd import _abi
    from humanoid_amd.engine import Engine
    from humanoid_amd.model import load_default_model
    from oracle import oracle as O
    if os.environ.get("HE_LIB"):  # compare another build of the engine library
        from humanoid_amd import engine
        engine.load_library(os.environ["HE_LIB"])
    model = load_default_model()
    he_model = _abi.make_model(model)
    rng = np.random.default_rng(3)
    root, dof = cases.random_state(96, rng, height=(0.85, 1.0), ang=0.8, vel=0.5)
    r2, d2 = cases.lying_state(32, rng)
    root = np.concatenate([root, r2])
    dof = np.concatenate([dof, d2])
    n = root.shape[0]
    targets = rng.uniform(-0.5, 0.5, (n, 69)).astype(np.float32)
    sp = _abi.default_sim_params()
    eng = Engine(he_model, n, device=0, sim_params=sp)
    eng.root_states.copy_(torch.from_numpy(root).cuda())
    eng.dof_state.copy_(torch.from_numpy(dof.reshape(n * 69, 2)).cuda())
    eng.dof_targets.copy_(torch.from_numpy(targets).cuda())
    eng.simulate(2)
    r_o, d_o = root.copy(), dof.copy()
    out = O.physics_step(eng.he_model, sp, r_o, d_o, targets, 2)
    torch.cuda.synchronize()
    rg = eng.root_states.cpu().numpy()
    dg = eng.dof_state.view(n, 69, 2).cpu().numpy()
    nc_g = eng.num_contacts.cpu().numpy()
    print("contacts gpu/oracle mismatch:", int((nc_g != out["num_contacts"]).sum()), "mean nc", nc_g.mean())
    q = np.minimum(np.abs(rg[:, 3:7] - r_o[:, 3:7]).max(-1), np.abs(rg[:, 3:7] + r_o[:, 3:7]).max(-1))
    rows = {"root_pos": np.abs(rg[:, :3] - r_o[:, :3]).max(-1), "root_quat": q,
            "dof_pos": np.abs(dg[:, :, 0] - d_o[:, :, 0]).max(-1), "root_vel": np.abs(rg[:, 7:] - r_o[:, 7:]).max(-1),
            "dof_vel": np.abs(dg[:, :, 1] - d_o[:, :, 1]).max(-1)}
    for k, v in rows.items():
        print(f"{k:10s} p50 {np.percentile(v, 50):.2e} p90 {np.percentile(v, 90):.2e} max {v.max():.2e} "
              f"argmax {int(v.argmax())} (nc {int(nc_g[v.argmax()])})")


if __name__ == "__main__":
    main()
