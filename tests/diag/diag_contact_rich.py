"""Diagnostics: per-env error of the engine against the fp64 oracle on the contact-rich parity case
(tests/test_gpu_parity.py::test_physics_contact_rich_matches_oracle), next to the oracle's own
sensitivity (1e-6 rad probe). HE_ENGINE_LIB selects a variant build. GPU."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import cases  # noqa: E402
from humanoid_amd import _abi  # noqa: E402
from humanoid_amd.engine import Engine  # noqa: E402
from humanoid_amd.model import load_default_model  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    model = load_default_model()
    hm = _abi.make_model(model)
    rng = np.random.default_rng(3)
    root, dof = cases.random_state(96, rng, height=(0.85, 1.0), ang=0.8, vel=0.5)
    r2, d2 = cases.lying_state(32, rng)
    root = np.concatenate([root, r2])
    dof = np.concatenate([dof, d2])
    targets = rng.uniform(-0.5, 0.5, (128, 69)).astype(np.float32)
    if os.environ.get("DIAG_AIRBORNE"):
        root[:, 2] += 3.0
    n = 128
    eng = Engine(hm, n, device=0, sim_params=_abi.default_sim_params())
    eng.root_states.copy_(torch.as_tensor(root, device="cuda:0"))
    eng.dof_state.copy_(torch.as_tensor(dof.reshape(n * 69, 2), device="cuda:0"))
    eng.dof_targets.copy_(torch.as_tensor(targets, device="cuda:0"))
    r_o, d_o = root.copy(), dof.copy()
    r_s, d_s = root.copy(), dof.copy()
    d_s[:, :, 0] += (1e-6 * np.random.default_rng(123).standard_normal(d_s[:, :, 0].shape)).astype(np.float32)
    sp = _abi.default_sim_params()
    eng.simulate(2)
    out = O.physics_step(hm, sp, r_o, d_o, targets, 2)
    O.physics_step(hm, sp, r_s, d_s, targets, 2)
    torch.cuda.synchronize()
    ok = eng.num_contacts.cpu().numpy() == out["num_contacts"]
    dg = eng.dof_state.view(n, 69, 2).cpu().numpy()[:, :, 0]
    err = np.abs(dg - d_o[:, :, 0]).max(-1)
    sens = np.abs(d_s[:, :, 0] - d_o[:, :, 0]).max(-1)
    excess = err - (1e-4 + 4 * sens)
    order = np.argsort(-excess)[:6]
    if len(sys.argv) > 1:
        np.save(sys.argv[1], np.concatenate([dg, eng.root_states.cpu().numpy()], -1))
    for i in order:
        print(f"env {i:3d} ok={ok[i]} nc={out['num_contacts'][i]:2d} err={err[i]:.3e} sens={sens[i]:.3e} excess={excess[i]:.3e}")


if __name__ == "__main__":
    main()
