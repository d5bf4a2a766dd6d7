"""Self-contact parity diagnostic: one physics step (substeps 1, one simulate) of the traj30 case's
envs from the same state, engine vs oracle: per env the contact keys, the impulses of every row
(warm-start cache words) and the max joint-velocity difference.

  python tests/diag/diag_self.py
"""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import cases  # noqa: E402


def main():
    import torch
    from humanoid_amd import _abi
    from humanoid_amd.engine import Engine
    from humanoid_amd.model import load_default_model
    from oracle import oracle as O
    model = load_default_model()
    hm = _abi.make_model(model)
    rng = np.random.default_rng(11)
    root, dof = cases.random_state(32, rng, height=(6.0, 7.0), ang=0.4, vel=0.5)
    targets = rng.uniform(-0.5, 0.5, (32, 69)).astype(np.float32)
    n = root.shape[0]
    for iters in (4, 0):
        sim = dict(substeps=1, solver_iterations=iters, warm_start=1)  # cold: the cache starts empty
        sp = _abi.default_sim_params(**sim)
        eng = Engine(hm, n, device=0, sim_params=_abi.default_sim_params(**sim))
        eng.root_states.copy_(torch.as_tensor(root, device="cuda:0"))
        eng.dof_state.copy_(torch.as_tensor(dof.reshape(n * 69, 2), device="cuda:0"))
        eng.dof_targets.copy_(torch.as_tensor(targets, device="cuda:0"))
        r_o, d_o = root.copy(), dof.copy()
        eng.simulate(1)
        c_o = O.new_cache(n)

        O.physics_step(hm, sp, r_o, d_o, targets, 1, cache=c_o)
        torch.cuda.synchronize()
        cg = eng.contact_cache.cpu().numpy()
        dg = eng.dof_state.view(n, 69, 2).cpu().numpy()
        print(f"== solver_iterations {iters}")
        for e in range(n):
            wg, wo = cg[e].view(np.int32), c_o[e].view(np.int32)
            dv = np.abs(dg[e, :, 1] - d_o[e, :, 1]).max()
            if wo[7] == 0 and dv < 1e-4:
                continue
            k = int(wo[7])
            print(f"env {e}: nc gpu {wg[7]} oracle {wo[7]} keys gpu {wg[8:8 + wg[7]].tolist()} oracle {wo[8:8 + k].tolist()} "
                  f"max |dv| {dv:.3e} at dof {int(np.abs(dg[e, :, 1] - d_o[e, :, 1]).argmax())}")
            print("   lam gpu   ", np.array2string(cg[e, 32:32 + 3 * k], precision=6))
            print("   lam oracle", np.array2string(c_o[e, 32:32 + 3 * k], precision=6))
        del eng


if __name__ == "__main__":
    main()
