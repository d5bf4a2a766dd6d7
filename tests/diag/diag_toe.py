"""Stand-still toe-yaw trace (diagnostic): env 0 of the 30-step stand-still parity case, per policy
step the GPU's and the oracle's L_Toe / R_Toe dof angles, the spread of 8 noise probes, and the
toe boxes' friction states (oracle cache)."""
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
    cases.random_state(32, rng, height=(6.0, 7.0), ang=0.4, vel=0.5)
    rng.uniform(-0.5, 0.5, (32, 69))
    root, dof = cases.standing_state(model, 32, rng, xy_jitter=1.0)
    n = 32
    targets = np.zeros((n, 69), np.float32)
    sp = _abi.default_sim_params()
    eng = Engine(hm, n, device=0, sim_params=sp)
    eng.root_states.copy_(torch.as_tensor(root, device="cuda:0"))
    eng.dof_state.copy_(torch.as_tensor(dof.reshape(n * 69, 2), device="cuda:0"))
    eng.dof_targets.zero_()
    r_o, d_o, c_o = root.copy(), dof.copy(), O.new_cache(n)
    probes = [[root.copy(), dof.copy(), O.new_cache(n)] for _ in range(8)]
    dofs = [9, 10, 11, 21, 22, 23]
    for step in range(30):
        eng.simulate(2)
        O.physics_step(hm, sp, r_o, d_o, targets, 2, cache=c_o)
        for k, pr in enumerate(probes):
            cases.rounding_noise(pr[0], pr[1], 123 + 1000 * k + step)
            O.physics_step(hm, sp, pr[0], pr[1], targets, 2, cache=pr[2])
        torch.cuda.synchronize()
        g = eng.dof_state.view(n, 69, 2).cpu().numpy()[0, dofs, 0]
        o = d_o[0, dofs, 0]
        ps = np.array([p[1][0, dofs, 0] for p in probes])
        cg = eng.contact_cache.cpu().numpy()[0]
        lam_g = cg[32:32 + 48].reshape(16, 3)
        lam_o = c_o[0, 32:32 + 48].reshape(16, 3)
        rg = np.abs(lam_g[:, 1:]).max(1) / np.maximum(lam_g[:, 0], 1e-12)
        ro = np.abs(lam_o[:, 1:]).max(1) / np.maximum(lam_o[:, 0], 1e-12)
        print(f"step {step:2d} gpu-oracle {np.array2string((g - o) * 1e6, precision=1)} e-6  probe spread "
              f"{np.array2string((ps.max(0) - ps.min(0)) * 1e6, precision=1)} e-6  sat gpu {int((rg > 0.999999).sum())} "
              f"oracle {int((ro > 0.999999).sum())}  max|lam diff| {np.abs(lam_g - lam_o).max():.2e}", flush=True)


if __name__ == "__main__":
    main()
