"""Per-step growth of the engine-vs-oracle difference along a multi-step parity case (diagnostic):
for every policy step, per env, max |gpu - oracle| of the joint angles, the oracle's own spread
under fp32-level noise (3 probes, tests/cases.rounding_noise), and the step's contact count.

  python tests/diag/diag_traj.py [case]   (case: traj30 | cold)
"""
import json
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
    case = sys.argv[1] if len(sys.argv) > 1 else "traj30"
    extra = json.loads(sys.argv[2]) if len(sys.argv) > 2 else {}
    max_steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    model = load_default_model()
    hm = _abi.make_model(model)
    if case == "traj30":
        rng = np.random.default_rng(11)
        root, dof = cases.random_state(32, rng, height=(6.0, 7.0), ang=0.4, vel=0.5)
        targets = rng.uniform(-0.5, 0.5, (32, 69)).astype(np.float32)
        sim, steps = {}, 30
    elif case == "stand30":
        rng = np.random.default_rng(11)
        cases.random_state(32, rng, height=(6.0, 7.0), ang=0.4, vel=0.5)  # the test's draws before
        rng.uniform(-0.5, 0.5, (32, 69))
        root, dof = cases.standing_state(model, 32, rng, xy_jitter=1.0)
        targets = np.zeros((32, 69), np.float32)
        sim, steps = {}, 30
    else:
        rng = np.random.default_rng(14)
        root, dof = cases.standing_state(model, 48, rng, xy_jitter=1.0)
        targets = rng.uniform(-0.2, 0.2, (48, 69)).astype(np.float32)
        sim, steps = dict(warm_start=0, solver_iterations=4), 5
    sim.update(extra)
    steps = min(steps, max_steps)
    n = root.shape[0]
    sp = _abi.default_sim_params(**sim)
    eng = Engine(hm, n, device=0, sim_params=_abi.default_sim_params(**sim))
    eng.root_states.copy_(torch.as_tensor(root, device="cuda:0"))
    eng.dof_state.copy_(torch.as_tensor(dof.reshape(n * 69, 2), device="cuda:0"))
    eng.dof_targets.copy_(torch.as_tensor(targets, device="cuda:0"))
    r_o, d_o, c_o = root.copy(), dof.copy(), O.new_cache(n)
    probes = [[root.copy(), dof.copy(), O.new_cache(n)] for _ in range(3)]
    rows = []
    for step in range(steps):
        eng.simulate(2)
        out = O.physics_step(hm, sp, r_o, d_o, targets, 2, cache=c_o)
        for k, pr in enumerate(probes):
            cases.rounding_noise(pr[0], pr[1], 123 + 1000 * k + step)
            O.physics_step(hm, sp, pr[0], pr[1], targets, 2, cache=pr[2])
        torch.cuda.synchronize()
        dg = eng.dof_state.view(n, 69, 2).cpu().numpy()
        err = np.abs(dg[..., 0] - d_o[..., 0])
        sens = np.max([np.abs(p[1][..., 0] - d_o[..., 0]) for p in probes], axis=0)
        ratio = err / np.maximum(sens, 1e-12)
        worst = int(np.argmax(err.max(1)))
        j = int(np.argmax(err[worst]))
        rows.append({"step": step, "worst_env": worst, "dof": j, "err": float(err[worst, j]),
                     "sens": float(sens[worst, j]), "err_over_sens_max": float(ratio[err > 1e-6].max()) if (err > 1e-6).any() else 0.0,
                     "nc": int(out["num_contacts"][worst]), "gpu_nc": int(eng.num_contacts[worst].item()),
                     "speed": float(np.abs(d_o[worst, :, 1]).max())})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
