"""PGS sweep count under motion ("warm start plus fewer iterations"): along one
trajectory (warm-started, 8 sweeps), every step is also re-solved from the same state and cache
with other settings, and each one-step result is compared with a converged solve (warm, 64 sweeps)
from that same state: the residual after the sweeps and the one-step deviation of the joint
velocities / positions. Scenarios: standing bodies under random actions (U(-0.5, 0.5) of the PD
scale, new each step) and lying bodies thrown out of the plane (cases.lying_state, tumbling).

  python tests/diag/pgs_iterations.py > profiles/r02/pgs_iterations.json
"""
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

SETTINGS = {"cold_8": (8, False), "warm_2": (2, True), "warm_4": (4, True), "warm_6": (6, True),
            "warm_8": (8, True), "warm_16": (16, True), "warm_8_tol1e-5": (8, True, 1e-5),
            "warm_8_tol1e-4": (8, True, 1e-4), "warm_16_tol1e-5": (16, True, 1e-5)}


def one_step(hm, r, d, c, targets, iters, warm, tol=0.0):
    sp = _abi.default_sim_params(solver_iterations=iters, warm_start=1 if warm else 0, solver_tolerance=tol)
    r, d = r.copy(), d.copy()
    cache = c.copy() if warm else None
    out = O.physics_step(hm, sp, r, d, targets, 2, cache=cache)
    return r, d, out["residual"]


def scenario(hm, root, dof, target_fn, steps):
    n = root.shape[0]
    r, d, c = root.copy(), dof.copy(), O.new_cache(n)
    res = {k: [] for k in SETTINGS}
    dv = {k: [] for k in SETTINGS}
    dq = {k: [] for k in SETTINGS}
    sp8 = _abi.default_sim_params()  # the trajectory: the engine default
    for t in range(steps):
        tg = target_fn(t)
        rr, dr, _ = one_step(hm, r, d, c, tg, 64, True)
        for k, st in SETTINGS.items():
            rs, ds, rsd = one_step(hm, r, d, c, tg, *st)
            res[k].append(rsd)
            dv[k].append(np.abs(ds[..., 1] - dr[..., 1]).max(1))
            dq[k].append(np.abs(ds[..., 0] - dr[..., 0]).max(1))
        O.physics_step(hm, sp8, r, d, tg, 2, cache=c)  # the trajectory: the default solve
    out = {}
    for k in SETTINGS:
        a, v, q = np.concatenate(res[k]), np.concatenate(dv[k]), np.concatenate(dq[k])
        out[k] = {"residual_median": float(np.median(a)), "residual_p99": float(np.percentile(a, 99)),
                  "dof_vel_dev_median": float(np.median(v)), "dof_vel_dev_p99": float(np.percentile(v, 99)),
                  "dof_pos_dev_median": float(np.median(q)), "dof_pos_dev_p99": float(np.percentile(q, 99))}
    return out


def main():
    model = load_default_model()
    hm = _abi.make_model(model)
    off, sc = pd_action_offset_scale(model)
    n, steps = 64, 40
    rng = np.random.default_rng(21)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=1.0)
    acts = [rng.uniform(-0.5, 0.5, (n, 69)).astype(np.float32) for _ in range(steps)]
    res = {"standing_random_actions": scenario(hm, root, dof, lambda t: (off + sc * acts[t]).astype(np.float32), steps)}
    root, dof = cases.lying_state(n, np.random.default_rng(22))
    zero = np.zeros((n, 69), np.float32)
    res["lying_tumbling"] = scenario(hm, root, dof, lambda t: zero, steps)
    res["definition"] = ("64 envs x 40 steps per scenario (oracle, fp64); each step re-solved from the trajectory's "
                         "state and warm-start cache with each setting; residual = max |w| violation after the sweeps "
                         "(m/s); deviations = max over dofs of |x - x_converged| after the step, x_converged = warm "
                         "start + 64 sweeps from the same state; median / p99 over envs x steps")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
