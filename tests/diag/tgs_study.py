"""How close are the engine's physics steps to PhysX's TGS?

The reference runs PhysX TGS with 4 position iterations and 0 velocity iterations
(isaacgym_env.py:16-18). Round 5 built it in-step (he_sim_params.solver_type 1, oracle substep_tgs,
physics_kernel_tgs; the default since): each 1/120 s physics step keeps its factor and contact set and
runs 4 position iterations of 1/480 s -- the drives implicit per iteration, one Gauss-Seidel sweep
against separations advanced by the iterations' motion, the positions integrated per iteration.

Every scheme is the fp64 oracle (oracle/he_oracle_physics.c), from the same start state, fed the same
PD targets, for 30 policy steps (2 simulate() calls each):
  tgs           the engine default: 2 substeps of 1/120 s, TGS in-step, 4 position iterations
  pgs           rounds 1-4's default: 2 substeps of 1/120 s, velocity-level PGS, 8 sweeps, midpoint bias
  tgs_fixed     TGS in-step with the drive implicit over the whole 1/120 s step (one factor, the
                iterations only re-solve the contacts; solver_type 2, study only): what sub-stepping the
                drives contributes
  tgs_4x1       TGS's small-step form: 8 substeps of 1/480 s per simulate, one PGS sweep each, contacts,
                mass matrix and drives regenerated per sub-step (PhysX TGS keeps the step's contacts)
  pgs_4         2 substeps of 1/120 s, 4 PGS sweeps (PhysX's iteration count at the engine's step)
  fine_8        8 substeps of 1/480 s, 8 PGS sweeps: a converged small-step reference
  floor         the default from the start state with joint angles moved by 1e-6 rad: the chaos floor
Distances per env over the 30 steps: max joint-angle L2 (69 exp-map coordinates) and max CoM
distance; median / p90 / max over envs, and at step 1, 5, 10, 30; each against `tgs` (the default),
`tgs_4x1` and `fine_8`.
Cases (48 envs each): standing (PD stand-still, actions 0), tumbling (lying bodies thrown out of the
plane, actions 0), tracking (configs[2]-style: synthetic clips, a = clip(ref_dof_pos / scale)).

  python tests/diag/tgs_study.py > profiles/r05/tgs_study.json
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, ".."))

import cases  # noqa: E402
from humanoid_amd import _abi  # noqa: E402
from humanoid_amd.model import load_default_model, pd_action_offset_scale  # noqa: E402
from humanoid_amd.synthetic import make_clip  # noqa: E402
from oracle import oracle as O  # noqa: E402

SCHEMES = {"tgs": dict(solver_type=1, solver_iterations=4),
           "pgs": dict(solver_type=0, solver_iterations=8),
           "tgs_fixed": dict(solver_type=2, solver_iterations=4),
           "tgs_4x1": dict(solver_type=0, substeps=8, solver_iterations=1),
           "pgs_4": dict(solver_type=0, solver_iterations=4),
           "fine_8": dict(solver_type=0, substeps=8, solver_iterations=8)}
REFS = ("tgs", "tgs_4x1", "fine_8")
STEPS = 30
MARKS = (1, 5, 10, 30)


def run(hm, model, root, dof, targets, scheme, perturb=0.0):
    sp = _abi.default_sim_params(**scheme)
    r, d = root.copy(), dof.copy()
    if perturb:
        d[..., 0] += np.float32(perturb)
    cache = O.new_cache(r.shape[0])
    q, com = [], []
    for t in range(STEPS):
        out = O.physics_step(hm, sp, r, d, targets(t), 2, cache=cache)
        q.append(d[..., 0].astype(np.float64).copy())
        com.append(cases.center_of_mass(model, out["rb_state"]))
    return np.stack(q), np.stack(com)


def distances(a, b):
    dq = np.linalg.norm(a[0] - b[0], axis=-1)          # [steps, envs]
    dc = np.linalg.norm(a[1] - b[1], axis=-1)
    mq, mc = dq.max(0), dc.max(0)
    pct = lambda x: {"median": float(np.median(x)), "p90": float(np.percentile(x, 90)), "max": float(x.max())}  # noqa: E731
    return {"joint_l2_max_over_steps_rad": pct(mq), "com_max_over_steps_m": pct(mc),
            "joint_l2_median_at_step": {str(s): float(np.median(dq[s - 1])) for s in MARKS},
            "com_median_at_step_m": {str(s): float(np.median(dc[s - 1])) for s in MARKS},
            "envs_within_1e-4_over_30_steps": int(((mq <= 1e-4) & (mc <= 1e-4)).sum())}


def tracking_case(model, n, rng):
    off, sc = pd_action_offset_scale(model)
    off, sc = np.asarray(off, np.float32), np.asarray(sc, np.float32)
    clips = [make_clip(model, rng, num_frames=STEPS + 2) for _ in range(n)]
    root = np.zeros((n, 13), np.float32)
    dof = np.zeros((n, 69, 2), np.float32)
    from scipy.spatial.transform import Rotation as sRot
    for e, c in enumerate(clips):
        root[e, :3] = c["root_trans_offset"][0]
        root[e, 2] += 0.01
        root[e, 3:7] = sRot.from_rotvec(c["pose_aa"][0, :3]).as_quat()
        dof[e, :, 0] = c["pose_aa"][0, 3:]
    ref = np.stack([c["pose_aa"][:, 3:] for c in clips], 1)  # [T, n, 69]
    tg = [(off + sc * np.clip(ref[t + 1] / sc, -1.0, 1.0)).astype(np.float32) for t in range(STEPS)]
    return root, dof, lambda t: tg[t]


def main():
    model = load_default_model()
    hm = _abi.make_model(model)
    n = int(os.environ.get("TGS_ENVS", 48))
    zero = np.zeros((n, 69), np.float32)
    off, _ = pd_action_offset_scale(model)
    rest = np.broadcast_to(np.asarray(off, np.float32), (n, 69)).copy() if np.any(off) else zero
    rng = np.random.default_rng(31)
    standing = cases.standing_state(model, n, rng, xy_jitter=1.0)
    lying = cases.lying_state(n, np.random.default_rng(32))
    res = {}
    for name, (root, dof, tg) in {"standing": (*standing, lambda t: rest),
                                  "tumbling": (*lying, lambda t: rest),
                                  "tracking": tracking_case(model, n, np.random.default_rng(33))}.items():
        runs = {k: run(hm, model, root, dof, tg, sch) for k, sch in SCHEMES.items()}
        runs["floor"] = run(hm, model, root, dof, tg, SCHEMES["tgs"], 1e-6)
        case = {}
        for ref in REFS:
            case[f"vs_{ref}"] = {k: distances(v, runs[ref]) for k, v in runs.items() if k != ref}
        res[name] = case
        print(name, {ref: {k: round(v["com_max_over_steps_m"]["median"], 6) for k, v in case[f"vs_{ref}"].items()}
                     for ref in REFS}, file=sys.stderr, flush=True)
    res["definition"] = __doc__.split("\n\n")[3].strip()
    res["schemes"] = SCHEMES
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
