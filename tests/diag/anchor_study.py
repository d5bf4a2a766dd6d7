"""Patch friction: the engine's centroid pair + torsional row against PhysX-style two friction
anchors per patch (VERDICT r03 weak 1 / missing 4: the documented difference, quantified).

The engine (and the oracle) give a body-ground patch of >= 2 points 2 tangential rows at the points'
centroid plus 1 torsional row about the patch normal, bounded by mu and mu r_patch times the
patch's normal impulses. PhysX's patch friction places friction at up to two anchor
points of the patch instead. The oracle's diagnostic mode (`ho_set_two_anchor`) builds that form:
2 tangential rows at the patch's first point and 2 at the point farthest from it in the tangent
plane, each bounded by mu / 2 x the patch's normal impulses (the anchors share the load; PhysX's
exact split is not published). Everything else is the shipped scheme.

Distances between the two forms over 30 policy steps from the same start state and PD targets (fp64
oracle, 48 envs per case), as in tests/diag/tgs_study.py, with the chaos floor (shipped, joint angles
+1e-6 rad) beside them; plus the sliding deceleration of tests/test_physics_invariants.py under both
forms.

  python tests/diag/anchor_study.py > profiles/r04/anchor_study.json
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, HERE)

import cases  # noqa: E402
from humanoid_amd import _abi  # noqa: E402
from humanoid_amd.model import load_default_model, pd_action_offset_scale  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tgs_study import SCHEMES, distances, run, tracking_case  # noqa: E402


def anchored(fn, on):
    O.set_two_anchor(on)
    try:
        return fn()
    finally:
        O.set_two_anchor(False)


def sliding(hm, model, mu, two):
    """A lying body, settled, then given 3 m/s along x; fitted deceleration while it slides (median of
    8 envs), as test_sliding_body_decelerates_at_mu_g."""
    rng = np.random.default_rng(3)
    n = 8
    root, dof = cases.lying_state(n, rng, on_floor=True, model=model)
    sp = _abi.default_sim_params(friction=mu)
    tg = np.zeros((n, 69), np.float32)

    def go():
        cache = O.new_cache(n)
        r, d = root.copy(), dof.copy()
        for _ in range(30):
            O.physics_step(hm, sp, r, d, tg, 2, cache=cache)
        r[:, 7] += 3.0
        rb = O.forward_kinematics(hm, r, d)
        v = []
        for _ in range(12):
            out = O.physics_step(hm, sp, r, d, tg, 2, cache=cache)
            v.append(cases.com_velocity(model, out["rb_state"])[:, 0])
        v = np.stack(v)
        t = np.arange(len(v)) / 30.0
        dec = []
        for e in range(n):
            ok = v[:, e] > 0.5
            dec.append(-np.polyfit(t[ok], v[ok, e], 1)[0] if ok.sum() >= 3 else np.nan)
        return float(np.nanmedian(dec)), rb
    return anchored(go, two)[0]


def main():
    model = load_default_model()
    hm = _abi.make_model(model)
    n = int(os.environ.get("ANCHOR_ENVS", 48))
    off, _ = pd_action_offset_scale(model)
    rest = np.broadcast_to(np.asarray(off, np.float32), (n, 69)).copy()
    rng = np.random.default_rng(31)
    standing = cases.standing_state(model, n, rng, xy_jitter=1.0)
    lying = cases.lying_state(n, np.random.default_rng(32))
    resting = cases.lying_state(n, np.random.default_rng(34), on_floor=True, model=model)
    res = {}
    for name, (root, dof, tg) in {"standing": (*standing, lambda t: rest),
                                  "lying at rest": (*resting, lambda t: rest),
                                  "tumbling": (*lying, lambda t: rest),
                                  "tracking": tracking_case(model, n, np.random.default_rng(33))}.items():
        sh = SCHEMES["shipped"]
        base = run(hm, model, root, dof, tg, sh)
        res[name] = {"chaos_floor (shipped+1e-6 rad)": distances(run(hm, model, root, dof, tg, sh, 1e-6), base),
                     "two_anchor vs centroid+torsion": distances(anchored(lambda: run(hm, model, root, dof, tg, sh), True),
                                                                 base)}
        print(name, {k: round(v["joint_l2_max_over_steps_rad"]["median"], 6) for k, v in res[name].items()},
              file=sys.stderr, flush=True)
    res["sliding_deceleration_m_s2"] = {
        f"mu={mu}": {"centroid+torsion": sliding(hm, model, mu, False), "two_anchor": sliding(hm, model, mu, True),
                     "mu_g": mu * 9.81} for mu in (0.25, 0.5)}
    res["definition"] = __doc__.split("\n\n")[1].strip() + " " + __doc__.split("\n\n")[2].strip()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
