"""TGS on the oracle (he_sim_params.solver_type = 1; oracle/he_oracle_physics.c substep_tgs).

The reference configures PhysX's TGS solver with 4 position iterations and 0 velocity iterations
(puffer_phc/envs/isaacgym_env.py:16-18). PhysX is closed and absent, so, as for the PGS step
(tests/test_physics_invariants.py), the restatement is pinned by physics and by its own limits:
* one iteration is the one-sweep PGS step exactly (same drive, bias, sweep and integration);
* free fall from rest: K position iterations of h = dt / K, each a semi-implicit sub-step, give the
  discrete parabola of the sub-steps;
* free flight: momentum / energy drift at first order, well under the explicit-bias PGS step's;
* the actuated runaway regime stays at the dt-refined level (TGS's purpose: the sub-steps' drives);
* PD stand-still settles and stands still; settled bodies rest within the Baumgarte steady state;
* the step is closer to the small-step form of TGS (8 x 1/480 s, one sweep: PhysX's "each position
  iteration re-integrates" with fresh contacts) than the PGS step is, on a standing body.
"""
import numpy as np
import pytest

from humanoid_amd import _abi
from oracle import oracle as O

import cases
from test_physics_invariants import G, _drives_off, _random_action_run, _run

TGS = dict(solver_type=1, solver_iterations=4)


@pytest.mark.parametrize("kind", ["standing", "random", "lying"])
def test_tgs_one_iteration_is_the_one_sweep_pgs_step(he_model, model, kind):
    """K = 1: the drive implicit over dt, one sweep against the gaps over dt, one integration: the
    PGS step with one sweep and the bias at u0 (bias_midpoint 0), to the bit."""
    rng = np.random.default_rng(1)
    st = {"standing": lambda: cases.standing_state(model, 16, rng),
          "random": lambda: cases.random_state(16, rng),
          "lying": lambda: cases.lying_state(16, rng, on_floor=True, model=model)}[kind]()
    tg = np.random.default_rng(5).uniform(-1, 1, (16, 69)).astype(np.float32)
    res = []
    for kw in (dict(solver_type=1, solver_iterations=1, bias_midpoint=0),
               dict(solver_type=0, solver_iterations=1, bias_midpoint=0)):
        r, d = st[0].copy(), st[1].copy()
        cache = O.new_cache(16)
        for _ in range(5):
            out = O.physics_step(he_model, _abi.default_sim_params(**kw), r, d, tg, 2, cache=cache)
        res.append((r, d, out["dof_force"], out["contact_forces"], cache))
    for a, b in zip(*res):
        np.testing.assert_array_equal(a, b)


def test_tgs_free_fall_is_the_substeps_parabola(he_model):
    """Drives off, zero velocities: iteration k of every physics step adds -g h to the velocity and
    moves the body by h times it, so after n physics steps of K iterations (N = n K sub-steps of h)
    z = z0 - g h^2 N (N + 1) / 2 exactly, as the PGS step's parabola at h."""
    rng = np.random.default_rng(0)
    root, dof = cases.random_state(8, rng, height=(3.5, 4.5), vel=0.0)
    dof[..., 1] = 0.0
    calls = 20
    r, d, out, sp = _run(he_model, root, dof, np.zeros((8, 69), np.float32), calls, **_drives_off(**TGS))
    assert (out["num_contacts"] == 0).all()
    h = sp.dt / sp.substeps / sp.solver_iterations
    N = calls * 2 * sp.substeps * sp.solver_iterations  # 2 simulate() per call, substeps physics steps each
    np.testing.assert_allclose(r[:, 2], root[:, 2] - G * h * h * N * (N + 1) / 2, atol=2e-5)
    np.testing.assert_allclose(r[:, 9], -G * h * N, atol=2e-5)
    np.testing.assert_allclose(r[:, :2], root[:, :2], atol=1e-6)
    np.testing.assert_allclose(d[..., 0], dof[..., 0], atol=1e-6)


def test_tgs_free_flight_drift_first_order(he_model, model):
    """Drives off, no gravity, no contact, 1 s: linear momentum, angular momentum about the CoM and the
    kinetic energy drift at first order in the physics step (the ratio between dt and dt/2 ~ 0.5). The
    velocity-dependent bias is explicit per iteration (h = dt / 4), so the rotational drift lies between
    the PGS step's two forms: well under the explicit bias at dt (measured 1.2 % of |L_com| against
    2.6 %), above the midpoint bias (0.26 %), which conserves the quadratic invariants of a free body."""
    from test_physics_invariants import _flight_drifts
    import test_physics_invariants as T
    rng = np.random.default_rng(1)
    root, dof = cases.random_state(8, rng, height=(3.0, 4.0), vel=0.5, ang=0.5)
    orig = T._drives_off
    try:
        T._drives_off = lambda **kw: dict(orig(**kw), bias_midpoint=0)
        explicit = _flight_drifts(model, he_model, root, dof, (0.0, 0.0, 0.0), 1)
        T._drives_off = lambda **kw: dict(orig(**kw), **TGS)
        res = {k: _flight_drifts(model, he_model, root, dof, (0.0, 0.0, 0.0), k) for k in (1, 2)}
    finally:
        T._drives_off = orig
    dP1, dL1, dE1, P, L = res[1]
    dP2, dL2, dE2, _, _ = res[2]
    assert dP1 < 0.015 * P and dL1 < 0.6 * explicit[1] and dE1 < 0.6 * explicit[2], (res[1], explicit)
    for a, b in ((dP1, dP2), (dL1, dL2), (dE1, dE2)):
        assert 0.35 < b / a < 0.65, (a, b)


def test_tgs_tames_the_runaway(he_model, model):
    """DESIGN §5's runaway regime (airborne bodies, U(+-1) PD targets renewed every step, 3 s): the
    internal kinetic energy stays at the dt-refined level (substeps 8, the PGS step at 1/480 s), and
    with the velocity-dependent bias frozen at the step's start (bias_midpoint 0) it is several times
    higher: the per-iteration re-evaluation is what keeps it there."""
    n = 48
    _, ke, _ = _random_action_run(he_model, model, 1.0, n, 90, airborne=True, **TGS)
    _, ke_frozen, _ = _random_action_run(he_model, model, 1.0, n, 90, airborne=True, bias_midpoint=0, **TGS)
    _, ke_ref, _ = _random_action_run(he_model, model, 1.0, n, 90, airborne=True, substeps=8, solver_type=0,
                                      solver_iterations=8)
    med = {k: float(np.median(v)) for k, v in (("tgs", ke), ("frozen", ke_frozen), ("refined", ke_ref))}
    assert med["tgs"] < 1.2e3 and abs(med["tgs"] / med["refined"] - 1.0) < 0.25, med
    assert med["frozen"] > 2.5 * med["tgs"], med


def test_tgs_saturated_random_actions_stay_physical(he_model, model):
    """Standing bodies, U(+-1) actions renewed every policy step for 2 s: median internal kinetic energy
    at the refined level, at most 1 of 128 roots over 10 m/s and none over 15 (measured: one pelvis
    whipped to 11.7 m/s by flailing legs while airborne, no contact rows, the CoM far slower; the PGS
    step's study found the same mechanism), no joint past its angle cap."""
    n = 128
    vmax, ke, dof = _random_action_run(he_model, model, 1.0, n, 60, **TGS)
    q = np.linalg.norm(dof[..., 0].reshape(n, 23, 3), axis=-1)
    assert (vmax > 10.0).sum() <= 1 and vmax.max() < 15.0, np.sort(vmax)[-3:]
    assert np.median(ke) < 1.2e3, np.median(ke)
    assert q.max() <= np.pi - 0.01 + 1e-5


def test_tgs_pd_stand_still(he_model, model):
    """configs[1] under TGS: the zero-pose PD humanoid settles, then stands still (< 0.2 mm over 5 s,
    velocities < 1e-4), the 16 foot / toe box corners in contact throughout."""
    rng = np.random.default_rng(4)
    n = 8
    root, dof = cases.standing_state(model, n, rng, xy_jitter=1.0)
    targets = np.zeros((n, 69), np.float32)
    sp = _abi.default_sim_params(**TGS)
    r, d = root.copy(), dof.copy()
    cache = O.new_cache(n)
    ncs = []
    for _ in range(300):
        out = O.physics_step(he_model, sp, r, d, targets, 2, cache=cache)
        ncs.append(out["num_contacts"].copy())
    r1 = r.copy()
    for _ in range(150):
        out = O.physics_step(he_model, sp, r, d, targets, 2, cache=cache)
        ncs.append(out["num_contacts"].copy())
    assert np.abs(r[:, :2] - root[:, :2]).max() < 0.05 and np.abs(r[:, 2] - root[:, 2]).max() < 5e-3
    assert np.abs(r[:, :3] - r1[:, :3]).max() < 2e-4
    assert np.abs(r[:, 7:]).max() < 1e-4 and np.abs(d[..., 1]).max() < 1e-4
    assert (np.array(ncs) == 16).all()


def test_tgs_penetration_within_contact_offset(he_model, model):
    """Standing and lying bodies settle with every terrain candidate above -2 mm under TGS (its
    per-iteration Baumgarte pushes out at baumgarte * gap / h)."""
    rng = np.random.default_rng(5)
    targets = np.zeros((8, 69), np.float32)
    for root, dof in (cases.standing_state(model, 8, rng, xy_jitter=1.0), cases.lying_state(8, rng)):
        r, d, out, sp = _run(he_model, root, dof, targets, 120, **TGS)
        gaps = cases.ground_gaps(model, out["rb_state"])
        assert gaps.min() > -2e-3, gaps.min()
        assert gaps.min() < sp.contact_offset


def test_tgs_is_closer_than_pgs_to_the_small_step_form(he_model, model):
    """A standing body over 30 policy steps: the CoM trajectory of the TGS step against TGS's small-step
    form (8 physics steps of 1/480 s per simulate, one sweep each, contacts and factor fresh per
    sub-step) is about 3x closer than the PGS step's (measured: 2.0e-4 against 5.9e-4 m median,
    tests/diag/tgs_study.py)."""
    n = 16
    root, dof = cases.standing_state(model, n, np.random.default_rng(31), xy_jitter=1.0)
    tg = np.zeros((n, 69), np.float32)

    def com_traj(**kw):
        sp = _abi.default_sim_params(**kw)
        r, d = root.copy(), dof.copy()
        cache = O.new_cache(n)
        out = []
        for _ in range(30):
            o = O.physics_step(he_model, sp, r, d, tg, 2, cache=cache)
            out.append(cases.center_of_mass(model, o["rb_state"]))
        return np.stack(out)
    small = com_traj(substeps=8, solver_iterations=1, solver_type=0)
    e_tgs = np.median(np.linalg.norm(com_traj(**TGS) - small, axis=-1).max(0))
    e_pgs = np.median(np.linalg.norm(com_traj(solver_type=0, solver_iterations=8) - small, axis=-1).max(0))
    assert e_tgs < 0.5 * e_pgs, (e_tgs, e_pgs)


def test_tgs_replays_the_runaway_trace_without_the_launch(he_model):
    """Round 4's fastest root (tests/data/trace_runaway_0.75.npz: env 3261 of the U(+-0.75) study,
    engine state, warm-start cache and PD targets from 6 policy steps before its 17.4 m/s peak; DESIGN
    §5 "the runaway tail"), replayed one physics step (1/120 s) at a time from the first recorded
    state, every row's gap at the step's start recorded (oracle row-gap diagnostic):
    * under the PGS step the right forearm and hand wedge into the thigh (self rows 8.5 cm deep) and
      the root is launched past 15 m/s;
    * under TGS no self contact gets deeper than 3 cm (measured 2.4 cm: the 2 cm contact offset plus
      one step's approach) and the root stays under 5 m/s (measured max 3.2 m/s), as under the PGS
      step at dt/4."""
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), "data", "trace_runaway_0.75.npz"))
    out = {}
    for name, sp in (("tgs", _abi.default_sim_params(dt=1.0 / 120.0, substeps=1, **TGS)),
                     ("pgs", _abi.pgs_sim_params(dt=1.0 / 120.0, substeps=1))):
        r, dd = d["root"][0][None].copy(), d["dof"][0][None].copy()
        c = d["cache"][0][None].copy()
        vmax, self_gap = 0.0, 0.0
        for i in range(d["targets"].shape[0]):
            for _ in range(4):  # a policy step: 2 simulate() x 2 substeps
                gp = np.zeros((1, _abi.MAX_ROWS), np.float32)
                O.set_row_gap_out(gp)
                try:
                    O.physics_step(he_model, sp, r, dd, d["targets"][i][None].copy(), 1, cache=c)
                finally:
                    O.set_row_gap_out(None)
                n, keys, _ = _abi.cache_rows(c)
                for k in range(int(n[0])):
                    b0, b1, sub, kind = _abi.key_fields(keys[0, k])
                    if kind == 0 and b1 >= 0:  # a self pair's normal row
                        self_gap = min(self_gap, float(gp[0, k]))
                vmax = max(vmax, float(np.linalg.norm(r[0, 7:10])))
        out[name] = (vmax, self_gap)
    assert out["pgs"][0] > 15.0 and out["pgs"][1] < -0.05, out
    assert out["tgs"][0] < 5.0 and out["tgs"][1] > -0.03, out
