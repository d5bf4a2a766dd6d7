"""Joint limits, contact capacity and warm starting in the fp64 oracle (CPU).

* Joint limits: the MJCF ranges (+-180 deg, +-720 deg at shoulders / elbows, humanoid_phc.py:305-324)
  as unilateral rows on the exp-map coordinates. The knee-y PD scale is 5 rad (humanoid_phc.py:441-446),
  so a saturated action targets +-5 rad, past the +-pi range: without limits the knee is driven through
  pi, its exp-map coordinate wraps to -pi and the drive keeps spinning it; with limits it stops at pi.
* Capacity: the engine has HE_MAX_CONTACTS = 40 contact slots and HE_MAX_ROWS = 63 solver rows (one
  wave; patch friction: a normal row per slot, 3 rows per body-ground patch, 3 per self pair). Overflow
  is counted (`dropped`) and the row budget goes to the deepest contacts first, so a lying body's hand keeps its penetrating
  contact (round 1 truncated in body order: the right arm sank).
* Warm start: the solve starting from the previous impulses converges where the cold 8-iteration PGS
  does not (stand-still jitter, lying-body residual).
"""
import numpy as np

from humanoid_amd import _abi
from oracle import oracle as O

import cases

KNEE_Y = (4, 16)  # L_Knee / R_Knee y (humanoid_phc.py:441-446)


def _knee_run(he_model, model, sign, steps=45, **sim):
    rng = np.random.default_rng(7)
    n = 4
    root, dof = cases.standing_state(model, n, rng, xy_jitter=0.5)
    root[:, 2] += 1.5  # airborne: nothing but the drives and the limits act on the knees
    targets = np.zeros((n, 69), np.float32)
    targets[:, list(KNEE_Y)] = sign * 5.0  # offset 0 + scale 5 x action +-1
    sp = _abi.default_sim_params(self_collision=0, **sim)
    cache = O.new_cache(n)
    r, d = root.copy(), dof.copy()
    hist = []
    for _ in range(steps):
        O.physics_step(he_model, sp, r, d, targets, 2, cache=cache)
        hist.append(np.stack([d[:, k - 1:k + 2, 0] for k in KNEE_Y], axis=1))
    return np.array(hist)  # [steps, n, knee, xyz]


def test_knee_limit_holds_at_pi(he_model, model):
    """The knee's rotation stops at the limit: |q| <= pi (|q| <= pi + 1e-3; the engine
    holds the angle 0.02 rad inside the branch cut) and its y coordinate never wraps sign."""
    for sign in (1.0, -1.0):
        q = _knee_run(he_model, model, sign)
        ang = np.linalg.norm(q, axis=-1)
        assert ang.max() <= np.pi - 2e-3, ang.max()  # the 0.02 guard less the linearised row's overshoot (~0.01)
        assert (ang[-10:] > np.pi - 0.05).all()  # driven onto the limit and held there
        assert (sign * q[5:, :, :, 1] > 0).all()  # no wrap through pi


def test_knee_without_limits_wraps(he_model, model):
    """The failure the limits prevent: the +5 rad target drives the knee through pi; its exp-map
    coordinate wraps to ~ -pi (the error to the target grows to ~8 rad) and the knee spins."""
    q = _knee_run(he_model, model, 1.0, joint_limits=0)
    assert (q[..., 1] < -2.0).any()


def test_limit_rows_keep_every_dof_in_range(he_model, model):
    """Random saturating actions (targets = the PD scale x U(-1, 1) clipped, as in early training)
    on a standing humanoid: every dof stays within its range."""
    from humanoid_amd.model import pd_action_offset_scale
    rng = np.random.default_rng(8)
    n = 8
    off, sc = pd_action_offset_scale(model)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=0.5)
    sp = _abi.default_sim_params()
    cache = O.new_cache(n)
    lo = np.array([he_model.dof_lower[k] for k in range(69)], np.float32)
    hi = np.array([he_model.dof_upper[k] for k in range(69)], np.float32)
    for step in range(30):
        a = rng.uniform(-1.0, 1.0, (n, 69)).astype(np.float32)
        tgt = (off + sc * a).astype(np.float32)
        O.physics_step(he_model, sp, root, dof, tgt, 2, cache=cache)
        q = dof[..., 0]
        assert (q <= hi + 1e-3).all() and (q >= lo - 1e-3).all(), step


def test_overflow_is_counted_and_keeps_the_deepest(he_model, model):
    """Lying bodies generate up to ~30 contacts. At the engine's 20 slots the overflow is reported
    per env, and the deepest-first reduction keeps the settled penetration at the level of a run
    with 64 slots (round 1's body-order truncation let the right hand sink 3.6 cm). cases.lying_state
    starts up to 0.43 m inside the plane, so the bodies are thrown out at up to 10 m/s and tumble for
    ~1.5 s (transient penetration ~2-3 cm with either capacity); they rest by 4 s."""
    rng = np.random.default_rng(5)
    root, dof = cases.lying_state(16, rng)
    targets = np.zeros((16, 69), np.float32)
    worst = {}
    dropped = {}
    for cap in (20, 64):
        sp = _abi.default_sim_params(max_contacts=cap)
        r, d = root.copy(), dof.copy()
        cache = O.new_cache(16) if cap <= _abi.MAX_CONTACTS else None
        drops = []
        for _ in range(120):
            out = O.physics_step(he_model, sp, r, d, targets, 2, cache=cache)
            drops.append(out["dropped"].copy())
            assert (out["num_contacts"] <= cap).all()
        worst[cap] = cases.ground_gaps(model, out["rb_state"]).min()
        dropped[cap] = np.array(drops)
        assert np.abs(r[:, 7:]).max() < 0.5  # at rest
    assert dropped[20][-1].sum() > 0 and dropped[64].max() == 0
    assert worst[20] > -2e-3 and worst[64] > -2e-3, worst


def test_warm_start_converges_on_lying_bodies(he_model):
    """the solve's complementarity residual on cases.lying_state after the bodies
    settle (steps 30-60) drops >= 5x with the warm start at the same 8 iterations."""
    rng = np.random.default_rng(3)
    n = 32
    root, dof = cases.lying_state(n, rng)
    targets = np.zeros((n, 69), np.float32)
    res = {}
    for ws in (0, 1):
        sp = _abi.pgs_sim_params(warm_start=ws)
        r, d = root.copy(), dof.copy()
        cache = O.new_cache(n)
        rr = []
        for step in range(60):
            out = O.physics_step(he_model, sp, r, d, targets, 2, cache=cache)
            if step >= 30:
                rr.append(np.median(out["residual"]))
        res[ws] = float(np.mean(rr))
    assert res[1] * 5 < res[0], res


def test_cache_signature_invalidates_on_external_write(he_model, model):
    """A state written from outside (a reset) invalidates the env's cache: the next solve is cold."""
    rng = np.random.default_rng(9)
    root, dof = cases.standing_state(model, 2, rng)
    targets = np.zeros((2, 69), np.float32)
    sp = _abi.default_sim_params()
    cache = O.new_cache(2)
    r, d = root.copy(), dof.copy()
    for _ in range(3):
        O.physics_step(he_model, sp, r, d, targets, 2, cache=cache)
    assert cache[:, 7].view(np.int32).tolist() == [28, 28]  # 4 boxes x (4 normal + 2 tangential + 1 torsional rows)
    np.testing.assert_array_equal(cache[:, :3], r[:, :3])
    # env 1 is "reset" to its start state: the warm and cold steps of it agree exactly
    r2, d2 = r.copy(), d.copy()
    r2[1], d2[1] = root[1], dof[1]
    c_warm = cache.copy()
    O.physics_step(he_model, sp, r2, d2, targets, 2, cache=c_warm)
    r3, d3 = r.copy(), d.copy()
    r3[1], d3[1] = root[1], dof[1]
    O.physics_step(he_model, sp, r3, d3, targets, 2, cache=O.new_cache(2))
    np.testing.assert_array_equal(r2[1], r3[1])
    np.testing.assert_array_equal(d2[1], d3[1])


def test_limit_backstop_holds_a_joint_the_rows_cannot(he_model, model):
    """A joint 5 mrad inside its limit with 60 rad/s outward (one substep covers 1 rad) and rows that
    cannot act (no solver sweeps: they stand for a limit against a contact it cannot win): the
    integration's backstop (limit_clamp) keeps the rotation angle at pi - 0.01 on the same side of
    pi, with the outward rate removed; joints inside the limit are left alone. With the sweeps the
    row alone holds it at pi - 0.02."""
    rng = np.random.default_rng(3)
    n = 4
    root, dof = cases.standing_state(model, n, rng, xy_jitter=0.5)
    root[:, 2] += 1.5
    axis = rng.standard_normal((n, 3))
    axis /= np.linalg.norm(axis, axis=1, keepdims=True)
    j = 10  # Neck's joint (body 11): a light link
    dof[:, 3 * j:3 * j + 3, 0] = (axis * (np.pi - 0.025)).astype(np.float32)
    dof[:, 3 * j:3 * j + 3, 1] = (axis * 60.0).astype(np.float32)
    # one physics step of 1/60 s (substeps 1): the backstop's own case
    sp = _abi.pgs_sim_params(self_collision=0, kp_scale=0.0, kd_scale=0.0, solver_iterations=0, warm_start=0,
                                 substeps=1)
    r, d = root.copy(), dof.copy()
    O.physics_step(he_model, sp, r, d, np.zeros((n, 69), np.float32), 1)
    q = d[:, 3 * j:3 * j + 3, 0].astype(np.float64)
    u = d[:, 3 * j:3 * j + 3, 1].astype(np.float64)
    t = np.linalg.norm(q, axis=1)
    np.testing.assert_allclose(t, np.pi - 0.01, atol=1e-6)
    assert ((q * axis).sum(1) > 0).all()  # not wrapped to the far side
    assert ((u * q).sum(1) / t <= 1e-6).all()  # no outward rate left
    # the other joints equal a run without limits (the backstop acts only past pi - 0.01)
    r2, d2 = root.copy(), dof.copy()
    O.physics_step(he_model, _abi.pgs_sim_params(self_collision=0, kp_scale=0.0, kd_scale=0.0, solver_iterations=0,
                                                     warm_start=0, joint_limits=0, substeps=1),
                   r2, d2, np.zeros((n, 69), np.float32), 1)
    others = [k for k in range(23) if k != j]
    qs = d[:, :, 0].reshape(n, 23, 3)[:, others]
    np.testing.assert_array_equal(qs, d2[:, :, 0].reshape(n, 23, 3)[:, others])
    # with the sweeps, the limit row holds it first, at pi - 0.02
    r3, d3 = root.copy(), dof.copy()
    O.physics_step(he_model, _abi.pgs_sim_params(self_collision=0, kp_scale=0.0, kd_scale=0.0, substeps=1), r3, d3,
                   np.zeros((n, 69), np.float32), 1)
    t3 = np.linalg.norm(d3[:, 3 * j:3 * j + 3, 0].astype(np.float64), axis=1)
    assert (t3 < np.pi - 0.015).all() and (t3 > np.pi - 0.03).all()


def test_moderate_random_actions_stay_physical(he_model, model):
    """Random actions U(-0.5, 0.5) of the PD scale on standing bodies for 2 s keep every root below
    5 m/s (measured 5.7 max over 512 envs, tests/diag/energy_probe.py; CoM below 4.4) and no joint past the
    limit. The saturated U(-1, 1) case is test_physics_invariants.py::test_saturated_random_actions_stay_physical."""
    from humanoid_amd.model import pd_action_offset_scale
    n = 64
    rng = np.random.default_rng(8)
    off, sc = pd_action_offset_scale(model)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=1.0)
    sp = _abi.default_sim_params()
    cache = O.new_cache(n)
    vmax = 0.0
    for _ in range(60):
        a = rng.uniform(-0.5, 0.5, (n, 69)).astype(np.float32)
        O.physics_step(he_model, sp, root, dof, (off + sc * a).astype(np.float32), 2, cache=cache)
        vmax = max(vmax, float(np.linalg.norm(root[:, 7:10], axis=1).max()))
    q = np.linalg.norm(dof[..., 0].reshape(n, 23, 3), axis=-1)
    assert vmax < 7.0, vmax
    assert q.max() < np.pi - 0.01


def test_limit_force_is_part_of_dof_force(he_model, model):
    """dof_force is the joint's solver force, drive and limit together (PhysX's articulation
    joint solver forces): knees driven at +5 rad targets (humanoid_phc.py:441-446) rest on their
    angle limit, where the saturated drive (500 N m along the joint's axis) is held by the limit, so
    the reported force along the axis is the small inertial remainder (~5 N m), not the drive's
    500. A joint off its limit reports its drive force alone (the power reward, humanoid_phc.py:
    1297-1305, reads these)."""
    n = 4
    rng = np.random.default_rng(7)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=0.5)
    root[:, 2] += 1.5
    targets = np.zeros((n, 69), np.float32)
    targets[:, [4, 16]] = 5.0
    sp = _abi.default_sim_params(self_collision=0)
    cache = O.new_cache(n)
    for _ in range(20):
        out = O.physics_step(he_model, sp, root, dof, targets, 2, cache=cache)
    for j in (1, 5):  # L_Knee, R_Knee joints
        q = dof[:, 3 * j:3 * j + 3, 0].astype(np.float64)
        t = np.linalg.norm(q, axis=1)
        assert (t > np.pi - 0.03).all()  # on the limit
        f = out["dof_force"][:, 3 * j:3 * j + 3].astype(np.float64)
        assert (np.abs((f * q).sum(1) / t) < 50.0).all(), (f * q).sum(1) / t
    # the first step of the same bodies, far from the limit: the drive force alone (the implicit
    # drive's 1504 N m command, effort-scaled, relieved by the step's motion: ~135 N m)
    r2, d2 = cases.standing_state(model, n, np.random.default_rng(7), xy_jitter=0.5)
    r2[:, 2] += 1.5
    o2 = O.physics_step(he_model, sp, r2, d2, targets, 2, cache=O.new_cache(n))
    f = o2["dof_force"][:, [4, 16]]
    assert (np.abs(f) > 100.0).all(), f


def test_patch_friction_rows(he_model, model):
    """Patch friction: a standing body's 16 box corners are 4 patches (feet and toes), so
    its solve has 16 normal rows, then per patch 2 tangential rows and 1 torsional row: 28 rows. The
    row keys: the normal rows carry their corner keys, a patch's friction rows the body's patch key
    (HE_KEY_PATCH) with kinds 1, 2, 3. The torsional rows' bound weight is mu times the corners'
    mean distance from their centroid (the oracle's row-weight diagnostic), between the foot boxes'
    half-widths and half-diagonals."""
    rng = np.random.default_rng(4)
    n = 3
    root, dof = cases.standing_state(model, n, rng)
    sp = _abi.default_sim_params()
    cache = O.new_cache(n)
    for _ in range(3):
        O.physics_step(he_model, sp, root, dof, np.zeros((n, 69), np.float32), 2, cache=cache)
    rw = np.zeros((n, _abi.MAX_ROWS), np.float32)
    O.set_row_weight_out(rw)
    try:
        O.physics_step(he_model, sp, root, dof, np.zeros((n, 69), np.float32), 2, cache=cache)
    finally:
        O.set_row_weight_out(None)
    cnt, keys, lam = _abi.cache_rows(cache)
    assert cnt.tolist() == [28] * n
    for e in range(n):
        f = [_abi.key_fields(k) for k in keys[e, :28]]
        normals = [x for x in f if x[3] == 0]
        friction = [x for x in f if x[3] > 0]
        assert len(normals) == 16 and all(x[1] == -1 and x[2] < 8 for x in normals)
        assert sorted({x[0] for x in normals}) == sorted({x[0] for x in friction})  # 4 bodies
        assert all(x[2] == _abi.KEY_PATCH for x in friction)
        assert sorted(x[3] for x in friction) == [1] * 4 + [2] * 4 + [3] * 4
        # Gauss-Seidel order: each patch's normal rows, then its friction rows
        for r in range(1, 28):
            if f[r][3] == 0 and f[r - 1][3] == 0:
                assert f[r][0] == f[r - 1][0]  # consecutive normals belong to one patch
        tors = rw[e, :28][[x[3] == 3 for x in f]]
        assert ((tors > 0.02) & (tors < 0.2)).all(), tors  # mu = 1: r_patch in metres
        assert (lam[e, :28][[x[3] == 0 for x in f]] >= 0).all()


def test_row_budget_caps_the_solve_at_63_rows(he_model, model):
    """Lying bodies generate up to ~30 contacts, more rows than one wave holds: the reduction keeps
    the deepest contacts while their rows fit (3 for a body's first terrain point or a self pair, 2
    for its second, 1 after), so every cached solve has at most 63 rows, and the envs that overflow
    drop only speculative contacts (gap > 0) once settled."""
    rng = np.random.default_rng(5)
    n = 32
    root, dof = cases.lying_state(n, rng, on_floor=True, model=model)
    sp = _abi.pgs_sim_params()
    cache = O.new_cache(n)
    tgt = dof[..., 0].copy()
    for _ in range(40):
        out = O.physics_step(he_model, sp, root, dof, tgt, 2, cache=cache)
    gaps = np.full(n, np.inf, np.float32)
    O.set_drop_gap_out(gaps)
    try:
        out = O.physics_step(he_model, sp, root, dof, tgt, 2, cache=cache)
    finally:
        O.set_drop_gap_out(None)
    cnt = cache[:, 7].view(np.int32)
    assert (cnt <= _abi.MAX_ROWS).all() and (out["num_contacts"] <= _abi.MAX_CONTACTS).all()
    dropping = out["dropped"] > 0
    assert dropping.any(), "the case must overflow the row budget"
    assert (gaps[dropping] > 5e-3).all(), gaps[dropping]  # only speculative contacts go
