"""The physics invariants of tests/test_physics_invariants.py held by the HIP engine itself, at the
bench's size (4096 envs) where the oracle is too slow to follow every env:
* free fall from rest (drives off): the discrete semi-implicit parabola, in float32;
* free flight with the drives off and no damping: linear momentum gains exactly M g t and angular
  momentum about the CoM drifts at first order (measured with the oracle's momentum function on the
  engine's states);
* configs[1] PD stand-still at full size: after a 5 s settle every env stands still, its feet on
  the plane within the Baumgarte steady state;
* joint angles never wrap past pi under saturated random actions (limit rows + the integration's
  backstop).
"""
import numpy as np
import pytest

from humanoid_amd import _abi
from oracle import oracle as O

import cases

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
G = 9.81


def _engine(he_model, n, **sim):
    from humanoid_amd.engine import Engine
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    return Engine(he_model, n, device=0, sim_params=_abi.default_sim_params(**sim))


def _load(eng, root, dof, targets=None):
    n = root.shape[0]
    eng.root_states.copy_(torch.as_tensor(root, device="cuda:0"))
    eng.dof_state.copy_(torch.as_tensor(dof.reshape(n * 69, 2), device="cuda:0"))
    if targets is None:
        eng.dof_targets.zero_()
    else:
        eng.dof_targets.copy_(torch.as_tensor(targets, device="cuda:0"))


def test_gpu_free_fall_is_the_discrete_parabola(he_model):
    n = 4096
    rng = np.random.default_rng(0)
    root, dof = cases.random_state(n, rng, height=(6.0, 7.0), vel=0.0)
    dof[..., 1] = 0.0
    eng = _engine(he_model, n, self_collision=0, kp_scale=0.0, kd_scale=0.0, angular_damping=0.0, joint_limits=0)
    _load(eng, root, dof)
    steps = 20
    for _ in range(steps):
        eng.simulate(2)
    torch.cuda.synchronize()
    r = eng.root_states.cpu().numpy()
    # semi-implicit sub-steps of h per simulate(): SimParams.substeps physics steps, each (TGS) of
    # solver_iterations position iterations
    sub = eng.params.substeps * (eng.params.solver_iterations if eng.params.solver_type == 1 else 1)
    k = 2 * steps * sub
    dt = 1.0 / 60.0 / sub
    assert (eng.num_contacts.cpu().numpy() == 0).all()
    # fp32: each sub-step's velocity and position update rounds once, so the bound grows with their
    # count (80 sub-steps of the PGS step 2e-5; TGS's 320 of 1/480 s 8e-5)
    tol = 2.5e-7 * k
    np.testing.assert_allclose(r[:, 2], root[:, 2] - G * dt * dt * k * (k + 1) / 2, atol=tol)
    np.testing.assert_allclose(r[:, 9], -G * dt * k, atol=tol)
    # in float32 the gravity bias cancels to rounding only: 80 physics steps accumulate <= ~1e-4 rad
    np.testing.assert_allclose(eng.dof_state.view(n, 69, 2).cpu().numpy()[..., 0], dof[..., 0], atol=2e-4)


def test_gpu_free_flight_momentum(he_model, model):
    """Drives off, no damping, gravity on, 1 s: P - M g t and L_com drift at the integrator's first
    order (tests/test_physics_invariants.py pins the rate); per env the engine's drift is the
    oracle's (the same integrator in fp64), and over 1024 random states it stays within 4% of |P|
    and 15% of |L_com| (the largest seen: 2.8% / 12.5%, r02)."""
    n = 1024
    rng = np.random.default_rng(1)
    root, dof = cases.random_state(n, rng, height=(9.0, 10.0), vel=0.5, ang=0.5)
    # no limits: a free joint may spin up to pi in 1 s of undriven flight (its limit row would act)
    sim = dict(self_collision=0, kp_scale=0.0, kd_scale=0.0, angular_damping=0.0, joint_limits=0)
    eng = _engine(he_model, n, **sim)
    _load(eng, root, dof)
    sp = _abi.default_sim_params(**sim)
    me0 = O.momentum_energy(he_model, sp, root, dof)
    for _ in range(30):
        eng.simulate(2)
    torch.cuda.synchronize()
    assert (eng.num_contacts.cpu().numpy() == 0).all()
    r = eng.root_states.cpu().numpy()
    d = eng.dof_state.view(n, 69, 2).cpu().numpy()
    me1 = O.momentum_energy(he_model, sp, r, d)
    M = float(np.sum(model.mass))

    def l_com(me, rr, dd):
        c = cases.center_of_mass(model, O.forward_kinematics(he_model, rr, dd))
        return me[:, 3:6] - np.cross(c, me[:, :3])

    g = M * np.array([0, 0, -G]) * 1.0
    dP = me1[:, :3] - (me0[:, :3] + g)
    dL = l_com(me1, r, d) - l_com(me0, root, dof)
    # the oracle on the same states
    ro, do = root.copy(), dof.copy()
    for _ in range(30):
        O.physics_step(he_model, sp, ro, do, np.zeros((n, 69), np.float32), 2)
    mo = O.momentum_energy(he_model, sp, ro, do)
    dPo = mo[:, :3] - (me0[:, :3] + g)
    dLo = l_com(mo, ro, do) - l_com(me0, root, dof)
    P = np.abs(me0[:, :3]).max()
    L = np.abs(l_com(me0, root, dof)).max()
    np.testing.assert_allclose(dP, dPo, atol=1e-3 * P)
    np.testing.assert_allclose(dL, dLo, atol=1e-3 * L)
    assert np.abs(dP).max() < 0.04 * P and np.abs(dL).max() < 0.15 * L, (np.abs(dP).max(), P, np.abs(dL).max(), L)


def test_gpu_full_size_stand_still(he_model, model):
    """configs[1] at 4096 envs: 5 s to settle, then 2 s of standing still; feet on the plane."""
    n = 4096
    rng = np.random.default_rng(4)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=1.0)
    eng = _engine(he_model, n)
    _load(eng, root, dof)
    for _ in range(150):
        eng.simulate(2)
    torch.cuda.synchronize()
    r1 = eng.root_states.cpu().numpy().copy()
    for _ in range(60):
        eng.simulate(2)
    torch.cuda.synchronize()
    r = eng.root_states.cpu().numpy()
    d = eng.dof_state.view(n, 69, 2).cpu().numpy()
    assert np.abs(r[:, :3] - r1[:, :3]).max() < 2e-4
    assert np.abs(r[:, 7:]).max() < 1e-3 and np.abs(d[..., 1]).max() < 1e-3
    assert (eng.num_contacts.cpu().numpy() == 16).all() and (eng.dropped_contacts.cpu().numpy() == 0).all()
    gaps = cases.ground_gaps(model, eng.rb_state.view(n, 24, 13).cpu().numpy())
    assert gaps.min() > -2e-3 and gaps.min() < 0.02


def test_gpu_joint_angles_never_wrap(he_model, model):
    """Saturated random actions (the PD scale x U(-1, 1): targets past pi on every joint, knee-y up
    to +-5 rad) on 4096 standing envs, one substep per launch: no joint's exp map ever passes
    pi - 0.01 or comes back from the log on the far side of pi. The limit rows alone do not
    guarantee it in this regime (a knee folded against a deep self contact has no solution, and
    joints reach the 100 rad/s cap), so the integration's backstop (limit_clamp) is what this pins.
    The regime itself is violent: 500 N m on every joint spins light links at the cap and the
    bodies fly; finiteness is asserted, not plausibility."""
    from humanoid_amd.model import pd_action_offset_scale
    n = 4096
    rng = np.random.default_rng(8)
    off, sc = pd_action_offset_scale(model)
    eng = _engine(he_model, n)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=1.0)
    _load(eng, root, dof)
    cap = np.pi - 0.01
    worst, flips = 0.0, 0
    for _ in range(30):
        a = rng.uniform(-1.0, 1.0, (n, 69)).astype(np.float32)
        eng.dof_targets.copy_(torch.as_tensor(off + sc * a, device="cuda:0"))
        for _sub in range(2):
            q0 = eng.dof_state.view(n, 69, 2)[..., 0].reshape(n, 23, 3).clone()
            eng.simulate(1)
            q1 = eng.dof_state.view(n, 69, 2)[..., 0].reshape(n, 23, 3)
            t1 = q1.norm(dim=-1, keepdim=True)
            far = -q1 / t1.clamp_min(1e-12) * (2 * np.pi - t1)  # the same rotation past pi
            flips += int(((far - q0).norm(dim=-1) < (q1 - q0).norm(dim=-1)).sum())
            worst = max(worst, float(t1.max()))
    assert worst <= cap + 1e-5, worst
    assert flips == 0, flips
    assert torch.isfinite(eng.root_states).all() and torch.isfinite(eng.dof_state).all()


def test_gpu_moderate_random_actions_stay_physical(he_model, model):
    """The engine side of tests/test_limits_contacts.py::test_moderate_random_actions_stay_physical
    at full size: U(-0.25, 0.25) random actions on 4096 standing envs for 2 s keep every root below
    10 m/s and every joint inside the limit (at U(-0.5, 0.5) 6 of 4096 envs already run
    away, profiles/r02/action_regimes.json)."""
    from humanoid_amd.model import pd_action_offset_scale
    n = 4096
    rng = np.random.default_rng(8)
    off, sc = pd_action_offset_scale(model)
    eng = _engine(he_model, n)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=1.0)
    _load(eng, root, dof)
    vmax = 0.0
    for _ in range(60):
        a = rng.uniform(-0.25, 0.25, (n, 69)).astype(np.float32)
        eng.dof_targets.copy_(torch.as_tensor(off + sc * a, device="cuda:0"))
        eng.simulate(2)
        vmax = max(vmax, float(eng.root_states[:, 7:10].norm(dim=1).max()))
    q = eng.dof_state.view(n, 69, 2)[..., 0].reshape(n, 23, 3).norm(dim=-1)
    assert vmax < 10.0, vmax
    assert float(q.max()) < np.pi - 0.01


def test_gpu_sliding_bodies_decelerate_at_mu_g(he_model, model):
    """The engine side of tests/test_physics_invariants.py::test_sliding_body_decelerates_at_mu_g at
    1024 envs: lying bodies, settled, given 3 m/s along x, decelerate at mu g while they slide on
    their contact patches (per-env friction 0.25 / 0.5 / 0.75 / 1.0). Per friction, the median fitted
    deceleration within 5 % of mu g, and at least 75 % of the envs within 5 % (bodies that tip and
    roll decelerate less)."""
    n = 1024
    rng = np.random.default_rng(3)
    root, dof = cases.lying_state(n, rng, on_floor=True, model=model)
    eng = _engine(he_model, n)
    _load(eng, root, dof, dof[..., 0])
    for _ in range(45):  # settle 1.5 s
        eng.simulate(2)
    mus = np.array([0.25, 0.5, 0.75, 1.0], np.float32)[np.arange(n) % 4]
    eng.set_env_properties(None, torch.as_tensor(mus, device="cuda:0"), None)
    eng.root_states[:, 7] += 3.0
    vs = []
    for _ in range(30):
        eng.simulate(2)
        vs.append(cases.com_velocity(model, eng.rb_state.view(n, 24, 13).cpu().numpy())[:, 0])
    dec = cases.sliding_deceleration(np.array(vs), 1.0 / 30.0)
    for mu in (0.25, 0.5, 0.75, 1.0):
        d = dec[mus == mu]
        good = np.abs(d + mu * 9.81) < 0.05 * mu * 9.81
        print(f"mu {mu}: median deceleration {np.nanmedian(d):.3f} (mu g {mu * 9.81:.3f}), within 5%: {good.mean():.2f}")
        assert abs(np.nanmedian(d) + mu * 9.81) < 0.05 * mu * 9.81
        assert good.mean() >= 0.75
