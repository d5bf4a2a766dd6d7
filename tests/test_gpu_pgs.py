"""The PGS step on the GPU (he_sim_params.solver_type = 0, physics_kernel; rounds 1-4's default, kept
as an option) against the fp64 oracle (oracle/he_oracle_physics.c substep; its invariants:
tests/test_physics_invariants.py). Since round 5 the default is the reference's TGS (solver_type 1,
physics_kernel_tgs), which tests/test_gpu_parity.py and the other GPU tests run; this file keeps the
same comparisons for PGS: velocity-level Gauss-Seidel, 8 warm-started sweeps per 1/120 s physics step,
the midpoint bias. Joint angles, positions and CoM at 1e-4, contact sets by key, the oracle's
sensitivity probes for ill-conditioned elements (tests/test_gpu_parity.py _physics_compare)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import cases  # noqa: E402
from test_gpu_parity import _physics_compare, _random_action_gpu, _require_gpu  # noqa: E402

pytestmark = pytest.mark.gpu

PGS = dict(solver_type=0, solver_iterations=8)


def test_pgs_airborne_matches_oracle(he_model):
    """Actuated airborne bodies, one policy step."""
    _require_gpu()
    rng = np.random.default_rng(1)
    root, dof = cases.random_state(64, rng, height=(3.0, 4.0))
    targets = rng.uniform(-0.5, 0.5, (64, 69)).astype(np.float32)
    _physics_compare(he_model, root, dof, targets, self_collision=0, max_skip=0.0, max_widened=0.0, **PGS)


def test_pgs_standing_matches_oracle(he_model, model):
    """PD stand-still on the plane, 5 policy steps (16 box corners, patch friction, warm start)."""
    _require_gpu()
    rng = np.random.default_rng(2)
    root, dof = cases.standing_state(model, 64, rng, xy_jitter=1.0)
    _physics_compare(he_model, root, dof, np.zeros((64, 69), np.float32), steps=5, max_skip=0.0,
                     max_widened=0.05, **PGS)


def test_pgs_trajectories_30_steps(he_model, model):
    """north_star's joint-angle and CoM trajectories at 1e-4 over 30 policy steps under PGS: airborne
    actuated bodies (self collision on) and the PD stand-still."""
    _require_gpu()
    rng = np.random.default_rng(11)
    root, dof = cases.random_state(32, rng, height=(6.0, 7.0), ang=0.4, vel=0.5)
    targets = rng.uniform(-0.5, 0.5, (32, 69)).astype(np.float32)
    _physics_compare(he_model, root, dof, targets, steps=30, max_skip=0.0, max_widened=0.01, **PGS)
    root, dof = cases.standing_state(model, 32, rng, xy_jitter=1.0)
    _physics_compare(he_model, root, dof, np.zeros((32, 69), np.float32), steps=30, max_skip=0.0,
                     max_widened=0.05, **PGS)


def test_pgs_contact_rich_matches_oracle(he_model):
    """Tumbling near the ground and lying bodies (many contacts, self pairs), one policy step."""
    _require_gpu()
    rng = np.random.default_rng(3)
    root, dof = cases.random_state(96, rng, height=(0.85, 1.0), ang=0.8, vel=0.5)
    r2, d2 = cases.lying_state(32, rng)
    root = np.concatenate([root, r2])
    dof = np.concatenate([dof, d2])
    targets = rng.uniform(-0.5, 0.5, (128, 69)).astype(np.float32)
    _physics_compare(he_model, root, dof, targets, **PGS)


def test_pgs_domain_randomised_terrain(he_model, model):
    """configs[4]'s per-env mass scale, friction and terrain kind under PGS, 3 policy steps."""
    _require_gpu()
    n = 48
    rng = np.random.default_rng(4)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=1.0)
    root[:, 2] += 0.1
    ms = rng.uniform(0.8, 1.2, (n, 24)).astype(np.float32)
    fr = rng.uniform(0.5, 1.25, n).astype(np.float32)
    tk = (np.arange(n) % 3).astype(np.int32)
    _physics_compare(he_model, root, dof, np.zeros((n, 69), np.float32), steps=3, env_props=(ms, fr, tk),
                     max_widened=0.01, **PGS)


def test_pgs_knee_limit_matches_oracle(he_model, model):
    """Knee-y driven at +-5 rad: the limit rows hold the joint inside pi under PGS, with the limit force
    in dof_force (compared with the oracle at 0.5 N m)."""
    _require_gpu()
    n = 8
    rng = np.random.default_rng(7)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=0.5)
    root[:, 2] += 1.5
    targets = np.zeros((n, 69), np.float32)
    targets[:, [4, 16]] = np.where(np.arange(n) % 2 == 0, 5.0, -5.0)[:, None]
    eng, _ = _physics_compare(he_model, root, dof, targets, steps=20, self_collision=0, max_skip=0.0, **PGS)
    q = eng.dof_state.view(n, 69, 2).cpu().numpy()[..., 0]
    ang = np.linalg.norm(q.reshape(n, 23, 3), axis=-1)
    assert ang.max() < np.pi and ang[:, [1, 5]].min() > np.pi - 0.05


def test_pgs_overflow_counted_and_reduced(he_model):
    """Lying bodies past the slot capacity (16): the same deepest-first reduced contact set, under PGS."""
    _require_gpu()
    rng = np.random.default_rng(5)
    root, dof = cases.lying_state(32, rng)
    root[:, 2] = 0.08 + rng.uniform(0, 0.02, 32).astype(np.float32)
    eng, out = _physics_compare(he_model, root, dof, np.zeros((32, 69), np.float32), steps=1, max_skip=0.05,
                                max_widened=0.05, max_contacts=16, **PGS)
    assert (out["dropped"] > 0).sum() >= 8


def test_pgs_saturated_random_actions_on_gpu(he_model, model):
    """4096 standing envs under U(+-1) random actions for 2 s under PGS (round 4's bar for the PGS
    step, whose tail is the wedged-limb launch and the whipped pelvis): at most 0.1 % of
    roots past 10 m/s, none past 20 m/s, median internal kinetic energy under 1.5 kJ, no joint past its
    cap."""
    _require_gpu()
    n = 4096
    vmax, ke, dg = _random_action_gpu(he_model, model, n, 1.0, 60, **PGS)
    q = np.linalg.norm(dg[..., 0].reshape(n, 23, 3), axis=-1)
    print(f"PGS U(+-1): envs over 10 m/s {int((vmax > 10).sum())}/{n}, max root speed {vmax.max():.2f} m/s, "
          f"median internal KE {np.median(ke):.1f} J")
    assert vmax.max() < 20.0 and int((vmax > 10).sum()) <= n // 1000
    assert np.median(ke) < 1.5e3
    assert q.max() <= np.pi - 0.01 + 1e-5
