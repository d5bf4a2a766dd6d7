"""Independent pins of the physics oracle's dynamics terms (VERDICT r04 "weak" 1: the oracle restates the
kernel's own algorithm -- the same spatial algebra about the root origin, CRBA, RNEA and row Jacobians --
so a modelling error shared by both passes the GPU-vs-oracle parity).

Here the terms are rebuilt from nothing but the body poses: a float64 numpy forward kinematics of the
model blob (parents, joint offsets, the exp-map ball joints), differentiated numerically along the
generalized velocity's own flow (root: world angular velocity w and origin velocity v, q_root(e) =
exp(e w) q_root, p(e) = p + e v; joint b: Rl_b(e) = Rl_b exp(e u_b), the child-frame relative rate --
the flow the integrator follows, oracle integrate_positions), and textbook rigid-body mechanics about
each body's centre of mass:
* the joint-space inertia: H = sum_b m_b Jv_b^T Jv_b + Jw_b^T (R_b I_b R_b^T) Jw_b, Jacobians by central
  differences of the centres of mass and rotations (against ``dynamics_terms``' CRBA H);
* the bias: at constant u the bodies' accelerations are the second derivatives of the poses along the
  flow, and c = sum_b Jv_b^T m_b (a_b - g) + Jw_b^T (I_w alpha_b + w_b x I_w w_b) (Newton-Euler by
  virtual power, against the oracle's RNEA bias with gravity);
* momentum and kinetic energy (against ``momentum_energy``, which the free-flight invariants of
  tests/test_physics_invariants.py read: those invariants are then measured by an independent yardstick);
* a contact row J_r = d . dx/du of a material point (against ``row_jacobian``'s S_i . (rho, d));
* the rigid-body rows' velocities (body origin linear velocity and world angular velocity, the state
  contract: DESIGN §3) and poses of ``forward_kinematics``.
Oracle-only (CPU); the GPU is held to the oracle by tests/test_gpu_parity.py and tests/test_full_size.py.
"""
import numpy as np
import pytest

from humanoid_amd import _abi
from oracle import oracle as O

import cases

NB, ND, NG = 24, 69, 75
G = np.array([0.0, 0.0, np.float32(-9.81)], np.float64)  # he_sim_params.gravity is fp32


def _skew(v):
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def _rot(v):
    """Rodrigues: rotation matrix of rotation vector v (float64)."""
    th = float(np.linalg.norm(v))
    K = _skew(v)
    if th < 1e-8:
        return np.eye(3) + K + 0.5 * K @ K
    return np.eye(3) + np.sin(th) / th * K + (1.0 - np.cos(th)) / (th * th) * K @ K


def _qmat(q):  # xyzw
    x, y, z, w = q / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def _vee_log(Rm):
    """Rotation vector of a rotation matrix (angles well below pi here)."""
    v = np.array([Rm[2, 1] - Rm[1, 2], Rm[0, 2] - Rm[2, 0], Rm[1, 0] - Rm[0, 1]]) / 2.0  # sin(th) axis
    s = np.linalg.norm(v)
    th = np.arctan2(s, (np.trace(Rm) - 1.0) / 2.0)  # accurate at small angles too (arccos is not)
    return v if s < 1e-300 else v * (th / s)


class Body:
    """The model blob as float64 arrays."""

    def __init__(self, m):
        self.parents = np.array(m.parents[:NB])
        self.local_pos = np.array([list(m.local_pos[b]) for b in range(NB)], np.float64)
        self.mass = np.array(m.mass[:NB], np.float64)
        self.com = np.array([list(m.com[b]) for b in range(NB)], np.float64)
        ib = np.array([list(m.inertia[b]) for b in range(NB)], np.float64)
        self.I = np.array([[[i[0], i[3], i[4]], [i[3], i[1], i[5]], [i[4], i[5], i[2]]] for i in ib])


def _flow(root, dof, u, e):
    """The pose after flowing for e along generalized velocity u [75] (root w, root v, 69 joint rates)
    from the fp32 state (root [13], dof [69,2]) taken exactly: (p0, R0, [Rl_b])."""
    p0 = root[:3].astype(np.float64) + e * u[3:6]
    R0 = _rot(e * u[0:3]) @ _qmat(root[3:7].astype(np.float64))
    q = dof[:, 0].astype(np.float64)
    Rl = [_rot(q[3 * b:3 * b + 3]) @ _rot(e * u[6 + 3 * b:9 + 3 * b]) for b in range(NB - 1)]
    return p0, R0, Rl


def _fk(B, pose):
    p0, R0, Rl = pose
    R = np.zeros((NB, 3, 3))
    p = np.zeros((NB, 3))
    R[0], p[0] = R0, p0
    for b in range(1, NB):
        a = B.parents[b]
        R[b] = R[a] @ Rl[b - 1]
        p[b] = p[a] + R[a] @ B.local_pos[b]
    return R, p


def _coms(B, R, p):
    return p + np.einsum("bij,bj->bi", R, B.com)


def _gen_u(root, dof):
    return np.concatenate([root[10:13], root[7:10], dof[:, 1]]).astype(np.float64)


def _jacobians(B, root, dof, h=1e-6):
    """Jv [NB,3,75] (centres of mass), Jo [NB,3,75] (world angular velocities), Jp [NB,3,75] (origins)."""
    Jv, Jo, Jp = np.zeros((NB, 3, NG)), np.zeros((NB, 3, NG)), np.zeros((NB, 3, NG))
    for i in range(NG):
        ei = np.zeros(NG)
        ei[i] = 1.0
        Rp, pp = _fk(B, _flow(root, dof, ei, h))
        Rm, pm = _fk(B, _flow(root, dof, ei, -h))
        Jv[:, :, i] = (_coms(B, Rp, pp) - _coms(B, Rm, pm)) / (2 * h)
        Jp[:, :, i] = (pp - pm) / (2 * h)
        for b in range(NB):
            Jo[b, :, i] = _vee_log(Rp[b] @ Rm[b].T) / (2 * h)
    return Jv, Jo, Jp


def _states(n, seed):
    rng = np.random.default_rng(seed)
    root, dof = cases.random_state(n, rng, height=(1.0, 2.0), vel=1.0, ang=0.6, tilt=0.8)
    return root, dof


@pytest.fixture(scope="module")
def B(he_model):
    return Body(he_model)


@pytest.fixture(scope="module")
def sample(he_model, B):
    root, dof = _states(4, 11)
    jac = [_jacobians(B, root[e], dof[e]) for e in range(root.shape[0])]
    return root, dof, jac


def test_forward_kinematics_poses_and_velocities(he_model, B, sample):
    """The oracle's rigid-body rows: body origins and rotations equal the numpy FK; their linear
    velocity is the origin's (Jp u) and the angular velocity the world rate (Jo u)."""
    root, dof, jac = sample
    rb = O.forward_kinematics(he_model, root, dof).astype(np.float64)
    for e in range(root.shape[0]):
        R, p = _fk(B, _flow(root[e], dof[e], np.zeros(NG), 0.0))
        Rq = np.stack([_qmat(rb[e, b, 3:7]) for b in range(NB)])
        np.testing.assert_allclose(rb[e, :, :3], p, atol=2e-6)
        np.testing.assert_allclose(Rq, R, atol=2e-6)
        u = _gen_u(root[e], dof[e])
        Jv, Jo, Jp = jac[e]
        np.testing.assert_allclose(rb[e, :, 7:10], Jp @ u, atol=2e-5, rtol=1e-5)
        np.testing.assert_allclose(rb[e, :, 10:13], Jo @ u, atol=2e-5, rtol=1e-5)


def test_joint_space_inertia_is_the_kinetic_energy_metric(he_model, B, sample):
    """CRBA's H (spatial inertias about the root origin, composite sums over subtrees) equals the
    metric of the bodies' kinetic energy about their centres of mass, entry by entry."""
    root, dof, jac = sample
    H, _ = O.dynamics_terms(he_model, _abi.default_sim_params(), root, dof)
    for e in range(root.shape[0]):
        Jv, Jo, _ = jac[e]
        R, _p = _fk(B, _flow(root[e], dof[e], np.zeros(NG), 0.0))
        Hi = np.zeros((NG, NG))
        for b in range(NB):
            Iw = R[b] @ B.I[b] @ R[b].T
            Hi += B.mass[b] * Jv[b].T @ Jv[b] + Jo[b].T @ Iw @ Jo[b]
        scale = np.abs(Hi).max()
        np.testing.assert_allclose(H[e], Hi, atol=1e-8 * scale)  # measured 1.6e-10 of the largest entry
        assert np.allclose(H[e], H[e].T)


def test_bias_is_newton_euler_along_the_flow(he_model, B, sample):
    """The RNEA bias (gravity and the velocity products) equals the generalized force of the bodies'
    Newton-Euler wrenches when u is held constant: accelerations are second derivatives of the poses
    along the flow, forces and torques about each centre of mass, mapped by virtual power."""
    root, dof, jac = sample
    _, bias = O.dynamics_terms(he_model, _abi.default_sim_params(), root, dof)
    h, d = 1e-4, 1e-5
    for e in range(root.shape[0]):
        u = _gen_u(root[e], dof[e])
        Jv, Jo, _ = jac[e]
        poses = {s: _fk(B, _flow(root[e], dof[e], u, s)) for s in (-h - d, -h + d, -h, 0.0, h - d, h + d, h, -d, d)}
        a = (_coms(B, *poses[h]) - 2 * _coms(B, *poses[0.0]) + _coms(B, *poses[-h])) / (h * h)

        def omega(s):  # world angular velocities at flow time s
            Rp, Rm = poses[s + d][0], poses[s - d][0]
            return np.stack([_vee_log(Rp[b] @ Rm[b].T) / (2 * d) for b in range(NB)])

        w = omega(0.0)
        alpha = (omega(h) - omega(-h)) / (2 * h)
        R0 = poses[0.0][0]
        c = np.zeros(NG)
        for b in range(NB):
            Iw = R0[b] @ B.I[b] @ R0[b].T
            F = B.mass[b] * (a[b] - G)
            T = Iw @ alpha[b] + np.cross(w[b], Iw @ w[b])
            c += Jv[b].T @ F + Jo[b].T @ T
        np.testing.assert_allclose(bias[e], c, atol=1e-7 * np.abs(c).max())  # measured <= 2.5e-9
        # and the velocity-product part alone (gravity is most of the bias at these rates)
        cg = sum(Jv[b].T @ (-B.mass[b] * G) for b in range(NB))
        np.testing.assert_allclose(bias[e] - cg, c - cg, atol=1e-6 * np.abs(c - cg).max())  # measured <= 5.9e-8


def test_momentum_and_energy_by_textbook_sums(he_model, B, sample):
    """``momentum_energy`` (which the free-flight invariants read) equals P = sum m v_c,
    L_0 = sum (c x m v_c + I_w w), KE = sum 1/2 (m |v_c|^2 + w . I_w w), PE = -sum m g . c."""
    root, dof, jac = sample
    me = O.momentum_energy(he_model, _abi.default_sim_params(), root, dof)
    for e in range(root.shape[0]):
        u = _gen_u(root[e], dof[e])
        Jv, Jo, _ = jac[e]
        R, p = _fk(B, _flow(root[e], dof[e], np.zeros(NG), 0.0))
        cm = _coms(B, R, p)
        vc, w = Jv @ u, Jo @ u
        P = (B.mass[:, None] * vc).sum(0)
        L = sum(np.cross(cm[b], B.mass[b] * vc[b]) + R[b] @ B.I[b] @ R[b].T @ w[b] for b in range(NB))
        ke = sum(0.5 * (B.mass[b] * vc[b] @ vc[b] + w[b] @ (R[b] @ B.I[b] @ R[b].T) @ w[b]) for b in range(NB))
        pe = -(B.mass * (cm @ G)).sum()
        np.testing.assert_allclose(me[e, :3], P, rtol=1e-7, atol=1e-7 * np.abs(P).max())
        np.testing.assert_allclose(me[e, 3:6], L, rtol=1e-7, atol=1e-7 * np.abs(L).max())
        np.testing.assert_allclose(me[e, 6], ke, rtol=1e-8)
        np.testing.assert_allclose(me[e, 7], pe, rtol=1e-8)


def test_contact_row_is_the_point_velocity_along_its_direction(he_model, B, sample):
    """A terrain contact row J_r = S_i . ((x - o) x d, d) over the body's chain equals d . dx/du of the
    material point x fixed to the body."""
    root, dof, jac = sample
    n = root.shape[0]
    rng = np.random.default_rng(5)
    body = rng.integers(0, NB, n)
    x, dvec, local = np.zeros((n, 3)), np.zeros((n, 3)), np.zeros((n, 3))
    for e in range(n):
        R, p = _fk(B, _flow(root[e], dof[e], np.zeros(NG), 0.0))
        local[e] = B.com[body[e]] + rng.normal(0.0, 0.05, 3)
        x[e] = p[body[e]] + R[body[e]] @ local[e]
        dv = rng.normal(size=3)
        dvec[e] = dv / np.linalg.norm(dv)
    z = O.point_jacobian(he_model, root, dof, body, x, dvec)
    h = 1e-6
    for e in range(n):
        zi = np.zeros(NG)
        for i in range(NG):
            ei = np.zeros(NG)
            ei[i] = 1.0
            Rp, pp = _fk(B, _flow(root[e], dof[e], ei, h))
            Rm, pm = _fk(B, _flow(root[e], dof[e], ei, -h))
            b = body[e]
            zi[i] = dvec[e] @ ((pp[b] + Rp[b] @ local[e]) - (pm[b] + Rm[b] @ local[e])) / (2 * h)
        np.testing.assert_allclose(z[e], zi, atol=1e-7 * max(1.0, np.abs(zi).max()))
        # only the body's chain carries the row
        assert np.count_nonzero(np.abs(zi) > 1e-9) <= 30  # the longest chain: 6 root + 8 x 3 dofs


def _log(Rm):
    """Rotation vector of a rotation matrix, any angle below pi."""
    return _vee_log(Rm)


@pytest.mark.parametrize("angle", [0.003, 0.4, 1.5, 2.8])
def test_limit_rows_map_the_joint_rate_to_exp_map_rates(angle):
    """The joint-limit rows read a ball joint's exp-map coordinate rates as J_r^-1(q) u (oracle
    jr_inv_row): d/de log(exp(q) exp(e u)) at e = 0, by central differences. The angle row's direction
    q^ = q / |q| is the rate of |q| (d|q|/dt = q^ . u)."""
    rng = np.random.default_rng(int(angle * 1000))
    for _ in range(4):
        ax = rng.normal(size=3)
        q = ax / np.linalg.norm(ax) * angle
        M = O.jr_inv(q)
        h = 1e-6
        Rq = _rot(q)
        for k in range(3):
            ek = np.zeros(3)
            ek[k] = 1.0
            fd = (_log(Rq @ _rot(h * ek)) - _log(Rq @ _rot(-h * ek))) / (2 * h)
            np.testing.assert_allclose(M[:, k], fd, atol=2e-8)
        u = rng.normal(size=3)
        hr = 1e-4 * angle  # |q| curves on the scale of |q| itself
        rate = (np.linalg.norm(_log(Rq @ _rot(hr * u))) - np.linalg.norm(_log(Rq @ _rot(-hr * u)))) / (2 * hr)
        np.testing.assert_allclose(rate, q / np.linalg.norm(q) @ u, atol=2e-8)
