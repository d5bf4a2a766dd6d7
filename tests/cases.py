"""Shared input builders for parity tests (seeded, small)."""
import numpy as np


def standing_state(model, n, rng=None, xy_jitter=0.0):
    """Root upright at the height where the lowest foot-box corner touches z=0, zero dofs."""
    from humanoid_amd.synthetic import forward_kinematics, min_foot_height
    T = 1
    local = np.zeros((T, model.num_bodies, 4))
    local[..., 3] = 1
    grot, gpos = forward_kinematics(model, np.array([[0, 0, 0, 1.0]]), local, np.zeros((T, 3)))
    z = -min_foot_height(model, grot, gpos)
    root = np.zeros((n, 13), np.float32)
    root[:, 2] = z
    root[:, 6] = 1.0
    if rng is not None and xy_jitter:
        root[:, :2] = rng.uniform(-xy_jitter, xy_jitter, (n, 2))
    dof = np.zeros((n, 69, 2), np.float32)
    return root, dof


def random_state(n, rng, height=(0.9, 1.6), ang=0.6, vel=1.0, tilt=0.3):
    root = np.zeros((n, 13), np.float32)
    root[:, :2] = rng.uniform(-1, 1, (n, 2))
    root[:, 2] = rng.uniform(*height, n)
    axis = rng.normal(size=(n, 3))
    axis /= np.linalg.norm(axis, axis=1, keepdims=True)
    th = rng.uniform(0, tilt, n)
    root[:, 3:6] = axis * np.sin(th / 2)[:, None]
    root[:, 6] = np.cos(th / 2)
    root[:, 7:10] = rng.normal(0, vel, (n, 3))
    root[:, 10:13] = rng.normal(0, vel, (n, 3))
    dof = np.zeros((n, 69, 2), np.float32)
    dof[..., 0] = rng.uniform(-ang, ang, (n, 69))
    dof[..., 1] = rng.normal(0, vel, (n, 69))
    return root, dof


def lying_state(n, rng, on_floor=False, model=None):
    """A body lying on its back/front (pi/2 about x) with random joint angles in +-0.2 rad. By default
    the root sits at 0.12-0.15 m, so limbs start up to ~0.4 m inside the plane and are thrown out
    (a violent, tumbling transient); with on_floor=True each body is lifted so its lowest contact
    candidate is 5 mm above the plane (a fallen body at rest: ~20-30 contacts)."""
    root = np.zeros((n, 13), np.float32)
    th = np.pi / 2
    root[:, 3] = np.sin(th / 2)
    root[:, 6] = np.cos(th / 2)
    root[:, 2] = 0.12 + rng.uniform(0, 0.03, n)
    dof = np.zeros((n, 69, 2), np.float32)
    dof[..., 0] = rng.uniform(-0.2, 0.2, (n, 69))
    if on_floor:
        from humanoid_amd import _abi
        from humanoid_amd.model import load_default_model
        from oracle import oracle as O
        model = model or load_default_model()
        rb = O.forward_kinematics(_abi.make_model(model), root, dof)
        root[:, 2] += (0.005 - ground_gaps(model, rb).min(-1)).astype(np.float32)
    return root, dof


def _qmat(q):
    """xyzw quaternions [...,4] -> rotation matrices [...,3,3] (float64)."""
    q = np.asarray(q, np.float64)
    x, y, z, w = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    return np.stack([
        np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
        np.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
        np.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)], -2)


def center_of_mass(model, rb_state):
    """Mass-weighted centre of mass [N,3] from rigid-body rows [N,24,13] (body origin + rotation)."""
    rb = np.asarray(rb_state, np.float64)
    R = _qmat(rb[..., 3:7])
    com_w = rb[..., :3] + np.einsum("nbij,bj->nbi", R, np.asarray(model.com, np.float64))
    m = np.asarray(model.mass, np.float64)
    return (com_w * m[None, :, None]).sum(1) / m.sum()


def com_velocity(model, rb_state):
    """Mass-weighted centre-of-mass velocity [N,3] from rigid-body rows [N,24,13] (origin velocity
    v, angular velocity w: each body's COM moves at v + w x R com)."""
    rb = np.asarray(rb_state, np.float64)
    R = _qmat(rb[..., 3:7])
    r = np.einsum("nbij,bj->nbi", R, np.asarray(model.com, np.float64))
    vc = rb[..., 7:10] + np.cross(rb[..., 10:13], r)
    m = np.asarray(model.mass, np.float64)
    return (vc * m[None, :, None]).sum(1) / m.sum()


def sliding_deceleration(vx, dt, v_min=0.5):
    """Fitted slope of the x velocity [T, N] over the samples while the env still slides (v > v_min),
    per env (nan with fewer than 4 such samples)."""
    t = (np.arange(vx.shape[0]) + 1) * dt
    out = []
    for e in range(vx.shape[1]):
        on = vx[:, e] > v_min
        out.append(np.polyfit(t[on], vx[on, e], 1)[0] if on.sum() > 3 else np.nan)
    return np.array(out)


def ground_gaps(model, rb_state):
    """Signed distance to the z=0 plane of every terrain contact candidate of each body (sphere
    centre, capsule end points, box corners, minus the radius) -> min over candidates [N,24]."""
    from humanoid_amd import _abi
    rb = np.asarray(rb_state, np.float64)
    R = _qmat(rb[..., 3:7])
    n = rb.shape[0]
    out = np.full((n, rb.shape[1]), np.inf)
    for b in range(rb.shape[1]):
        g = np.asarray(model.geom_params[b], np.float64)
        t = int(model.geom_type[b])
        if t == 0:
            pts, rad = g[None, 0:3], g[3]
        elif t == 1:
            pts, rad = np.stack([g[0:3], g[3:6]]), g[6]
        else:
            bm = _qmat(g[6:10])
            sg = np.array([[(c & 1) * 2 - 1, ((c >> 1) & 1) * 2 - 1, ((c >> 2) & 1) * 2 - 1] for c in range(8)], np.float64)
            pts, rad = g[None, 0:3] + (sg * g[3:6]) @ bm.T, 0.0
        w = rb[:, b, None, :3] + np.einsum("nij,kj->nki", R[:, b], pts)
        out[:, b] = w[..., 2].min(-1) - rad
    return out


def expmap_tol(dof_pos, atol=1e-4, dq=1e-6):
    """Per-element tolerance of exp-map joint coordinates (quat_to_exp_map, torch_utils.py) computed
    from float32 quaternions: the angle is 2 acos(w), whose conditioning is 1 / sin(theta / 2), so a
    quaternion that agrees to dq (a few float32 ulps of w ~ 1) gives an angle -- and exp-map
    components -- that agree to 2 dq / sin(theta / 2): 1e-4 (north_star) for joints bent past
    ~1.2 deg, the fp32 acos bound below that (torch's own float32 rounding of the reference)."""
    v = np.asarray(dof_pos, np.float64).reshape(dof_pos.shape[0], -1, 3)
    th = np.linalg.norm(v, axis=-1, keepdims=True)
    tol = atol + 2.0 * dq / np.maximum(np.sin(th / 2.0), 1e-12)
    return np.broadcast_to(tol, v.shape).reshape(dof_pos.shape)


def assert_expmap_close(got, ref):
    tol = expmap_tol(ref)
    bad = np.abs(np.asarray(got) - np.asarray(ref)) > tol
    assert not bad.any(), (f"{bad.sum()} exp-map coordinates out of tolerance: got {np.asarray(got)[bad][:4]} "
                           f"ref {np.asarray(ref)[bad][:4]} tol {tol[bad][:4]}")


def rounding_noise(root, dof, seed):
    """In place: the fp32 engine's rounding, modelled for the oracle's sensitivity probes
    (test_gpu_parity._cond_close): joint angles + 1e-6 rad N(0, 1), joint and root velocities
    x (1 + 1e-6 N(0, 1)) -- a few fp32 ulps of each, drawn afresh in every policy step, since the
    engine rounds in every step (its velocity solve through a stiff factor most of all)."""
    rng = np.random.default_rng(seed)
    dof[..., 0] += (1e-6 * rng.standard_normal(dof[..., 0].shape)).astype(np.float32)
    dof[..., 1] *= (1.0 + 1e-6 * rng.standard_normal(dof[..., 1].shape)).astype(np.float32)
    root[:, 7:13] *= (1.0 + 1e-6 * rng.standard_normal(root[:, 7:13].shape)).astype(np.float32)


def probe_physics_step(he_model, sp, root, dof, targets, calls, cache, seed, **props):
    """One oracle policy step of a sensitivity probe (test_gpu_parity._cond_close), in place on
    root / dof / cache: the fp32 engine's rounding modelled on the state (rounding_noise) and on the
    contact solve's Delassus operator and right-hand side (oracle set_probe_noise, relative 1e-6),
    fresh in every step."""
    from oracle import oracle as O
    rounding_noise(root, dof, seed)
    O.set_probe_noise(seed, 1e-6)
    try:
        return O.physics_step(he_model, sp, root, dof, targets, calls, cache=cache, **props)
    finally:
        O.set_probe_noise(0, 0.0)
