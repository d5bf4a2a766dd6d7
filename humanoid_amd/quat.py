"""Host-side (numpy) quaternion helpers, xyzw convention (``puffer_phc/torch_utils.py:61``).

Used by the host motion-library loader and host glue; the device kernels carry their own
inline copies in ``csrc/he_math.h``.
"""
import numpy as np


def quat_mul(a, b):
    x1, y1, z1, w1 = a[..., 0], a[..., 1], a[..., 2], a[..., 3]
    x2, y2, z2, w2 = b[..., 0], b[..., 1], b[..., 2], b[..., 3]
    return np.stack([
        w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
        w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
        w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2,
        w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
    ], axis=-1)


def quat_conj(q):
    out = q.copy()
    out[..., :3] = -out[..., :3]
    return out


def quat_pos(q):
    """Flip sign so the real part is >= 0 (``torch_utils.py:153-161``)."""
    return np.where(q[..., 3:] < 0, -q, q)


def quat_unit(q):
    return q / np.maximum(np.linalg.norm(q, axis=-1, keepdims=True), 1e-9)


def quat_mul_norm(a, b):
    """``torch_utils.quat_mul_norm``: normalize(quat_pos(a*b))."""
    return quat_unit(quat_pos(quat_mul(a, b)))


def quat_rotate(q, v):
    qv = q[..., :3]
    w = q[..., 3:]
    t = 2.0 * np.cross(qv, v)
    return v + w * t + np.cross(qv, t)


def quat_angle_axis_poselib(q):
    """``torch_utils.quat_angle_axis`` (poselib velocity path): angle in [0, pi]."""
    s = 2 * q[..., 3] ** 2 - 1
    angle = np.arccos(np.clip(s, -1, 1))
    axis = q[..., :3] / np.maximum(np.linalg.norm(q[..., :3], axis=-1, keepdims=True), 1e-9)
    return angle, axis


def quat_to_angle_axis(q):
    """``torch_utils.quat_to_angle_axis`` (acos form, angle normalised to (-pi, pi])."""
    w = q[..., 3]
    with np.errstate(invalid="ignore", divide="ignore"):
        sin_theta = np.sqrt(1 - w * w)
        angle = 2 * np.arccos(w)
        angle = np.arctan2(np.sin(angle), np.cos(angle))
        axis = q[..., :3] / sin_theta[..., None]
        mask = np.abs(sin_theta) > 1e-5
    angle = np.where(mask, angle, 0.0)
    default = np.zeros_like(axis)
    default[..., 2] = 1
    axis = np.where(mask[..., None], axis, default)
    return angle, axis


def quat_to_exp_map(q):
    angle, axis = quat_to_angle_axis(q)
    return angle[..., None] * axis


def exp_map_to_quat(e):
    angle = np.linalg.norm(e, axis=-1)
    with np.errstate(invalid="ignore", divide="ignore"):
        axis = e / angle[..., None]
    angle_n = np.arctan2(np.sin(angle), np.cos(angle))
    mask = np.abs(angle_n) > 1e-5
    angle_n = np.where(mask, angle_n, 0.0)
    default = np.zeros_like(e)
    default[..., 2] = 1
    axis = np.where(mask[..., None], axis, default)
    axis = axis / np.maximum(np.linalg.norm(axis, axis=-1, keepdims=True), 1e-9)
    half = angle_n[..., None] / 2
    q = np.concatenate([axis * np.sin(half), np.cos(half)], axis=-1)
    return quat_unit(q)
