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


def lying_state(n, rng):
    root = np.zeros((n, 13), np.float32)
    th = np.pi / 2
    root[:, 3] = np.sin(th / 2)
    root[:, 6] = np.cos(th / 2)
    root[:, 2] = 0.12 + rng.uniform(0, 0.03, n)
    dof = np.zeros((n, 69, 2), np.float32)
    dof[..., 0] = rng.uniform(-0.2, 0.2, (n, 69))
    return root, dof
