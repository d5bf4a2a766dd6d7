"""Synthetic AMASS-schema clips (SURVEY §8d recipe) -- AMASS / SMPL data are not available offline.

Each clip is a dict with the schema written by ``scripts/phc_convert_amass_data.py:186-194``:
``root_trans_offset`` [T,3], ``pose_aa`` [T,72], ``pose_quat_global`` [T,24,4] (xyzw),
``beta`` zeros(16), ``gender`` "neutral", ``fps`` 30.

Recipe (seeded ``numpy.random.default_rng``):
* local rotation vectors: random walk in exp-map, sigma 0.05 rad/frame, Gaussian-smoothed
  (sigma 2 frames), magnitude clipped to 1.2 rad;
* ``pose_quat_global`` by forward kinematics over the MJCF tree;
* root translation: random walk at ~1 m/s in a random heading; z chosen so the lowest foot-box
  corner over the clip touches z = 0.
"""
from __future__ import annotations

import numpy as np
from scipy.ndimage import gaussian_filter1d
from scipy.spatial.transform import Rotation as sRot

from .model import GEOM_BOX, HumanoidModel

FOOT_BODIES = ("L_Ankle", "L_Toe", "R_Ankle", "R_Toe")


def _box_corners(p):
    c, e = p[:3], p[3:6]
    signs = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)], np.float64)
    R = sRot.from_quat(p[6:10]).as_matrix()
    return c + (signs * e) @ R.T


def forward_kinematics(model: HumanoidModel, root_rot: np.ndarray, local_rot: np.ndarray,
                       root_pos: np.ndarray):
    """root_rot [T,4] xyzw, local_rot [T,B,4] (entry 0 ignored), root_pos [T,3] ->
    global rot [T,B,4], global pos [T,B,3] (float64)."""
    T, B = local_rot.shape[:2]
    grot = [None] * B
    gpos = [None] * B
    grot[0] = sRot.from_quat(root_rot)
    gpos[0] = root_pos.astype(np.float64)
    for b in range(1, B):
        p = model.parents[b]
        gpos[b] = gpos[p] + grot[p].apply(model.local_pos[b])
        grot[b] = grot[p] * sRot.from_quat(local_rot[:, b])
    q = np.stack([r.as_quat() for r in grot], axis=1)
    return q, np.stack(gpos, axis=1)


def min_foot_height(model: HumanoidModel, grot: np.ndarray, gpos: np.ndarray) -> float:
    zmin = np.inf
    for name in FOOT_BODIES:
        b = model.body_names.index(name)
        if model.geom_type[b] != GEOM_BOX:
            continue
        corners = _box_corners(model.geom_params[b])  # [8,3] body frame
        R = sRot.from_quat(grot[:, b])
        for c in corners:
            zmin = min(zmin, float((gpos[:, b] + R.apply(c))[:, 2].min()))
    return zmin


def _to_clip(model, root_rotvec, local_rotvec, root_xy, fps):
    T = root_rotvec.shape[0]
    B = model.num_bodies
    local_q = np.zeros((T, B, 4))
    local_q[..., 3] = 1.0
    local_q[:, 1:] = sRot.from_rotvec(local_rotvec.reshape(-1, 3)).as_quat().reshape(T, B - 1, 4)
    root_q = sRot.from_rotvec(root_rotvec).as_quat()
    # local_pos[0] of the root body is its MJCF offset; translation starts from 0 z then is fixed
    root_pos = np.concatenate([root_xy, np.zeros((T, 1))], axis=-1)
    grot, gpos = forward_kinematics(model, root_q, local_q, root_pos)
    root_pos[:, 2] -= min_foot_height(model, grot, gpos)
    grot, gpos = forward_kinematics(model, root_q, local_q, root_pos)
    pose_aa = np.concatenate([root_rotvec[:, None], local_rotvec], axis=1).reshape(T, -1)
    return {
        "root_trans_offset": root_pos.astype(np.float32),
        "pose_aa": pose_aa.astype(np.float32),
        "pose_quat_global": grot.astype(np.float32),
        "beta": np.zeros(16, np.float32),
        "gender": "neutral",
        "fps": int(fps),
    }


def make_clip(model: HumanoidModel, rng: np.random.Generator, num_frames=150, fps=30,
              step_sigma=0.05, smooth_sigma=2.0, max_angle=1.2, speed=1.0):
    T, B = num_frames, model.num_bodies
    walk = np.cumsum(rng.normal(0.0, step_sigma, size=(T, B - 1, 3)), axis=0)
    walk = gaussian_filter1d(walk, smooth_sigma, axis=0, mode="nearest")
    ang = np.linalg.norm(walk, axis=-1, keepdims=True)
    walk = np.where(ang > max_angle, walk * (max_angle / np.maximum(ang, 1e-12)), walk)
    heading = rng.uniform(-np.pi, np.pi)
    # root: heading about z plus a small smoothed tilt walk
    tilt = gaussian_filter1d(np.cumsum(rng.normal(0.0, 0.01, size=(T, 3)), axis=0), smooth_sigma,
                             axis=0, mode="nearest")
    tilt[:, 2] = 0.0
    root_rotvec = (sRot.from_rotvec(np.array([0.0, 0.0, heading])) * sRot.from_rotvec(tilt)).as_rotvec()
    dt = 1.0 / fps
    direction = np.array([np.cos(heading), np.sin(heading)])
    spd = speed * (1.0 + 0.2 * gaussian_filter1d(rng.normal(size=T), smooth_sigma, mode="nearest"))
    root_xy = np.cumsum(spd[:, None] * direction[None] * dt, axis=0)
    root_xy -= root_xy[0]
    return _to_clip(model, root_rotvec, walk, root_xy, fps)


def make_standstill_clip(model: HumanoidModel, num_frames=150, fps=30):
    """Config 2: identity local rotations, constant root, feet on the ground."""
    T, B = num_frames, model.num_bodies
    return _to_clip(model, np.zeros((T, 3)), np.zeros((T, B - 1, 3)), np.zeros((T, 2)), fps)


def make_clip_set(model: HumanoidModel, num_clips: int, seed=0, num_frames=150, fps=30):
    rng = np.random.default_rng(seed)
    return {f"synthetic_{i:04d}": make_clip(model, rng, num_frames=num_frames, fps=fps)
            for i in range(num_clips)}
