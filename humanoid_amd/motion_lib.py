"""Motion library: host-side clip ingestion + device-side sampling.

Ingestion (host, once per resample) restates, in numpy, what the reference does per clip in
``MotionLibSMPL.load_motion_with_skeleton`` (``motion_lib.py:743-824``) on its deterministic
path (no random crop / heading, ``is_deterministic=True``):

* ``SkeletonState.from_rotation_and_root_translation(..., is_local=False)``
  (``poselib_skeleton.py:716-736``): global rotations given; local rotations
  ``quat_mul_norm(inv(parent), child)`` (``:574-592``); global translations by FK (``:518-539``);
* ``SkeletonMotion.from_skeleton_state`` (``poselib_skeleton.py:1166-1190``): velocities by
  ``np.gradient`` + Gaussian filter sigma 2 (``:1230-1238``), angular velocities from successive
  rotation differences (``:1240-1251``);
* ``compute_motion_dof_vels_jit`` (``motion_lib.py:119-140``);
* concatenation into flat frame tables with ``length_starts`` (``motion_lib.py:396-420``).

Sampling (``get_motion_state``, ``motion_lib.py:549-673``) runs on the device inside the fused
imitation kernel (``csrc/he_imitation.hip``); this module only holds and uploads the tables.
"""
from __future__ import annotations

import os
import os.path as osp
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
from scipy.ndimage import gaussian_filter1d

from . import quat as Q
from .model import HumanoidModel


@dataclass
class MotionTables:
    """Concatenated per-frame tables (all float32 except the index arrays)."""
    gts: np.ndarray      # [F,B,3] global translation
    grs: np.ndarray      # [F,B,4] global rotation xyzw
    lrs: np.ndarray      # [F,B,4] local rotation xyzw
    gvs: np.ndarray      # [F,B,3] global velocity
    gavs: np.ndarray     # [F,B,3] global angular velocity
    dvs: np.ndarray      # [F,B-1,3] dof velocity
    num_frames: np.ndarray   # int64 [M]
    length_starts: np.ndarray  # int64 [M]
    lengths: np.ndarray  # f32 [M]   (num_frames-1)/fps
    dt: np.ndarray       # f32 [M]   1/fps
    fps: np.ndarray      # f32 [M]

    @property
    def num_motions(self) -> int:
        return int(self.num_frames.shape[0])

    @property
    def total_frames(self) -> int:
        return int(self.gts.shape[0])


def clip_to_motion(model: HumanoidModel, clip: dict) -> Dict[str, np.ndarray]:
    """One clip -> per-frame tables (numpy restatement of the poselib path, float32 math)."""
    grs = np.asarray(clip["pose_quat_global"], np.float32)
    trans = np.asarray(clip["root_trans_offset"], np.float32)
    fps = int(clip.get("fps", 30))
    T, B = grs.shape[:2]
    parents = model.parents
    # local rotations (poselib_skeleton.py:574-592)
    lrs = np.empty_like(grs)
    lrs[:, 0] = grs[:, 0]
    for b in range(1, B):
        lrs[:, b] = Q.quat_mul_norm(Q.quat_conj(grs[:, parents[b]]), grs[:, b])
    # FK translations (poselib_skeleton.py:518-539; transform_mul torch_utils.py:321-330)
    local_t = model.local_pos.astype(np.float32)
    g_r = [None] * B
    g_t = [None] * B
    g_r[0] = lrs[:, 0]
    g_t[0] = trans
    for b in range(1, B):
        p = parents[b]
        g_r[b] = Q.quat_mul_norm(g_r[p], lrs[:, b])
        g_t[b] = Q.quat_rotate(g_r[p], np.broadcast_to(local_t[b], (T, 3))) + g_t[p]
    gts = np.stack(g_t, axis=1).astype(np.float32)
    dt = 1.0 / fps
    # global velocity (poselib_skeleton.py:1230-1238)
    gvs = np.gradient(gts, axis=-3) / dt
    gvs = gaussian_filter1d(gvs, 2, axis=-3, mode="nearest").astype(np.float32)
    # global angular velocity (poselib_skeleton.py:1240-1251)
    diff = np.zeros_like(grs)
    diff[..., 3] = 1.0
    diff[:-1] = Q.quat_mul_norm(grs[1:], Q.quat_conj(grs[:-1]))
    ang, axis = Q.quat_angle_axis_poselib(diff)
    gavs = axis * ang[..., None] / dt
    gavs = gaussian_filter1d(gavs.astype(np.float32), 2, axis=-3, mode="nearest").astype(np.float32)
    # dof velocities (motion_lib.py:119-140)
    if T > 1:
        d = Q.quat_mul(Q.quat_conj(lrs[:-1]), lrs[1:])
        a, ax = Q.quat_to_angle_axis(d)
        dv = (ax * a[..., None] / dt)[:, 1:]
        dvs = np.concatenate([dv, dv[-1:]], axis=0).astype(np.float32)
    else:
        dvs = np.zeros((T, B - 1, 3), np.float32)
    return {"gts": gts, "grs": grs, "lrs": lrs.astype(np.float32), "gvs": gvs, "gavs": gavs,
            "dvs": dvs, "fps": fps, "num_frames": T}


def build_tables(model: HumanoidModel, clips: List[dict]) -> MotionTables:
    ms = [clip_to_motion(model, c) for c in clips]
    nf = np.array([m["num_frames"] for m in ms], np.int64)
    starts = np.concatenate([[0], np.cumsum(nf)[:-1]]).astype(np.int64)
    fps = np.array([m["fps"] for m in ms], np.float32)
    # motion_lib.py:376-379: curr_len = 1/fps * (num_frames-1) (python float) -> float32
    lengths = np.array([1.0 / m["fps"] * (m["num_frames"] - 1) for m in ms], np.float32)
    dts = np.array([1.0 / m["fps"] for m in ms], np.float32)
    cat = lambda k: np.ascontiguousarray(np.concatenate([m[k] for m in ms], axis=0), np.float32)  # noqa: E731
    return MotionTables(gts=cat("gts"), grs=cat("grs"), lrs=cat("lrs"), gvs=cat("gvs"),
                        gavs=cat("gavs"), dvs=cat("dvs"), num_frames=nf, length_starts=starts,
                        lengths=lengths, dt=dts, fps=fps)


def tables_from_arrays(d: dict) -> MotionTables:
    return MotionTables(**{k: np.asarray(d[k]) for k in MotionTables.__dataclass_fields__})


def load_motion_file(motion_file) -> Dict[str, dict]:
    """Clip dictionary from a joblib ``.pkl`` file / a directory of them / an in-memory dict
    (``MotionLibBase.load_data``, ``motion_lib.py:192-231``). Files are the user's own data."""
    if isinstance(motion_file, dict):
        return motion_file
    import joblib
    if osp.isfile(motion_file):
        return joblib.load(motion_file)
    files = sorted(f for f in os.listdir(motion_file) if f.endswith(".pkl"))
    out = {}
    for f in files:
        key = f.split(".")[0]
        out[key] = joblib.load(osp.join(motion_file, f))[key]
    return out


class MotionLibSMPL:
    """Host-side motion library with the reference's sampling API (``motion_lib.py:180-547``).

    Device-side sampling lives in the engine; :meth:`upload` hands the tables to it.
    """

    def __init__(self, motion_file, model: HumanoidModel, device="cuda:0", min_length=-1,
                 im_eval=False, is_deterministic=False, seed: Optional[int] = None):
        import torch
        self._device = device
        self.model = model
        data = load_motion_file(motion_file)
        if min_length != -1:
            data = {k: v for k, v in data.items() if len(v["pose_quat_global"]) >= min_length}
        elif im_eval:
            data = dict(sorted(data.items(), key=lambda kv: len(kv[1]["pose_quat_global"]), reverse=True))
        self._motion_data_keys = np.array(list(data.keys()))
        self._motion_data_list = list(data.values())
        self._num_unique_motions = len(self._motion_data_list)
        self.is_deterministic = is_deterministic
        n = self._num_unique_motions
        self._termination_history = torch.zeros(n, device=device)
        self._success_rate = torch.zeros(n, device=device)
        self._sampling_history = torch.zeros(n, device=device)
        self._sampling_prob = torch.ones(n, device=device) / n
        self._curr_motion_ids = None
        self.tables: Optional[MotionTables] = None
        self._gen = None if seed is None else torch.Generator(device=device).manual_seed(seed)

    # -- loading (motion_lib.py:257-429) -------------------------------------------------
    def select_motions(self, num_motion_to_load: int, random_sample=True, start_idx=0, sample_idxes=None):
        """Motion sampling of ``load_motions`` (motion_lib.py:305-345) without building tables:
        returns (unique clip dicts, per-motion index into them) and sets the per-motion metadata."""
        import torch
        if sample_idxes is None or len(sample_idxes) != num_motion_to_load:
            if not self.is_deterministic and random_sample:
                sample_idxes = torch.multinomial(self._sampling_prob, num_samples=num_motion_to_load,
                                                 replacement=True, generator=self._gen)
            else:
                sample_idxes = torch.remainder(torch.arange(num_motion_to_load) + start_idx,
                                               self._num_unique_motions)
        sample_idxes = torch.as_tensor(sample_idxes).to(self._device)
        self._curr_motion_ids = sample_idxes
        self.curr_motion_keys = self._motion_data_keys[sample_idxes.cpu().numpy()]
        idx = sample_idxes.cpu().numpy()
        uniq, inv = np.unique(idx, return_inverse=True)
        clips = [self._motion_data_list[i] for i in uniq]
        nf = np.array([len(c["pose_quat_global"]) for c in clips], np.int64)[inv]
        fps = np.array([int(c.get("fps", 30)) for c in clips], np.int64)[inv]
        # motion_lib.py:376-379 (python floats -> float32)
        lengths = np.array([1.0 / int(f) * (int(k) - 1) for f, k in zip(fps, nf)], np.float32)
        self._motion_lengths = torch.as_tensor(lengths, device=self._device)
        self._motion_num_frames = torch.as_tensor(nf, device=self._device)
        self._motion_fps = torch.as_tensor(fps.astype(np.float32), device=self._device)
        self._motion_dt = torch.as_tensor(np.array([1.0 / int(f) for f in fps], np.float32), device=self._device)
        self._num_loaded = int(num_motion_to_load)
        return clips, inv.astype(np.int32)

    def load_motions(self, num_motion_to_load: int, random_sample=True, start_idx=0,
                     sample_idxes=None) -> MotionTables:
        """Host ingestion (the checker for the engine's he_ingest_clips): sample + build tables."""
        clips, inv = self.select_motions(num_motion_to_load, random_sample, start_idx, sample_idxes)
        # unique clips are ingested once and shared by all envs that sampled them
        base = build_tables(self.model, clips)
        # per-env motion entries point into the unique-clip tables (same values as the
        # reference's per-env copies, ``motion_lib.py:407-419``, without duplicating frames)
        self.tables = MotionTables(
            gts=base.gts, grs=base.grs, lrs=base.lrs, gvs=base.gvs, gavs=base.gavs, dvs=base.dvs,
            num_frames=base.num_frames[inv], length_starts=base.length_starts[inv],
            lengths=base.lengths[inv], dt=base.dt[inv], fps=base.fps[inv])
        return self.tables

    def num_motions(self) -> int:
        return self._num_loaded

    def get_total_length(self) -> float:
        return float(self._motion_lengths.sum())

    # -- sampling weights (motion_lib.py:454-500) -----------------------------------------
    def update_hard_sampling_weight(self, failed_keys):
        import torch
        if len(failed_keys) > 0:
            keys = self._motion_data_keys.tolist()
            idx = [keys.index(k) for k in failed_keys]
            self._sampling_prob[:] = 0
            self._sampling_prob[idx] = 1 / len(idx)
        else:
            self._sampling_prob = torch.ones(self._num_unique_motions, device=self._device) / self._num_unique_motions

    def update_soft_sampling_weight(self, failed_keys):
        import torch
        if len(failed_keys) > 0:
            keys = self._motion_data_keys.tolist()
            idx = [keys.index(k) for k in failed_keys]
            self._termination_history[idx] += 1
            self.update_sampling_prob(self._termination_history)
        else:
            self._sampling_prob = torch.ones(self._num_unique_motions, device=self._device) / self._num_unique_motions

    def update_sampling_prob(self, termination_history):
        if len(termination_history) == len(self._termination_history) and termination_history.sum() > 0:
            self._sampling_prob[:] = termination_history / termination_history.sum()
            self._termination_history = termination_history
            return True
        return False

    # -- time sampling (motion_lib.py:515-547) ---------------------------------------------
    def sample_time_interval(self, motion_ids, phase=None):
        import torch
        if phase is None:
            phase = torch.rand(motion_ids.shape, device=self._device, generator=self._gen)
        motion_len = self._motion_lengths[motion_ids]
        curr_fps = 1 / 30
        return ((phase * motion_len) / curr_fps).long() * curr_fps

    def get_motion_length(self, motion_ids=None):
        return self._motion_lengths if motion_ids is None else self._motion_lengths[motion_ids]

    def get_motion_num_steps(self, motion_ids=None, sim_fps=30.0):
        nf = self._motion_num_frames if motion_ids is None else self._motion_num_frames[motion_ids]
        fps = self._motion_fps if motion_ids is None else self._motion_fps[motion_ids]
        return (nf * sim_fps / fps).ceil().int()
