"""ctypes shim over ``libhumanoid_engine.so`` (``include/humanoid_engine.h``).

This replaces ``gymtorch`` (``packages/gymtorch/gymtorch/gymtorch.cpp:33-158``, ``wrapper.py:11-56``)
and the Isaac Gym tensor API: engine-owned device buffers are exposed as zero-copy, non-owning
torch tensors (``__cuda_array_interface__``, DLPack fallback) and every compute call is enqueued on
torch's current stream. Errors raise :class:`EngineError` (gymtorch printed and returned an empty
tensor, ``gymtorch.cpp:40-51``). There is no CPU fallback: without the HIP library or a GPU the
constructor raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

from . import _abi

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhumanoid_engine.so")
_lib = None


class EngineError(RuntimeError):
    pass


HE_SYMBOLS = (
    "he_last_error", "he_version", "he_device_count", "he_create", "he_set_model", "he_create_envs", "he_destroy",
    "he_get_buffer", "he_set_dof_targets", "he_set_root_state_indexed", "he_set_dof_state_indexed",
    "he_set_dof_targets_indexed", "he_set_env_properties", "he_simulate", "he_set_pd_params", "he_step_actions",
    "he_refresh", "he_load_motions", "he_imitation_step", "he_motion_state", "he_reset_envs", "he_env_step",
    "he_imitation_reset_step", "he_set_debug_stamps", "he_hash_uniform", "he_ingest_clips", "he_set_eval",
    "he_set_amp", "he_amp_observations", "he_set_fused_step",
    # include/humanoid_rollout.h
    "he_rollout_store", "he_rollout_order", "he_rollout_gather", "he_gae", "he_gae_minibatch", "he_episode_step",
)


def load_library(path: Optional[str] = None):
    """Load (never build) the HIP engine library; raise loudly when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    # HE_ENGINE_LIB: diagnostics only (A/B timing of a variant build, tools/build_variant.py)
    p = path or os.environ.get("HE_ENGINE_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise EngineError(f"{p} not found: build it with `python -m humanoid_amd.build` (hipcc, gfx950)")
    lib = C.CDLL(p)
    V, I, F = C.c_void_p, C.c_int, C.c_float
    lib.he_last_error.restype = C.c_char_p
    lib.he_hash_uniform.restype = F
    lib.he_hash_uniform.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32]
    sigs = {
        "he_create": [V, I, V], "he_set_model": [V, V], "he_create_envs": [V, I, V], "he_destroy": [V],
        "he_get_buffer": [V, I, V, V, V, V], "he_set_dof_targets": [V, V, V],
        "he_set_root_state_indexed": [V, V, V, I, V], "he_set_dof_state_indexed": [V, V, V, I, V],
        "he_set_dof_targets_indexed": [V, V, V, I, V], "he_set_env_properties": [V, V, V, V],
        "he_simulate": [V, I, V], "he_set_pd_params": [V, V, V, V, I], "he_step_actions": [V, V, I, V],
        "he_refresh": [V, V],
        "he_load_motions": [V, C.c_int64, I, V, V, V, V, V, V, V, V, V, V],
        "he_ingest_clips": [V, I, V, V, V, V, I, V, V],
        "he_imitation_step": [V, V, V, V, V, V, V, V, V],
        "he_motion_state": [V, I, V, V, V, V, V, V, V, V, V, V],
        "he_reset_envs": [V, V, V, V, I, V, V, V, V, V],
        "he_env_step": [V, V, V, V, I, C.c_uint64, C.c_uint64, V, V, V, V, V, V],
        "he_imitation_reset_step": [V, V, V, C.c_uint64, C.c_uint64, V, V, V, V, V, V],
        "he_device_count": [V],
        "he_set_debug_stamps": [V, V],
        "he_set_eval": [V, V],
        "he_set_amp": [V, V],
        "he_set_fused_step": [V, I],
        "he_amp_observations": [I, V, V, V, V, V, V, V, V, V],
        "he_rollout_store": [V, V, I, C.c_int64, V, V, C.c_int64, C.c_int32, V],
        "he_rollout_order": [V, C.c_int64, V, I, V],
        "he_rollout_gather": [V, I, V, C.c_int64, C.c_int32, C.c_int32, C.c_int32, V],
        "he_gae": [V, V, V, C.c_int64, F, F, V, V],
        "he_gae_minibatch": [V, V, V, V, V, C.c_int64, F, F, C.c_int32, C.c_int32, C.c_int32, V, V, V],
        "he_episode_step": [C.c_int32] + [V] * 14,
    }
    for name, args in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = I
    _lib = lib
    return lib


def _check(rc):
    if rc != 0:
        raise EngineError(_lib.he_last_error().decode())


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


class _CudaArray:
    """Minimal ``__cuda_array_interface__`` holder for a non-owning device view."""

    def __init__(self, ptr, shape, typestr, owner):
        self._owner = owner  # keep the engine alive while the view exists
        self.__cuda_array_interface__ = {"data": (int(ptr), False), "shape": tuple(int(s) for s in shape),
                                         "typestr": typestr, "strides": None, "version": 3}


def wrap_device_pointer(ptr: int, shape, dtype, device_index: int, owner=None):
    """Zero-copy torch view of engine memory (gymtorch.wrap_tensor equivalent)."""
    import torch
    typestr = {torch.float32: "<f4", torch.int32: "<i4", torch.int64: "<i8", torch.int16: "<i2", torch.uint8: "|u1"}[dtype]
    t = torch.as_tensor(_CudaArray(ptr, shape, typestr, owner), device=f"cuda:{device_index}")
    if t.data_ptr() != ptr:
        raise EngineError("zero-copy wrap produced a copy")
    return t


class Engine:
    """One engine instance = one simulation of ``num_envs`` humanoids on one GPU."""

    def __init__(self, model, num_envs: int, device: int = 0, sim_params: Optional[_abi.HeSimParams] = None,
                 start_xy: Optional[np.ndarray] = None):
        import torch
        self.lib = load_library()
        if not torch.cuda.is_available():
            raise EngineError("no HIP device visible: the engine has no CPU path")
        self.device_index = int(device)
        self.device = torch.device("cuda", self.device_index)
        self.params = sim_params if sim_params is not None else _abi.default_sim_params()
        self.he_model = model if isinstance(model, _abi.HeModel) else _abi.make_model(model)
        torch.cuda.set_device(self.device)
        torch.zeros(1, device=self.device)  # make sure torch's context exists on this device
        h = C.c_void_p()
        _check(self.lib.he_create(C.byref(self.params), self.device_index, C.byref(h)))
        self.h = h
        _check(self.lib.he_set_model(self.h, C.byref(self.he_model)))
        xy = None
        if start_xy is not None:
            xy = np.ascontiguousarray(start_xy, np.float32).reshape(num_envs, 2)
        _check(self.lib.he_create_envs(self.h, int(num_envs), None if xy is None else xy.ctypes.data_as(C.c_void_p)))
        self.num_envs = int(num_envs)
        self._views = {}
        self.has_motions = False

    def __del__(self):
        try:
            if getattr(self, "h", None) and self.lib is not None:
                self.lib.he_destroy(self.h)
                self.h = None
        except Exception:
            pass

    @property
    def stream(self):
        import torch
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------------ buffers (acquire_*)
    def buffer(self, kind: int):
        import torch
        if kind in self._views:
            return self._views[kind]
        ptr = C.c_void_p()
        shape = (C.c_int64 * 8)()
        ndim = C.c_int()
        dtype = C.c_int()
        _check(self.lib.he_get_buffer(self.h, kind, C.byref(ptr), shape, C.byref(ndim), C.byref(dtype)))
        tdt = torch.float32 if dtype.value == _abi.DTYPE_F32 else torch.int32
        t = wrap_device_pointer(ptr.value, [shape[i] for i in range(ndim.value)], tdt, self.device_index, owner=self)
        self._views[kind] = t
        return t

    @property
    def root_states(self):
        return self.buffer(_abi.BUF_ROOT_STATE)

    @property
    def dof_state(self):
        return self.buffer(_abi.BUF_DOF_STATE)

    @property
    def rb_state(self):
        return self.buffer(_abi.BUF_RB_STATE)

    @property
    def contact_forces(self):
        return self.buffer(_abi.BUF_CONTACT_FORCE)

    @property
    def dof_force(self):
        return self.buffer(_abi.BUF_DOF_FORCE)

    @property
    def dof_targets(self):
        return self.buffer(_abi.BUF_DOF_TARGET)

    @property
    def num_contacts(self):
        """i32 [N]: contact slots (joint limits included) used by the last substep."""
        return self.buffer(_abi.BUF_NUM_CONTACTS)

    @property
    def dropped_contacts(self):
        """i32 [N]: contacts generated past the capacity in the last substep (the deepest kept)."""
        return self.buffer(_abi.BUF_DROPPED_CONTACTS)

    @property
    def contact_cache(self):
        """f32 [N, HE_CACHE_WORDS]: the solver's warm-start cache (signature, keys, impulses)."""
        return self.buffer(_abi.BUF_CONTACT_CACHE)

    @property
    def initial_root_states(self):
        """f32 [N,13]: _initial_humanoid_root_states (humanoid_phc.py:522-523), the root state the
        Default / Hybrid state init resets to; writable."""
        return self.buffer(_abi.BUF_INIT_ROOT_STATE)

    @property
    def physics_order(self):
        """i32 [N]: the physics launch's dispatch order (the env of each workgroup, expensive envs
        first; diagnostics, DESIGN §4.1 "Dispatch order"). A copy: the engine's own buffer is read
        by every physics launch and must not be written from outside."""
        return self.buffer(_abi.BUF_PHYS_ORDER).clone()

    @property
    def physics_cost(self):
        """i32 [N]: each env's wave cycles in the last physics launch (the order's input; a copy)."""
        return self.buffer(_abi.BUF_PHYS_COST).clone()

    # ------------------------------------------------------------------ state writes
    def _contig(self, t, dtype=None):
        import torch
        if t.device != self.device:
            raise EngineError(f"tensor on {t.device}, engine on {self.device}")
        if dtype is not None and t.dtype != dtype:
            raise EngineError(f"expected {dtype}, got {t.dtype}")
        if not t.is_contiguous():
            raise EngineError("Input tensor must be contiguous")  # wrapper.py:47-49
        return t

    def set_dof_targets(self, t):
        import torch
        t = self._contig(t, torch.float32)
        if t.numel() != self.num_envs * _abi.ND:
            raise EngineError("dof target tensor must hold num_envs*69 floats")
        _check(self.lib.he_set_dof_targets(self.h, C.c_void_p(t.data_ptr()), self.stream))

    def _indexed(self, fn, src, ids, row):
        import torch
        src = self._contig(src, torch.float32)
        ids = self._contig(ids, torch.int32)
        if src.numel() != self.num_envs * row:
            raise EngineError("indexed writes take the full-size source tensor")
        _check(fn(self.h, C.c_void_p(src.data_ptr()), C.c_void_p(ids.data_ptr()), int(ids.numel()), self.stream))

    def set_root_state_indexed(self, src, ids):
        self._indexed(self.lib.he_set_root_state_indexed, src, ids, 13)

    def set_dof_state_indexed(self, src, ids):
        self._indexed(self.lib.he_set_dof_state_indexed, src, ids, 2 * _abi.ND)

    def set_dof_targets_indexed(self, src, ids):
        self._indexed(self.lib.he_set_dof_targets_indexed, src, ids, _abi.ND)

    def set_env_properties(self, mass_scale=None, friction=None, terrain_kind=None):
        import torch
        self._env_props = (mass_scale, friction, terrain_kind)  # keep alive
        vp = lambda t, dt: None if t is None else C.c_void_p(self._contig(t, dt).data_ptr())  # noqa: E731
        _check(self.lib.he_set_env_properties(self.h, vp(mass_scale, torch.float32), vp(friction, torch.float32),
                                              vp(terrain_kind, torch.int32)))

    # ------------------------------------------------------------------ stepping
    def simulate(self, num_simulate: int = 2):
        """gym.simulate() x num_simulate (control_freq_inv), each he_sim_params.substeps physics steps."""
        _check(self.lib.he_simulate(self.h, int(num_simulate), self.stream))

    def set_pd_params(self, offset, scale, frozen_mask=None, clip_actions=True):
        off = np.ascontiguousarray(offset, np.float32)
        sc = np.ascontiguousarray(scale, np.float32)
        fz = None if frozen_mask is None else np.ascontiguousarray(frozen_mask, np.int32)
        _check(self.lib.he_set_pd_params(self.h, off.ctypes.data_as(C.c_void_p), sc.ctypes.data_as(C.c_void_p),
                                         None if fz is None else fz.ctypes.data_as(C.c_void_p), int(bool(clip_actions))))

    def step_actions(self, actions, num_simulate: int = 2):
        import torch
        a = self._contig(actions, torch.float32)
        _check(self.lib.he_step_actions(self.h, C.c_void_p(a.data_ptr()), int(num_simulate), self.stream))

    # ------------------------------------------------------------------ motion library
    def load_motions(self, tables):
        t = tables
        arrs = [np.ascontiguousarray(x, np.float32) for x in (t.gts, t.grs, t.lrs, t.gvs, t.gavs, t.dvs)]
        starts = np.ascontiguousarray(t.length_starts, np.int64)
        nf = np.ascontiguousarray(t.num_frames, np.int64)
        lens = np.ascontiguousarray(t.lengths, np.float32)
        dts = np.ascontiguousarray(t.dt, np.float32)
        F = arrs[0].shape[0]
        _check(self.lib.he_load_motions(self.h, int(F), int(nf.shape[0]), *[a.ctypes.data_as(C.c_void_p) for a in arrs],
                                        starts.ctypes.data_as(C.c_void_p), nf.ctypes.data_as(C.c_void_p),
                                        lens.ctypes.data_as(C.c_void_p), dts.ctypes.data_as(C.c_void_p)))
        self.has_motions = True

    def ingest_clips(self, clips, motion_clip=None):
        """Device-side motion ingestion (he_ingest_clips): ``clips`` are dicts with the .pkl
        schema's ``pose_quat_global`` [T,24,4] and ``root_trans_offset`` [T,3] (+ ``fps``);
        library motion i uses clip ``motion_clip[i]`` (default: one motion per clip)."""
        import torch
        nf = np.array([len(c["pose_quat_global"]) for c in clips], np.int64)
        fps = np.array([float(c.get("fps", 30)) for c in clips], np.float32)
        pose = torch.as_tensor(np.concatenate([np.asarray(c["pose_quat_global"], np.float32) for c in clips], 0))
        trans = torch.as_tensor(np.concatenate([np.asarray(c["root_trans_offset"], np.float32).reshape(-1, 3)
                                                for c in clips], 0))
        pose = pose.to(self.device).contiguous()
        trans = trans.to(self.device).contiguous()
        if pose.shape[1:] != (24, 4) or trans.shape[0] != pose.shape[0]:
            raise EngineError(f"clip arrays have shapes {tuple(pose.shape)} / {tuple(trans.shape)}")
        mc = None
        m = len(clips)
        if motion_clip is not None:
            mc = np.ascontiguousarray(motion_clip, np.int32)
            m = int(mc.shape[0])
        _check(self.lib.he_ingest_clips(self.h, len(clips), nf.ctypes.data_as(C.c_void_p), fps.ctypes.data_as(C.c_void_p),
                                        C.c_void_p(pose.data_ptr()), C.c_void_p(trans.data_ptr()), m,
                                        None if mc is None else mc.ctypes.data_as(C.c_void_p), self.stream))
        self.has_motions = True

    def motion_state(self, ids, times, offset=None, want_dof=True):
        import torch
        k = int(ids.numel())
        ids = self._contig(ids, torch.int64)
        times = self._contig(times, torch.float32)
        if offset is not None:
            offset = self._contig(offset, torch.float32)
        dev = self.device
        out = dict(rg_pos=torch.empty(k, 24, 3, device=dev), rb_rot=torch.empty(k, 24, 4, device=dev),
                   body_vel=torch.empty(k, 24, 3, device=dev), body_ang_vel=torch.empty(k, 24, 3, device=dev))
        if want_dof:
            out["dof_pos"] = torch.empty(k, 69, device=dev)
            out["dof_vel"] = torch.empty(k, 69, device=dev)
        vp = lambda x: None if x is None else C.c_void_p(x.data_ptr())  # noqa: E731
        _check(self.lib.he_motion_state(self.h, k, vp(ids), vp(times), vp(offset), vp(out["rg_pos"]), vp(out["rb_rot"]),
                                        vp(out["body_vel"]), vp(out["body_ang_vel"]), vp(out.get("dof_pos")),
                                        vp(out.get("dof_vel")), self.stream))
        return out

    def env_motion(self, motion_ids, start_times, start_offsets, global_offset, progress) -> _abi.HeEnvMotion:
        """Per-env motion bookkeeping block; the returned struct keeps the tensors alive."""
        import torch
        n = self.num_envs
        checks = ((motion_ids, torch.int64, (n,)), (start_times, torch.float32, (n,)),
                  (start_offsets, torch.float32, (n,)), (global_offset, torch.float32, (n, 3)),
                  (progress, torch.int16, (n,)))
        for t, dt, shape in checks:
            self._contig(t, dt)
            if tuple(t.shape) != shape:
                raise EngineError(f"env motion buffer has shape {tuple(t.shape)}, expected {shape}")
        em = _abi.HeEnvMotion(motion_ids.data_ptr(), start_times.data_ptr(), start_offsets.data_ptr(),
                              global_offset.data_ptr(), progress.data_ptr())
        em.keep_alive = (motion_ids, start_times, start_offsets, global_offset, progress)
        return em

    def imitation_step(self, params: _abi.HeImitationParams, em: _abi.HeEnvMotion, obs, rew, reward_raw, reset,
                       terminate):
        _check(self.lib.he_imitation_step(self.h, C.byref(params), C.byref(em), C.c_void_p(obs.data_ptr()),
                                          C.c_void_p(rew.data_ptr()), C.c_void_p(reward_raw.data_ptr()),
                                          C.c_void_p(reset.data_ptr()), C.c_void_p(terminate.data_ptr()), self.stream))

    def reset_envs(self, params, em, env_ids, phases, obs, reset, terminate):
        import torch
        env_ids = self._contig(env_ids, torch.int32)
        phases = self._contig(phases, torch.float32)
        _check(self.lib.he_reset_envs(self.h, C.byref(params), C.byref(em), C.c_void_p(env_ids.data_ptr()),
                                      int(env_ids.numel()), C.c_void_p(phases.data_ptr()), C.c_void_p(obs.data_ptr()),
                                      C.c_void_p(reset.data_ptr()), C.c_void_p(terminate.data_ptr()), self.stream))

    def env_step(self, params, em, actions, obs, rew, reward_raw, reset, terminate, seed: int, step_index: int,
                 num_simulate: int = 2):
        import torch
        a = self._contig(actions, torch.float32)
        _check(self.lib.he_env_step(self.h, C.byref(params), C.byref(em), C.c_void_p(a.data_ptr()), int(num_simulate),
                                    C.c_uint64(seed), C.c_uint64(step_index), C.c_void_p(obs.data_ptr()),
                                    C.c_void_p(rew.data_ptr()), C.c_void_p(reward_raw.data_ptr()),
                                    C.c_void_p(reset.data_ptr()), C.c_void_p(terminate.data_ptr()), self.stream))

    def set_fused_step(self, enable):
        """he_set_fused_step: env_step as one launch (True / 1), as step_actions + imitation_reset_step
        (False / 0), or None / -1 = auto (the engine default: one launch up to 2048 envs)."""
        mode = -1 if enable is None or (not isinstance(enable, bool) and int(enable) < 0) else int(bool(enable))
        _check(self.lib.he_set_fused_step(self.h, mode))

    def imitation_reset_step(self, params, em, obs, rew, reward_raw, reset, terminate, seed: int, step_index: int):
        _check(self.lib.he_imitation_reset_step(self.h, C.byref(params), C.byref(em), C.c_uint64(seed),
                                                C.c_uint64(step_index), C.c_void_p(obs.data_ptr()),
                                                C.c_void_p(rew.data_ptr()), C.c_void_p(reward_raw.data_ptr()),
                                                C.c_void_p(reset.data_ptr()), C.c_void_p(terminate.data_ptr()),
                                                self.stream))

    def set_eval(self, buffers: Optional[_abi.HeEvalBuffers]):
        """Attach eval recording (he_set_eval; the struct is copied, call again per frame) or detach."""
        _check(self.lib.he_set_eval(self.h, None if buffers is None else C.byref(buffers)))

    def set_amp(self, amp_obs, amp_obs_demo=None):
        """Attach the AMP buffers (he_set_amp): ``amp_obs`` / ``amp_obs_demo`` f32 [N, S, 196]
        device tensors (humanoid_phc.py:600-611), updated by every following imitation launch;
        ``None`` detaches."""
        import torch
        if amp_obs is None:
            self._amp = None
            _check(self.lib.he_set_amp(self.h, None))
            return
        for t in (amp_obs, amp_obs_demo):
            if t is None:
                continue
            self._contig(t, torch.float32)
            if t.dim() != 3 or t.shape[0] != self.num_envs or t.shape[2] != _abi.AMP_OBS_STEP:
                raise EngineError(f"AMP buffer has shape {tuple(t.shape)}, expected [{self.num_envs}, S, 196]")
        if amp_obs_demo is not None and amp_obs_demo.shape != amp_obs.shape:
            raise EngineError("amp_obs_demo must have the shape of amp_obs")
        b = _abi.HeAmpBuffers(amp_obs.data_ptr(), None if amp_obs_demo is None else amp_obs_demo.data_ptr(),
                              int(amp_obs.shape[1]), 0)
        self._amp = (amp_obs, amp_obs_demo)  # keep alive while attached
        _check(self.lib.he_set_amp(self.h, C.byref(b)))

    def set_debug_stamps(self, buf=None):
        """Diagnostics: int64 [num_envs, 32] (HE_STAMP_SLOTS) device tensor receiving per-phase cycles, or None."""
        import torch
        if buf is not None:
            self._contig(buf, torch.int64)
        self._stamps = buf
        _check(self.lib.he_set_debug_stamps(self.h, None if buf is None else C.c_void_p(buf.data_ptr())))

    def hash_uniform(self, seed, step, env):
        return self.lib.he_hash_uniform(seed, step, env)


def amp_observations(root_pos, root_rot, root_vel, root_ang_vel, dof_pos, dof_vel, key_body_pos):
    """build_amp_observations_smpl (envs/common.py:191-267) with the reference's constant flags on
    device tensors (he_amp_observations): key_body_pos [K,4,3] in KEY_BODIES order -> [K,196]."""
    import torch
    lib = load_library()
    k = int(root_pos.shape[0])
    ins = (root_pos, root_rot, root_vel, root_ang_vel, dof_pos, dof_vel, key_body_pos)
    shapes = ((k, 3), (k, 4), (k, 3), (k, 3), (k, 69), (k, 69), (k, 4, 3))
    dev = root_pos.device
    for t, sh in zip(ins, shapes):
        if t.device != dev or t.dtype != torch.float32 or not t.is_contiguous() or tuple(t.shape) != sh:
            raise EngineError(f"he_amp_observations: expected contiguous f32 {sh} on {dev}, got "
                              f"{t.dtype} {tuple(t.shape)} on {t.device}")
    out = torch.empty(k, _abi.AMP_OBS_STEP, device=dev)
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _check(lib.he_amp_observations(k, *[C.c_void_p(t.data_ptr()) for t in ins], C.c_void_p(out.data_ptr()), stream))
    return out
