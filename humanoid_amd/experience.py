"""Rollout -> trainer handoff on the device.

Mirrors puffer_phc/clean_pufferl/structs.py ``Experience`` (same constructor, ``store``,
``sort_training_data``, ``flatten_batch``, ``full``; the ``b_*`` minibatch tensors the PPO loop
reads, core.py:289-296) and the Cython ``compute_gae`` (c_gae.pyx:11-32), with every buffer resident
on the GPU and the work done by the HIP kernels behind include/humanoid_rollout.h:

  reference (host)                                          here (device)
  store: 6 ``.cpu().numpy()`` copies + Python key list      he_rollout_store (row copies + keys)
  sort_training_data: ``sorted`` over (env_id, step)        he_rollout_order (counting sort)
  flatten_batch: host gathers + H2D                         he_rollout_gather (one launch, all fields)
  compute_gae on the host + layout (core.py:213-258)        he_gae_minibatch (fused, into b_* layout)

The only host synchronisations left are the ones the reference's own control flow needs: the
stored-row count when a mask is given (the reference's ``mask.sum().item()``, core.py:136) and the
error check once per batch in ``sort_training_data``. There is no CPU path: without the engine
library or a GPU these classes raise.
"""
import ctypes as C
from typing import Optional

import numpy as np

from . import _abi
from .engine import EngineError, _check, load_library

__all__ = ["Experience", "compute_gae"]


def _stream(device):
    import torch
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _f32(t, device, shape=None):
    """Device float32 contiguous view/copy of ``t`` (tensor or array)."""
    import torch
    if isinstance(t, torch.Tensor) and t.device == device and t.is_contiguous():  # the hot path: no copy
        if t.dtype == torch.bool:
            t = t.view(torch.uint8)
        if t.dtype in (torch.float32, torch.uint8):
            return t.view(shape) if shape is not None else t
    x = torch.as_tensor(t)
    if x.dtype == torch.bool:
        x = x.to(torch.uint8)
    if x.dtype not in (torch.float32, torch.uint8):
        x = x.to(torch.float32)
    x = x.to(device, non_blocking=True).contiguous()
    return x.reshape(shape) if shape is not None else x


def _field(src, dst, width):
    import torch
    kind = _abi.ROLLOUT_U8 if src.dtype == torch.uint8 else _abi.ROLLOUT_F32
    return _abi.HeRolloutField(src.data_ptr(), dst.data_ptr(), int(width), kind)


def _fields(pairs):
    arr = (_abi.HeRolloutField * _abi.ROLLOUT_MAX_FIELDS)()
    for i, f in enumerate(pairs):
        arr[i] = f
    return arr, len(pairs)


def compute_gae(dones, values, rewards, gamma: float, gae_lambda: float):
    """c_gae.pyx:11-32 ``compute_gae`` on the GPU, same float32 results.

    Device tensors in -> device tensor out. NumPy arrays in (the Cython signature) -> they are moved
    to ``cuda`` and the advantages come back as a NumPy float32 array."""
    import torch
    lib = load_library()
    host = isinstance(values, np.ndarray)
    dev = torch.device("cuda", torch.cuda.current_device()) if host else torch.as_tensor(values).device
    if dev.type != "cuda":
        raise EngineError("compute_gae: inputs must be CUDA tensors or NumPy arrays (no CPU path)")
    d = _f32(dones, dev).to(torch.float32).reshape(-1)
    v = _f32(values, dev).reshape(-1)
    r = _f32(rewards, dev).reshape(-1)
    n = r.numel()
    if d.numel() != n or v.numel() != n:
        raise EngineError("compute_gae: dones, values and rewards must have the same length")
    adv = torch.empty(n, dtype=torch.float32, device=dev)
    _check(lib.he_gae(d.data_ptr(), v.data_ptr(), r.data_ptr(), n, float(gamma), float(gae_lambda), adv.data_ptr(),
                      _stream(dev)))
    return adv.cpu().numpy() if host else adv


class Experience:
    """structs.py:22-179 ``Experience`` with device-resident storage (``cpu_offload`` is accepted and
    ignored: nothing is staged through host memory)."""

    def __init__(self, batch_size, bptt_horizon, minibatch_size, num_minibatches, minibatch_rows, obs_shape,
                 obs_dtype, atn_shape, atn_dtype, cpu_offload, device, lstm, lstm_total_agents, use_amp_obs,
                 amp_obs_size=1960, amp_obs_update_prob=0.01):
        import torch
        self.lib = load_library()
        if minibatch_size is None:
            minibatch_size = batch_size
        dev = torch.device(device)
        if dev.type != "cuda":
            raise EngineError("Experience: device must be a CUDA (ROCm) device; there is no CPU path")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        if num_minibatches * minibatch_rows * bptt_horizon != batch_size:
            raise EngineError("Experience: batch_size != num_minibatches * minibatch_rows * bptt_horizon")
        self.device = dev
        obs_shape = tuple(obs_shape)
        atn_shape = tuple(atn_shape)
        for name, dt in (("obs_dtype", obs_dtype), ("atn_dtype", atn_dtype)):
            if np.dtype(dt) != np.float32:
                raise EngineError(f"Experience: {name} must be float32 (the PHC env's)")
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)  # noqa: E731
        self.obs = z(batch_size, *obs_shape)
        self.actions = z(batch_size, *atn_shape)
        self.logprobs = z(batch_size)
        self.rewards = z(batch_size)
        self.dones = z(batch_size)
        self.truncateds = z(batch_size)
        self.values = z(batch_size)
        self.obs_width = int(np.prod(obs_shape))
        self.atn_width = int(np.prod(atn_shape))
        self.obs_shape, self.atn_shape = obs_shape, atn_shape

        self.lstm_h = self.lstm_c = None
        if lstm is not None:
            assert lstm_total_agents > 0
            shape = (lstm.num_layers, lstm_total_agents, lstm.hidden_size)
            self.lstm_h = torch.zeros(shape, device=dev)
            self.lstm_c = torch.zeros(shape, device=dev)

        self.num_minibatches = num_minibatches
        self.minibatch_rows = minibatch_rows
        self.batch_size = batch_size
        self.bptt_horizon = bptt_horizon
        self.minibatch_size = minibatch_size
        self.ptr = 0
        self.step = 0

        self.use_amp_obs = use_amp_obs
        if use_amp_obs:
            self.amp_obs = z(batch_size, amp_obs_size)
            self.amp_obs_replay = z(batch_size, amp_obs_size)
            self.amp_obs_replay_filled = False
            self.amp_obs_update_prob = amp_obs_update_prob
            self.amp_obs_size = amp_obs_size

        # sort-key bookkeeping (structs.py:121 sort_keys): per-env counters, per-row (env, rank)
        self.num_keys = max(int(lstm_total_agents or 0), 1)
        self._scratch_rows = 0
        self._alloc_index(self.num_keys, 1 << 12)
        self._last_env_ids = None
        self._idxs = torch.empty(batch_size, dtype=torch.int64, device=dev)
        self._b = None

    # ------------------------------------------------------------------ bookkeeping buffers
    def _alloc_index(self, num_keys, scratch_rows):
        """(Re)allocate the per-env counters (only between collections) and/or grow the scratch."""
        import torch
        dev = self.device
        i32 = dict(dtype=torch.int32, device=dev)
        if num_keys != getattr(self, "num_keys_alloc", None):
            self.num_keys = self.num_keys_alloc = int(num_keys)
            self._key_count = torch.zeros(self.num_keys, **i32)
            self._key_last = torch.full((self.num_keys,), -1, **i32)
            self._key_offset = torch.zeros(self.num_keys, **i32)
        if not hasattr(self, "_row_env"):
            self._row_env = torch.zeros(self.batch_size, **i32)
            self._row_rank = torch.zeros(self.batch_size, **i32)
            self._status = torch.zeros(4, **i32)
        if scratch_rows > self._scratch_rows:
            self._scratch = torch.zeros(scratch_rows, **i32)
            self._scratch_rows = scratch_rows
        self._ix = _abi.HeRolloutIndex(self.num_keys, 0, self.batch_size, self._scratch_rows,
                                       self._key_count.data_ptr(), self._key_last.data_ptr(),
                                       self._key_offset.data_ptr(), self._row_env.data_ptr(),
                                       self._row_rank.data_ptr(), self._scratch.data_ptr(), self._status.data_ptr())

    def _env_id_tensor(self, env_id, rows):
        import torch
        if isinstance(env_id, torch.Tensor) and env_id.device == self.device and env_id.dtype == torch.int32:
            ids = env_id.contiguous()
        else:
            if self._last_env_ids is not None and env_id is self._last_env_ids[0]:
                return self._last_env_ids[1]
            ids = torch.as_tensor(np.asarray(env_id, dtype=np.int32)).to(self.device)
            self._last_env_ids = (env_id, ids)
        if ids.numel() != rows:
            raise EngineError("store: env_id must have one entry per row")
        return ids

    @property
    def full(self):
        return self.ptr >= self.batch_size

    def store(self, obs, amp_obs, value, action, logprob, reward, done, trunc, env_id, mask=None):
        """structs.py:108-126. Rows with ``mask`` set (None: all rows) go to the next free flat rows, in
        order, up to ``batch_size``; their (env_id, step) key is recorded for sort_training_data."""
        import torch
        rows = int(torch.as_tensor(value).numel())
        if env_id is not None and not isinstance(env_id, torch.Tensor):
            kmax = int(np.max(env_id)) + 1 if len(env_id) else 0
        else:
            kmax = 0
        if kmax > self.num_keys:  # env ids beyond lstm_total_agents: grow the per-env counters
            if self.ptr:
                raise EngineError("store: env ids grew in the middle of a collection")
            self._alloc_index(kmax, self._scratch_rows)
        if rows > self._scratch_rows:
            self._alloc_index(self.num_keys, rows)
        ids = self._env_id_tensor(env_id, rows)
        dev = self.device
        f = [_field(_f32(obs, dev, (rows, self.obs_width)), self.obs, self.obs_width),
             _field(_f32(value, dev, (rows,)), self.values, 1),
             _field(_f32(action, dev, (rows, self.atn_width)), self.actions, self.atn_width),
             _field(_f32(logprob, dev, (rows,)), self.logprobs, 1),
             _field(_f32(reward, dev, (rows,)), self.rewards, 1),
             _field(_f32(done, dev, (rows,)), self.dones, 1),
             _field(_f32(trunc, dev, (rows,)), self.truncateds, 1)]
        keep = [f]  # the temporaries must outlive the launch: held until the next store
        if self.use_amp_obs:
            a = _f32(amp_obs, dev, (rows, self.amp_obs_size))
            f.append(_field(a, self.amp_obs, self.amp_obs_size))
            keep.append(a)
        m = None
        if mask is not None:
            m = torch.as_tensor(mask).to(dev, non_blocking=True).to(torch.uint8).contiguous()
            if m.numel() != rows:
                raise EngineError("store: mask must have one entry per row")
        arr, nf = _fields(f)
        self._keep = (keep, m, ids)
        _check(self.lib.he_rollout_store(C.byref(self._ix), arr, nf, rows, ids.data_ptr(),
                                         None if m is None else m.data_ptr(), self.ptr, self.step, _stream(dev)))
        if m is None:
            stored = min(rows, self.batch_size - self.ptr)
        else:
            stored = int(self._status[0].item())  # the reference's mask.sum().item() (core.py:136)
        self.ptr += stored
        self.step += 1

    def sort_training_data(self):
        """structs.py:128-142: rows ordered by (env_id, step); returns the device index tensor."""
        import torch
        n = self.ptr
        if n != self.batch_size:
            raise EngineError(f"sort_training_data: batch not full ({n} of {self.batch_size} rows)")
        _check(self.lib.he_rollout_order(C.byref(self._ix), n, self._idxs.data_ptr(), 1, _stream(self.device)))
        idxs = self._idxs
        self.b_idxs_obs = idxs.reshape(self.minibatch_rows, self.num_minibatches, self.bptt_horizon).transpose(1, 0)
        self.b_idxs = self.b_idxs_obs
        self.b_idxs_flat = self.b_idxs.reshape(self.num_minibatches, self.minibatch_size)
        return idxs

    def _minibatch_buffers(self):
        import torch
        if self._b is None:
            nm, rows, bp = self.num_minibatches, self.minibatch_rows, self.bptt_horizon
            z = lambda *s: torch.empty(*s, dtype=torch.float32, device=self.device)  # noqa: E731
            b = dict(obs=z(nm, rows, bp, *self.obs_shape), actions=z(nm, rows, bp, *self.atn_shape),
                     logprobs=z(nm, rows, bp), dones=z(nm, rows, bp), truncated=z(nm, rows, bp),
                     values=z(nm, self.minibatch_size), advantages=z(nm, self.minibatch_size),
                     returns=z(nm, self.minibatch_size))
            if self.use_amp_obs:
                b["amp_obs"] = z(nm, self.minibatch_size, self.amp_obs_size)
            self._b = b
        return self._b

    def flatten_batch(self):
        """structs.py:144-179: every b_* tensor in the [num_minibatches, rows, bptt] order, one launch."""
        import torch
        b = self._minibatch_buffers()
        pairs = [(self.obs, b["obs"], self.obs_width), (self.actions, b["actions"], self.atn_width),
                 (self.logprobs, b["logprobs"], 1), (self.dones, b["dones"], 1),
                 (self.truncateds, b["truncated"], 1), (self.values, b["values"], 1)]
        if self.use_amp_obs:
            pairs.append((self.amp_obs, b["amp_obs"], self.amp_obs_size))
        arr, nf = _fields([_field(s, d, w) for s, d, w in pairs])
        _check(self.lib.he_rollout_gather(arr, nf, self._idxs.data_ptr(), self.batch_size, self.num_minibatches,
                                          self.minibatch_rows, self.bptt_horizon, _stream(self.device)))
        self.b_obs, self.b_actions, self.b_logprobs = b["obs"], b["actions"], b["logprobs"]
        self.b_dones, self.b_truncated, self.b_values = b["dones"], b["truncated"], b["values"]
        if self.use_amp_obs:  # the replay refresh, as structs.py:164-179 (torch RNG on the device)
            self.b_amp_obs = b["amp_obs"]
            if not self.amp_obs_replay_filled:
                self.amp_obs_replay[:] = self.amp_obs[:]
                self.amp_obs_replay_filled = True
            else:
                upd = torch.rand(self.batch_size, device=self.device) < self.amp_obs_update_prob
                self.amp_obs_replay[upd] = self.amp_obs[upd]
            rep = torch.randperm(self.batch_size, device=self.device).reshape(self.num_minibatches,
                                                                               self.minibatch_size)
            self.b_amp_obs_replay = self.amp_obs_replay[rep]

    def compute_advantages(self, gamma: float, gae_lambda: float, extra_reward=None):
        """core.py:213-260 after sort + flatten: GAE over the sorted rows (+ ``extra_reward``, the
        adversarial reward, per sorted position) straight into ``b_advantages`` / ``b_returns``;
        ``returns`` is the reference's ``returns_np`` (sorted advantages + storage-order values)."""
        import torch
        b = self._minibatch_buffers()
        ex = None
        if extra_reward is not None:
            ex = _f32(extra_reward, self.device, (self.batch_size,))
        _check(self.lib.he_gae_minibatch(self.dones.data_ptr(), self.values.data_ptr(), self.rewards.data_ptr(),
                                         None if ex is None else ex.data_ptr(), self._idxs.data_ptr(),
                                         self.batch_size, float(gamma), float(gae_lambda), self.num_minibatches,
                                         self.minibatch_rows, self.bptt_horizon, b["advantages"].data_ptr(),
                                         b["returns"].data_ptr(), _stream(self.device)))
        self._keep_extra = ex
        self.b_advantages, self.b_returns = b["advantages"], b["returns"]
        adv_sorted = self.b_advantages.reshape(self.num_minibatches, self.minibatch_rows, self.bptt_horizon)
        adv_sorted = adv_sorted.transpose(0, 1).reshape(-1)
        self.advantages = adv_sorted
        self.returns = adv_sorted + self.values
        return self.b_advantages

    def explained_variance(self):
        """core.py:413-417 on the device (y_pred = values, y_true = returns, storage order)."""
        import torch
        var_y = torch.var(self.returns, unbiased=False)
        ev = 1 - torch.var(self.returns - self.values, unbiased=False) / var_y
        return float("nan") if float(var_y) == 0 else float(ev)

    def reset_collection(self):
        """core.py:200-202 (ptr = step = 0 after a collection)."""
        self.ptr = 0
        self.step = 0
