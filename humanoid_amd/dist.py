"""Multi-GPU plumbing for the rollout engine.

Environments never interact (each env is its own collision group, ``humanoid_phc.py:333-338``),
so the data path has no collective: rank r owns envs [r*N, (r+1)*N) with its own engine, motion
sample and seed (``config.py:173``: seed = 1 + rank). The collectives below belong to the learner
that consumes the rollouts, one process per GPU over ``torch.distributed`` (RCCL over xGMI on the
GPU box, gloo in the CPU tests):

* :func:`allreduce_gradients` -- bucketed average of policy gradients, once per minibatch step
  (16.98 M fp32 params = 67.9 MB for the reference policy; 2 buckets at the default 64 MB, one
  ring all-reduce each -- large buckets suit xGMI's point-to-point links);
* :func:`synced_running_norm_update` -- the obs normaliser update (``running_norm.py:22-34``) fed
  with global batch moments so replicas' normalisers stay identical;
* :func:`all_gather_failed_keys` -- eval/PMCP failed motion keys, so every rank updates the same
  ``_sampling_prob`` (``phc_train.py:185, 230``; ``motion_lib.py:472-492``).
"""
from __future__ import annotations

import os
from typing import Iterable, List, Sequence, Tuple


def env_info() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (1-process defaults)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str | None = None):
    """Initialise the default process group when WORLD_SIZE > 1 (rendezvous from MASTER_ADDR /
    MASTER_PORT; use 127.0.0.1). Returns (rank, world, local_rank)."""
    import torch
    import torch.distributed as dist
    rank, world, local = env_info()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, **kw)
    return rank, world, local


def env_shard(rank: int, num_envs_per_rank: int) -> range:
    """Global env ids owned by ``rank`` (weak scaling: fixed per-rank count)."""
    return range(rank * num_envs_per_rank, (rank + 1) * num_envs_per_rank)


def rank_seed(base_seed: int, rank: int) -> int:
    return base_seed + rank  # config.py:173 (seed 1 + rank with the default base 1)


def _buckets(tensors: Sequence, bucket_bytes: int) -> List[List]:
    out, cur, size = [], [], 0
    for t in tensors:
        nb = t.numel() * t.element_size()
        if cur and size + nb > bucket_bytes:
            out.append(cur)
            cur, size = [], 0
        cur.append(t)
        size += nb
    if cur:
        out.append(cur)
    return out


def allreduce_gradients(params: Iterable, bucket_bytes: int = 64 << 20, average: bool = True, group=None,
                        min_world: int = 2) -> int:
    """Average ``p.grad`` over all ranks, flattened into buckets of ``bucket_bytes`` (per dtype,
    device). Parameters without a gradient are skipped consistently (same on every rank for the
    same model). Groups smaller than ``min_world`` are skipped (``min_world=1`` runs the
    collective on a one-rank group too: the single-GPU rehearsal of the RCCL path). Returns the
    number of all-reduce calls issued."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) < min_world:
        return 0
    world = dist.get_world_size(group)
    grads = [p.grad for p in params if getattr(p, "grad", None) is not None]
    by_kind = {}
    for g in grads:
        by_kind.setdefault((g.dtype, g.device), []).append(g)
    calls = 0
    for kind, gs in by_kind.items():
        for bucket in _buckets(gs, bucket_bytes):
            flat = torch.cat([g.reshape(-1) for g in bucket])
            dist.all_reduce(flat, group=group)
            if average:
                flat.div_(world)
            off = 0
            for g in bucket:
                n = g.numel()
                g.copy_(flat[off:off + n].view_as(g))
                off += n
            calls += 1
    return calls


class GradBuckets:
    """Gradient storage laid out as flat all-reduce buckets (DDP's ``gradient_as_bucket_view``).

    Every trainable parameter's ``.grad`` is made a view into one of a few flat buffers, so the
    all-reduce runs on the buffers in place: no flatten / copy-back around the collective (that copy
    cost 1.3 ms of a 31 ms minibatch step at 16.98 M params, bench ``learner_configs3``). Buckets are
    filled in reverse parameter order, the order backward produces gradients. With ``overlap``, a
    post-accumulate-grad hook counts each bucket's gradients and launches its all-reduce
    asynchronously as soon as the bucket is complete, so the collective of the last layers runs
    under the backward of the first; :meth:`finish` waits and averages. The optimizer must zero
    gradients in place (``zero_grad(set_to_none=False)``), or the views are lost (checked).
    """

    def __init__(self, params, bucket_bytes: int = 16 << 20, overlap: bool = True, group=None, min_world: int = 2):
        import torch
        import torch.distributed as dist
        self.params = [p for p in params if p.requires_grad]
        self.group, self.min_world = group, min_world
        self.active = dist.is_initialized() and dist.get_world_size(group) >= min_world
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.buckets = []  # (flat buffer, [params])
        by_kind = {}
        for p in reversed(self.params):
            by_kind.setdefault((p.dtype, p.device), []).append(p)
        self._bucket_of = {}
        for (dtype, device), ps in by_kind.items():
            for bucket in _buckets(ps, bucket_bytes):
                flat = torch.zeros(sum(p.numel() for p in bucket), dtype=dtype, device=device)
                off = 0
                for p in bucket:
                    n = p.numel()
                    p.grad = flat[off:off + n].view_as(p)
                    self._bucket_of[p] = len(self.buckets)
                    off += n
                self.buckets.append((flat, bucket))
        self._pending = [0] * len(self.buckets)
        self._handles = [None] * len(self.buckets)
        self._next = 0  # the next bucket to launch (index order)
        self.calls = 0
        self.overlap = bool(overlap) and self.active
        self._hooks = []
        if self.overlap:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._ready))

    def _ready(self, p):
        """A parameter's gradient is final. Buckets are launched in index order only (as DDP does):
        a complete bucket waits for every bucket before it, so all ranks issue their collectives in
        the same order even when some parameter gets no gradient on some ranks (its bucket is then
        launched by :meth:`finish`, after every earlier one). Contract: one ``backward()`` per
        :meth:`finish` -- a second backward (gradient accumulation) would add into a buffer whose
        all-reduce is in flight, and raises here instead."""
        import torch.distributed as dist
        b = self._bucket_of[p]
        if self._handles[b] is not None or self._pending[b] >= len(self.buckets[b][1]):
            raise RuntimeError("GradBuckets: a gradient arrived for a bucket already complete or in flight "
                               "(one backward() per finish(); no gradient accumulation across backward calls)")
        self._pending[b] += 1
        while self._next < len(self.buckets) and self._pending[self._next] == len(self.buckets[self._next][1]):
            self._handles[self._next] = dist.all_reduce(self.buckets[self._next][0], group=self.group, async_op=True)
            self.calls += 1
            self._next += 1

    def check_views(self):
        for flat, ps in self.buckets:
            base = flat.data_ptr()
            end = base + flat.numel() * flat.element_size()
            for p in ps:
                if p.grad is None or not (base <= p.grad.data_ptr() < end):
                    raise RuntimeError("GradBuckets: a .grad is no longer a bucket view "
                                       "(zero gradients with set_to_none=False)")

    def finish(self, average: bool = True) -> int:
        """All-reduce (or wait for the overlapped all-reduces of) every bucket and average; returns
        the number of collectives issued this step."""
        import torch.distributed as dist
        self.check_views()
        if not self.active:
            return 0
        for b, (flat, ps) in enumerate(self.buckets):
            h = self._handles[b]
            if h is None:
                dist.all_reduce(flat, group=self.group)
                self.calls += 1
            else:
                h.wait()
            if average:
                flat.div_(self.world)
        n = self.calls
        self.calls = 0
        self._pending = [0] * len(self.buckets)
        self._handles = [None] * len(self.buckets)
        self._next = 0
        return n

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


def global_batch_moments(x, group=None):
    """Mean and (biased) variance over the concatenation of every rank's ``x`` [B,D] (equal B on
    all ranks): one all-reduce of [mean, mean(x^2)]."""
    import torch
    import torch.distributed as dist
    x = x.float()
    m = x.mean(0, keepdim=True)
    m2 = (x * x).mean(0, keepdim=True)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        buf = torch.cat([m, m2], 0)
        dist.all_reduce(buf, group=group)
        buf /= dist.get_world_size(group)
        m, m2 = buf[0:1], buf[1:2]
    return m, (m2 - m * m).clamp_min(0.0)


def synced_running_norm_update(norm, x, group=None):
    """``RunningNorm.update`` (running_norm.py:22-34) with the global batch moments, so every
    rank's normaliser evolves identically."""
    import torch
    with torch.no_grad():
        mean, var = global_batch_moments(x, group)
        weight = 1 / norm.count
        norm.running_mean = norm.running_mean * (1 - weight) + mean * weight
        norm.running_var = norm.running_var * (1 - weight) + var * weight
        norm.count += 1


def all_gather_failed_keys(keys: Sequence[str], group=None) -> List[str]:
    """Union (sorted, de-duplicated) of every rank's failed motion keys."""
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return sorted(set(keys))
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, list(keys), group=group)
    return sorted(set(k for ks in out for k in ks))
