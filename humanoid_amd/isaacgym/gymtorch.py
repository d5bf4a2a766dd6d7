"""``isaacgym.gymtorch`` facade: zero-copy torch views of engine memory and back.

``wrap_tensor`` follows ``packages/gymtorch/gymtorch/gymtorch.cpp:33-158`` (non-owning view of a
device pointer, ``DataPtr`` without deleter, ``:90``) but raises instead of printing and returning
an empty tensor (``:40-51``). ``unwrap_tensor`` follows ``gymtorch/wrapper.py:47-56`` (contiguous
tensors only).
"""
from __future__ import annotations

from .gymapi import GymTensor

_DTYPES = None


def _dtype_map():
    global _DTYPES
    if _DTYPES is None:
        import torch
        # GymTensor.h:20-28 -- Fp32=1, Uint32->int32, Uint64->int64, Uint8, Int16
        _DTYPES = {1: torch.float32, 2: torch.int32, 3: torch.int64, 4: torch.uint8, 5: torch.int16}
    return _DTYPES


def wrap_tensor(gym_tensor: GymTensor, offsets=None, counts=None):
    """Torch view of an engine buffer (or of an unwrapped torch tensor), sharing its memory."""
    import torch
    from ..engine import wrap_device_pointer
    owner = gym_tensor._owner
    if isinstance(owner, torch.Tensor) and owner.data_ptr() == gym_tensor.data_ptr:
        t = owner
    else:
        dt = _dtype_map().get(gym_tensor.dtype)
        if dt is None:
            raise ValueError(f"unsupported gym tensor dtype {gym_tensor.dtype}")
        t = wrap_device_pointer(gym_tensor.data_ptr, list(gym_tensor.shape), dt, gym_tensor.device, owner=owner)
    if offsets is not None or counts is not None:  # gymtorch.cpp:122-150 strided sub-views
        offsets = offsets or (0,) * t.dim()
        counts = counts or tuple(t.shape)
        for d, (o, c) in enumerate(zip(offsets, counts)):
            t = t.narrow(d, o, c)
    return t


def unwrap_tensor(t) -> GymTensor:
    import torch
    if not t.is_contiguous():
        raise ValueError("Input tensor must be contiguous")  # wrapper.py:52
    code = {v: k for k, v in _dtype_map().items()}.get(t.dtype)
    if code is None:
        raise ValueError(f"unsupported dtype {t.dtype}")
    dev = t.device.index if t.device.type == "cuda" else -1
    return GymTensor(t.data_ptr(), tuple(t.shape), code, dev if dev is not None else torch.cuda.current_device(),
                     owner=t)
