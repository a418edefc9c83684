"""MI355X kernel ops (HIP, gfx950) with torch reference implementations for CPU / parity tests.

Each public op takes torch tensors.  On CUDA(=HIP) tensors it calls the hand-written kernel in
``_C/libdpa_hip.so`` (required: raises if missing); on CPU tensors it runs the plain-torch
reference of the same math, which the numerics tests compare against.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import available as hip_available, check, ptr, stream_ptr

c_float = ctypes.c_float
c_ll = ctypes.c_longlong


def adam_step(p, g, m, v, *, lr, beta1, beta2, eps, weight_decay, bc1, bc2):
    """In-place Adam (L2 decay) over flat fp32 tensors ``p, g, m, v`` (one launch)."""
    if not p.is_cuda:
        from ..optim import adam_reference
        return adam_reference(p, g, m, v, lr, beta1, beta2, eps, weight_decay, bc1, bc2)
    assert p.dtype == g.dtype == m.dtype == v.dtype == torch.float32
    assert p.is_contiguous() and g.is_contiguous() and m.is_contiguous() and v.is_contiguous()
    assert p.numel() == g.numel() == m.numel() == v.numel()
    L = _lib.lib()
    err = L.dpa_adam_flat(ptr(p), ptr(g), ptr(m), ptr(v), c_ll(p.numel()), c_float(lr), c_float(beta1),
                          c_float(beta2), c_float(eps), c_float(weight_decay), c_float(bc1), c_float(bc2),
                          ctypes.c_void_p(stream_ptr(p.device)))
    check(err, "adam_flat")


def adam_step_dev(p, g, m, v, state, *, beta1, beta2, eps, weight_decay):
    """Adam whose step count, lr and bias corrections live in ``state`` (fp64 device tensor
    ``[step, lr, 1/bc1, 1/sqrt(bc2)]``); the step increments ``state[0]`` itself, so one captured
    launch sequence is valid for every replay of a HIP graph."""
    assert state.dtype == torch.float64 and state.numel() >= 4 and state.device == p.device
    if not p.is_cuda:
        from ..optim import adam_reference
        t = float(state[0]) + 1.0
        state[0] = t
        return adam_reference(p, g, m, v, float(state[1]), beta1, beta2, eps, weight_decay,
                              1 - beta1 ** t, 1 - beta2 ** t)
    assert p.dtype == g.dtype == m.dtype == v.dtype == torch.float32
    assert p.is_contiguous() and g.is_contiguous() and m.is_contiguous() and v.is_contiguous()
    assert p.numel() == g.numel() == m.numel() == v.numel()
    L = _lib.lib()
    err = L.dpa_adam_flat_dev(ptr(p), ptr(g), ptr(m), ptr(v), c_ll(p.numel()), ptr(state), ctypes.c_double(beta1),
                              ctypes.c_double(beta2), c_float(eps), c_float(weight_decay),
                              ctypes.c_void_p(stream_ptr(p.device)))
    check(err, "adam_flat_dev")


__all__ = ["adam_step", "adam_step_dev", "hip_available"]
