"""Loader for the in-tree HIP kernel library ``distributedpytorch_amd/_C/libdpa_hip.so``.

The library is plain HIP C++ (``csrc/*.hip``) compiled by ``hipcc --offload-arch=gfx950`` with
``extern "C"`` launchers; it links the *same* ``libamdhip64.so.7`` that torch already loaded
(identical SONAME, rpath -> torch/lib), so the ``hipStream_t`` handles we pass from
``torch.cuda.current_stream().cuda_stream`` are valid in it.  Calls go through ctypes: no torch
headers, seconds to rebuild, and every launcher takes raw device pointers + the stream.

On a machine with a GPU the library is REQUIRED: ``lib()`` raises if it is missing instead of
silently falling back to eager torch ops.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent.parent
# DPA_LIB_PATH: load another build of the same library (tools/asan_host.sh: host code under ASan)
LIB_PATH = Path(os.environ["DPA_LIB_PATH"]) if os.environ.get("DPA_LIB_PATH") else _HERE / "_C" / "libdpa_hip.so"
_lib = None
_err = None


def _load():
    global _lib, _err
    if _lib is not None or _err is not None:
        return _lib
    try:
        import torch  # noqa: F401  (must be loaded first so the HIP runtime is torch's)
        _lib = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
        _declare(_lib)
    except OSError as e:  # missing or unloadable
        _err = e
        _lib = None
    return _lib


def available() -> bool:
    return _load() is not None


def lib():
    L = _load()
    if L is None:
        raise RuntimeError(
            f"HIP kernel library not available ({LIB_PATH}): {_err}. Build it with "
            f"`python -c 'import __graft_entry__ as g; g.build()'` or `python tools/build_hip.py`.")
    return L


def _declare(L):
    for name in ("dpa_version", "dpa_igemm", "dpa_wgrad", "dpa_wgrad_reduce", "dpa_input_nhwc8", "dpa_maxpool2",
                 "dpa_pool_bwd", "dpa_pool_bwd_code_blocks", "dpa_chan_sum_bf16", "dpa_pack_weights", "dpa_head_fwd", "dpa_head_bwd", "dpa_adam_flat",
                 "dpa_igemm_halo", "dpa_wgrad_halo", "dpa_igemm_stream", "dpa_wgrad_stream", "dpa_wgrad_gemm", "dpa_wgrad_band", "dpa_wgrad_band128", "dpa_adam_flat_dev", "dpa_igemm_glds",
                 "dpa_loss_finish", "dpa_loss_grad", "dpa_pool_bwd_code", "dpa_bn_fwd", "dpa_bn_bwd", "dpa_bn_bwd_coef",
                 "dpa_up2_fwd", "dpa_up2_bwd", "dpa_deconv_bwd", "dpa_deconv_fwd", "dpa_slab_sum",
                 "dpa_igemm_stream_blocks", "dpa_slab_fold", "dpa_bwd_stream", "dpa_head_grad_from_slab", "dpa_bwd_stream_pool_ok",
                 "dpa_wgrad_reduce_cfg", "dpa_igemm_f32", "dpa_wgrad_f32", "dpa_relu_bwd_f32", "dpa_maxpool2_f32",
                 "dpa_maxpool2_bwd_f32", "dpa_head_f32_blocks", "dpa_head_f32", "dpa_head_bwd_f32", "dpa_nchw_to_nhwc4_f32",
                 "dpa_channel_sum_f32", "dpa_enc_out_bwd_f32", "dpa_pack_weights_f32", "dpa_zero", "dpa_comm_probe"):
        getattr(L, name).restype = ctypes.c_int
    L.dpa_head_slab_blocks.restype = ctypes.c_int
    L.dpa_head_slab_blocks.argtypes = [ctypes.c_longlong]
    L.dpa_bn_slab_rows.restype = ctypes.c_int
    L.dpa_bn_slab_rows.argtypes = [ctypes.c_longlong, ctypes.c_int]
    L.dpa_bwd_stream_geom.restype = ctypes.c_int
    L.dpa_bwd_stream_geom.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    L.dpa_error_string.restype = ctypes.c_char_p
    from .config import KernelConfig
    kc = KernelConfig.from_env()
    L.dpa_wgrad_set_presum(ctypes.c_int(int(kc.wgrad_presum)))
    L.dpa_igemm_set_slpp(ctypes.c_int(int(kc.slpp)))
    L.dpa_igemm_set_slp256(ctypes.c_int(int(kc.slp256)))
    L.dpa_wgrad_set_presum_y(ctypes.c_int(int(kc.wgrad_presum_y)))


def check(err: int, name: str):
    """Raise on a launch error.  Under debug-sync (``--debug-sync`` / ``DPA_DEBUG_SYNC=1``) also wait
    for the kernel and attribute any asynchronous fault to ``name`` (stream-ordering / race triage:
    every launch becomes a synchronisation point)."""
    if err != 0:
        L = lib()
        msg = L.dpa_error_string(err).decode()
        raise RuntimeError(f"{name} failed: hip error {err} ({msg})")
    if _DEBUG_SYNC[0]:
        import torch
        if torch.cuda.is_current_stream_capturing():
            return
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:
            raise RuntimeError(f"{name}: asynchronous fault detected right after launch: {e}") from e


_DEBUG_SYNC = [os.environ.get("DPA_DEBUG_SYNC", "0") == "1"]


def set_debug_sync(on: bool):
    _DEBUG_SYNC[0] = bool(on)


def debug_sync() -> bool:
    return _DEBUG_SYNC[0]


def stream_ptr(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())
