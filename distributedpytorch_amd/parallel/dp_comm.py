"""ctypes binding of the native single-process RCCL clique (``csrc/dp_comm.cpp`` ->
``_C/libdpa_comm.so``) used by ``-t DP`` (:mod:`.dp`).

``DPComm(devices)`` creates one RCCL communicator per local device with ``ncclCommInitAll``; its
collectives take one tensor per device and issue all of them in one RCCL group, each on that
device's *current* stream (no host synchronisation: ordered after the kernels that produced the
data).  Replaces torch.nn.DataParallel's broadcast_coalesced / nccl.reduce (reference
``utils/train_utils.py:98,138-144``)."""
from __future__ import annotations

import ctypes
from pathlib import Path
from typing import List, Sequence

import torch

LIB_PATH = Path(__file__).resolve().parent.parent / "_C" / "libdpa_comm.so"
_lib = None
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3}
_OP = {"sum": 0, "avg": 1, "max": 2}


def lib():
    global _lib
    if _lib is None:
        import torch.cuda  # noqa: F401  (torch's librccl.so.1 / libamdhip64 first)
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} missing: build with `python tools/build_hip.py`")
        L = ctypes.CDLL(str(LIB_PATH))
        for n in ("dpa_dp_comm_init", "dpa_dp_comm_destroy", "dpa_dp_comm_size", "dpa_dp_all_reduce",
                  "dpa_dp_broadcast", "dpa_dp_version"):
            getattr(L, n).restype = ctypes.c_int
        L.dpa_dp_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except (OSError, RuntimeError):
        return False


class DPComm:
    def __init__(self, devices: Sequence):
        self.devices = [torch.device(d) for d in devices]
        assert all(d.type == "cuda" for d in self.devices), "DPComm needs CUDA/HIP devices"
        idx = [d.index if d.index is not None else 0 for d in self.devices]
        assert len(set(idx)) == len(idx), "one communicator per distinct device"
        arr = (ctypes.c_int * len(idx))(*idx)
        h = ctypes.c_void_p()
        self._check(lib().dpa_dp_comm_init(ctypes.c_int(len(idx)), arr, ctypes.byref(h)), "ncclCommInitAll")
        self._h = h

    @staticmethod
    def _check(r: int, what: str):
        if r != 0:
            raise RuntimeError(f"{what} failed: rccl error {r} ({lib().dpa_dp_error(r).decode()})")

    def _args(self, tensors: List[torch.Tensor], streams=None):
        assert len(tensors) == len(self.devices)
        n = tensors[0].numel()
        dt = tensors[0].dtype
        for t, d in zip(tensors, self.devices):
            assert t.device == d and t.is_contiguous() and t.numel() == n and t.dtype == dt, (t.device, d)
        bufs = (ctypes.c_void_p * len(tensors))(*[t.data_ptr() for t in tensors])
        if streams is None:
            streams = [torch.cuda.current_stream(d) for d in self.devices]
        assert len(streams) == len(self.devices)
        sts = (ctypes.c_void_p * len(tensors))(*[s.cuda_stream for s in streams])
        return bufs, sts, n, _DT[dt]

    def all_reduce(self, tensors: List[torch.Tensor], op: str = "sum", streams=None):
        """In-place all-reduce, one tensor per device, on ``streams`` (default: each device's
        current stream)."""
        bufs, sts, n, dt = self._args(tensors, streams)
        self._check(lib().dpa_dp_all_reduce(self._h, bufs, ctypes.c_longlong(n), ctypes.c_int(dt),
                                            ctypes.c_int(_OP[op]), sts), "ncclAllReduce")

    def broadcast(self, tensors: List[torch.Tensor], root: int = 0):
        bufs, sts, n, dt = self._args(tensors)
        self._check(lib().dpa_dp_broadcast(self._h, bufs, ctypes.c_longlong(n), ctypes.c_int(dt),
                                           ctypes.c_int(root), sts), "ncclBroadcast")

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().dpa_dp_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
