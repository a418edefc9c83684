"""roctx ranges around the framework's own units of work (SURVEY §5 "Tracing / profiling": the
reference has only wall-clock deltas, utils/train_utils.py:52,78).

``trace_range("enc2")`` pushes a roctx range (``torch.cuda.nvtx`` is roctx on ROCm builds) around a
UNet block, a pipeline send/recv, a gradient bucket's all-reduce launch.  Off by default (a range is
a host call per block); on with ``--trace-ranges`` or ``DPA_ROCTX=1``.  The ranges appear in
``rocprofv3 --marker-trace`` timelines and in torch.profiler traces next to the HIP kernels they
enclose, so a kernel can be attributed to its layer / stage / bucket.
"""
from __future__ import annotations

import contextlib
import os

_ON = [os.environ.get("DPA_ROCTX", "0") == "1"]


def enable_ranges(on: bool = True):
    _ON[0] = bool(on)


def ranges_enabled() -> bool:
    return _ON[0]


@contextlib.contextmanager
def trace_range(name: str):
    if not _ON[0]:
        yield
        return
    import torch
    pushed = False
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)
        pushed = True
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()
