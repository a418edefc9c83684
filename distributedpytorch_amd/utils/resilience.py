"""Failure detection and race triage around the training loop (the reference has none —
torchrun defaults, no signal handling, no NCCL timeout, no sanitizer mode; ``train.py:29-61``,
``utils/train_utils.py:59-79``).

* :class:`StepWatchdog` — a daemon thread that expects ``kick()`` at least every ``timeout_s``;
  on a stall (a hung collective, a wave that never finishes, a dead peer) it writes every
  thread's Python stack to the rank's log and, by default, aborts the process so ``torchrun
  --max-restarts`` can restart the job from the last checkpoint (``--resume``).  It never
  ``exec``s and never touches the GPU.
* :class:`ShutdownGuard` — SIGTERM/SIGUSR1 set a flag that the loop checks at step boundaries;
  the loop then writes ``checkpoints/<method>_last.pt`` and exits cleanly (torchrun sends
  SIGTERM to surviving workers when a peer fails).
* :func:`check_finite` — non-finite loss detection at the (already host-synchronised) logging
  points, so it costs no extra device sync.
* :func:`comm_env_defaults` — RCCL async error handling so a failed collective raises instead of
  hanging; the process-group timeout comes from ``--comm-timeout``.
* Debug-sync (``--debug-sync`` / ``DPA_DEBUG_SYNC=1``, ``ops._lib.set_debug_sync``): every HIP
  launch is followed by a device synchronisation and the fault is attributed to that kernel; the
  pipeline also synchronises after every stage op.  Comparing a run with and without it
  (bitwise, ``tools/determinism_check.py``) separates stream-ordering races from kernel bugs.
"""
from __future__ import annotations

import faulthandler
import logging
import math
import os
import signal
import sys
import threading
import time
from typing import Callable, Iterable, Optional

log = logging.getLogger("dpa")


class StepWatchdog:
    def __init__(self, timeout_s: float, *, abort: bool = True, stream=None,
                 on_stall: Optional[Callable[[int, float], None]] = None):
        self.timeout_s = float(timeout_s)
        self.abort = abort
        self.stream = stream if stream is not None else sys.stderr
        self.on_stall = on_stall
        self._last = time.monotonic()
        self._step = -1
        self._stop = threading.Event()
        self.fired = False
        self._thread = None
        if self.timeout_s > 0:
            self._thread = threading.Thread(target=self._run, name="dpa-watchdog", daemon=True)
            self._thread.start()

    def kick(self, step: int):
        self._step = step
        self._last = time.monotonic()

    def _run(self):
        period = min(5.0, max(self.timeout_s / 4, 0.05))
        while not self._stop.wait(period):
            idle = time.monotonic() - self._last
            if idle < self.timeout_s:
                continue
            self.fired = True
            msg = f"[watchdog] no training progress for {idle:.0f}s (last step {self._step}); stacks follow"
            log.error(msg)
            try:
                print(msg, file=self.stream, flush=True)
                faulthandler.dump_traceback(file=self.stream, all_threads=True)
            except (ValueError, OSError):
                pass
            if self.on_stall is not None:
                self.on_stall(self._step, idle)
            if self.abort:
                os._exit(124)   # leave the exit code for torchrun's restart policy
            self._last = time.monotonic()

    def close(self):
        self._stop.set()


class ShutdownGuard:
    """Turn SIGTERM/SIGUSR1 into a flag checked between steps (install from the main thread)."""

    SIGNALS = (signal.SIGTERM, signal.SIGUSR1)

    def __init__(self, install: bool = True):
        self.requested: Optional[int] = None
        self._old = {}
        if install and threading.current_thread() is threading.main_thread():
            for s in self.SIGNALS:
                self._old[s] = signal.signal(s, self._handler)

    def _handler(self, signum, frame):
        self.requested = signum
        log.warning(f"received signal {signum}: checkpointing at the next step boundary")

    def close(self):
        for s, h in self._old.items():
            signal.signal(s, h)
        self._old.clear()


def check_finite(values: Iterable[float], step: int, policy: str = "raise") -> bool:
    """True if all finite; otherwise log and raise (policy ``raise``) or return False (``warn``)."""
    bad = [v for v in values if not math.isfinite(v)]
    if not bad:
        return True
    msg = f"non-finite loss at step {step}: {bad[:4]}"
    if policy == "raise":
        log.error(msg)
        raise FloatingPointError(msg)
    if policy == "warn":
        log.warning(msg)
    return False


def comm_env_defaults():
    """RCCL/NCCL: raise on a failed or timed-out collective instead of hanging the job."""
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.setdefault("TORCH_NCCL_DUMP_ON_TIMEOUT", "0")
