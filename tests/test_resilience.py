"""Failure detection / race-triage helpers (watchdog, signal-driven checkpoint,
non-finite loss detection, debug-sync)."""
import io
import os
import signal
import threading
import time

import pytest

from distributedpytorch_amd.config import parse_args
from distributedpytorch_amd.utils.resilience import ShutdownGuard, StepWatchdog, check_finite


def test_watchdog_fires_on_stall_and_not_while_kicked():
    hits = []
    buf = io.StringIO()
    dog = StepWatchdog(0.3, abort=False, stream=buf, on_stall=lambda s, idle: hits.append(s))
    for i in range(6):          # kicked faster than the timeout: silent
        dog.kick(i)
        time.sleep(0.1)
    assert not hits
    time.sleep(0.8)             # stall
    dog.close()
    assert hits and hits[0] == 5
    assert "no training progress" in buf.getvalue()


def test_check_finite_policies():
    assert check_finite([1.0, 2.0], 3)
    with pytest.raises(FloatingPointError):
        check_finite([1.0, float("nan")], 7, "raise")
    assert not check_finite([float("inf")], 7, "warn")


def test_shutdown_guard_flag():
    g = ShutdownGuard()
    os.kill(os.getpid(), signal.SIGUSR1)
    time.sleep(0.05)
    g.close()
    assert g.requested == signal.SIGUSR1


def test_train_stops_on_signal_and_resumes(tmp_path):
    """SIGUSR1 mid-run: the loop saves <method>_last.pt at the next step boundary and returns;
    --resume picks up from that step."""
    from distributedpytorch_amd.trainer import train
    args = ["-e", "200", "-b", "2", "--synthetic", "--synthetic-len", "16", "--img-size", "32",
            "--model", "unet-tiny", "--backend", "torch", "--dtype", "fp32", "--out-dir", str(tmp_path),
            "--log-every", "1", "--watchdog", "300", "--debug-sync"]
    done = threading.Event()

    def fire():
        # only once train() has installed its handler (SIGUSR1's default action would end the process -- under
        # a loaded machine the 1.5 s of a fixed timer can pass before that), then a few steps later
        deadline = time.monotonic() + 120
        while signal.getsignal(signal.SIGUSR1) in (signal.SIG_DFL, None) and time.monotonic() < deadline:
            if done.wait(0.05):
                return
        if not done.wait(1.0):
            os.kill(os.getpid(), signal.SIGUSR1)

    t = threading.Thread(target=fire, daemon=True)
    t.start()
    out = train(parse_args(args))
    done.set()
    t.join()
    assert out.get("stopped_by_signal") == signal.SIGUSR1
    assert os.path.exists(tmp_path / "checkpoints" / "singleGPU_last.pt")
    stopped = out["step"]
    assert 0 < stopped < 200 * 7
    from distributedpytorch_amd.ops._lib import set_debug_sync
    set_debug_sync(False)
    args2 = [a if a != "200" else "1" for a in args] + ["--resume"]
    out2 = train(parse_args(args2))
    assert out2["step"] >= stopped


def test_cli_resilience_flags():
    cfg = parse_args(["--watchdog", "60", "--comm-timeout", "120", "--nan-policy", "warn", "--debug-sync",
                      "--cuda-graph"])
    assert cfg.watchdog == 60 and cfg.comm_timeout == 120 and cfg.nan_policy == "warn"
    assert cfg.debug_sync and cfg.cuda_graph


def test_trace_ranges_wrap_blocks_without_changing_results():
    """roctx/record_function ranges (utils.tracing) around blocks: results identical, ranges visible
    in a torch.profiler trace."""
    import torch
    from distributedpytorch_amd.compute import make_compute
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.utils import tracing
    torch.manual_seed(0)
    m = build_model("unet-tiny")
    comp = make_compute(m, backend="torch", dtype="fp32")
    x = torch.rand(2, 3, 32, 32)
    t = (torch.rand(2, 1, 32, 32) > 0.5).float()
    s0 = comp.forward_partials(x, t)
    tracing.enable_ranges(True)
    try:
        with torch.profiler.profile() as prof:
            s1 = comp.forward_partials(x, t)
    finally:
        tracing.enable_ranges(False)
    assert torch.equal(s0, s1)
    names = {e.name for e in prof.events()}
    assert {"enc0", "enc1", "mid", "dec0", "dec1", "head"} <= names
