"""``--dtype fp32`` (the reference's precision, utils/train_utils.py:60-61) on a GPU: ``backend=auto``
resolves to the torch backend instead of crashing in the bf16-only HIP engine; an explicit
``--backend hip --dtype fp32`` is a clear error."""
import os
import subprocess
import sys

import pytest

from distributedpytorch_amd.compute import resolve_backend

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_resolve_backend_fp32_picks_torch():
    assert resolve_backend("auto", "cuda:0", "bf16") == "hip"
    assert resolve_backend("auto", "cuda:0", "fp32") == "torch"
    assert resolve_backend("auto", "cpu", "bf16") == "torch"
    assert resolve_backend("torch", "cuda:0", "fp32") == "torch"
    with pytest.raises(ValueError, match="bf16"):
        resolve_backend("hip", "cuda:0", "fp32")


@pytest.mark.gpu
def test_train_py_fp32_on_gpu(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "train.py"), "--dtype", "fp32", "--synthetic", "--synthetic-len", "16",
           "--img-size", "128", "-e", "1", "-b", "4", "--out-dir", str(tmp_path)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert (tmp_path / "checkpoints" / "singleGPU.pth").exists()
    log = (tmp_path / "logs" / "singleGPU.log").read_text()
    assert "backend=torch" in log, log[-2000:]
