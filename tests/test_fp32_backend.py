"""``--dtype fp32`` (the reference's precision, utils/train_utils.py:60-61): on a GPU ``backend=auto``
resolves to the fp32 HIP engine (models/hip_unet_f32.py, csrc/fp32.hip) for the reference UNet family and
its BatchNorm / bilinear variants (round 6), and to the torch backend for configurations it does not cover
(channel widths not divisible by 32); an explicit ``--backend hip --dtype fp32`` on an uncovered model is a
clear error."""
import os
import subprocess
import sys

import pytest

from distributedpytorch_amd.compute import resolve_backend
from distributedpytorch_amd.models.unet import build_model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_resolve_backend_fp32():
    unet, bn, bil = build_model("unet"), build_model("unet-bn"), build_model("unet-bn-bilinear")
    tiny = build_model("unet-tiny")                     # base 8: widths not divisible by 32
    assert resolve_backend("auto", "cuda:0", "bf16") == "hip"
    assert resolve_backend("auto", "cuda:0", "fp32") == "hip"
    assert resolve_backend("auto", "cuda:0", "fp32", unet) == "hip"
    assert resolve_backend("auto", "cuda:0", "fp32", bn) == "hip"
    assert resolve_backend("auto", "cuda:0", "fp32", bil) == "hip"
    assert resolve_backend("auto", "cuda:0", "fp32", tiny) == "torch"
    assert resolve_backend("auto", "cpu", "fp32", unet) == "torch"
    assert resolve_backend("torch", "cuda:0", "fp32") == "torch"
    assert resolve_backend("hip", "cuda:0", "fp32", unet) == "hip"
    with pytest.raises(ValueError, match="fp32 engine"):
        resolve_backend("hip", "cuda:0", "fp32", tiny)


@pytest.mark.gpu
def test_train_py_fp32_on_gpu(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "train.py"), "--dtype", "fp32", "--synthetic", "--synthetic-len", "16",
           "--img-size", "128", "-e", "1", "-b", "4", "--out-dir", str(tmp_path)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert (tmp_path / "checkpoints" / "singleGPU.pth").exists()
    log = (tmp_path / "logs" / "singleGPU.log").read_text()
    assert "backend=hip-fp32" in log, log[-2000:]
