"""Per-device forward "compute" backends and the sum-decomposed loss.

The reference loss (``utils/utils.py:14-25``) is a function of four global sums over the batch:

    S = [sum BCE(p,t), sum p*[t==1], sum p, sum [t==1]],   N = #pixels
    loss = S0/N - log(2*S1 / (S2 + S3 + 1e-15))

so every parallel strategy computes *partial* sums where its data lives and combines them:
DP adds the per-device S on device 0 (= the reference's loss on the gathered batch), the pipeline
adds per-microbatch S on the last stage (= the loss on the whole batch, like the reference MP),
DDP uses its local S (reference per-rank semantics) or all-reduces it (``--global-dice``).

Backends (block implementations, ``models.blocks``):
* ``torch`` - stock PyTorch ops (MIOpen convs), bf16 autocast + channels_last activations.  This is
  the measured "stock PyTorch-ROCm" baseline of BASELINE.md and the CPU path.
* ``hip`` (``models.hip_unet.HipBlocks``) - hand-written gfx950 kernels, NHWC bf16.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .loss import EPS


def loss_partials_from_probs(p: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    p = p.float()
    t = t.float()
    dt = (t == 1).float()
    bce = F.binary_cross_entropy(p, t, reduction="sum")
    return torch.stack([bce, (p * dt).sum(), p.sum(), dt.sum()])


def loss_from_partials(S: torch.Tensor, n: int, dice: bool = True) -> torch.Tensor:
    if S.is_cuda and S.dtype == torch.float32:
        from .ops import kernels as K
        return K.loss_from_partials(S, n, dice)      # one HIP launch each way (csrc/unet_aux.hip)
    loss = S[0] / n
    if dice:
        loss = loss - torch.log(2 * S[1] / (S[2] + S[3] + EPS))
    return loss


class Compute:
    """Whole-model forward on one device through a block backend (see ``models.blocks``)."""

    def __init__(self, model: torch.nn.Module, blocks):
        self.model = model
        self.blocks = blocks
        self.depth = model.cfg.depth
        self.name = blocks.name

    def forward_partials(self, x: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        from .models.blocks import run_segment, n_blocks
        return run_segment(self.blocks, 0, n_blocks(self.depth), self.depth, {"x": x}, t)["partials"]

    def probs(self, x: torch.Tensor) -> torch.Tensor:
        from .models.blocks import run_segment, n_blocks
        return run_segment(self.blocks, 0, n_blocks(self.depth), self.depth, {"x": x}, want="probs")["probs"]


def resolve_backend(backend: str, device, dtype: str = "bf16", model=None) -> str:
    """``auto`` -> the HIP engines on a GPU, stock ops on CPU.  bf16: :class:`.models.hip_unet.HipBlocks`
    (bf16 storage, fp32 accumulate); fp32 -- the reference's precision, utils/train_utils.py:60-61 --:
    :class:`.models.hip_unet_f32.HipF32Blocks` (fp32 storage, fp32 MFMA) for the configurations it
    supports (``model`` given: checked; the reference family incl. the BN / bilinear variants, widths % 32),
    else the torch backend (fp32 on the GPU) for ``auto`` and an error for an explicit ``hip``.

    Stock MIOpen fp32 against this engine, same box, interleaved runs: profiles/fp32_vs_stock_same_box_r06.jsonl
    (BASELINE.md "Round 6"); MIOpen's first iteration also spends minutes compiling and searching solvers
    (449 s at b16; the b64 search did not finish in 600 s), while the HIP engine has no warm-up."""
    device = torch.device(device)
    if backend == "auto":
        if device.type != "cuda":
            return "torch"
        backend = "hip"
        if dtype == "fp32" and model is not None and not _f32_supported(model):
            import logging
            logging.getLogger(__name__).info(
                "dtype=fp32: this model configuration is not covered by the fp32 HIP engine; using the torch backend")
            return "torch"
        return backend
    if backend == "hip" and dtype not in ("bf16", "fp32"):
        raise ValueError(f"--backend hip computes in bf16 or fp32, not {dtype}")
    if backend == "hip" and dtype == "fp32" and model is not None and not _f32_supported(model):
        raise ValueError("--backend hip --dtype fp32: the fp32 engine covers the reference UNet family (with the "
                         "BatchNorm / bilinear variants) at channel widths divisible by 32")
    return backend


def _f32_supported(model) -> bool:
    from .models.hip_unet_f32 import supported
    return supported(model)


def make_blocks(model, backend: str = "auto", dtype: str = "bf16", device=None, owned=None):
    dev = torch.device(device) if device is not None else next(model.parameters()).device
    backend = resolve_backend(backend, dev, dtype, model)
    if backend == "hip" and dtype == "fp32":
        from .models.hip_unet_f32 import HipF32Blocks
        return HipF32Blocks(model, device=dev, owned=owned)
    if backend == "hip":
        from .models.hip_unet import HipBlocks
        return HipBlocks(model, dtype=dtype, device=dev, owned=owned)
    from .models.blocks import TorchBlocks
    return TorchBlocks(model, dtype=dtype)


def make_compute(model, backend: str = "auto", dtype: str = "bf16") -> Compute:
    return Compute(model, make_blocks(model, backend, dtype))
