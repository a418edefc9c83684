"""Public torch.library ops over the gfx950 kernels (SURVEY §7.1 "custom ops -> HIP kernels, each with
a torch fallback"): standard NCHW tensors in and out, usable outside the UNet engine, traceable
(fake/meta kernels), CPU tensors run the plain-torch reference of the same math.

    import distributedpytorch_amd.ops.library            # registers the ops
    y = torch.ops.dpa.conv3x3(x, w, b, True)             # conv3x3 s1 p1 + bias (+ReLU)
    p = torch.ops.dpa.max_pool2x2(y)                      # 2x2 / s2 max-pool (floor)
    l = torch.ops.dpa.bce_dice_loss(probs, target)        # reference loss: BCE - log(global Dice)

On a GPU the conv packs its fp32 weights to the kernel's bf16 GEMM layout (one pack launch) and
runs the same dispatch as the engine (row-streaming / row-halo / LDS-DMA / generic implicit GEMM),
bf16 operands with fp32 accumulation; the result is a channels_last bf16 tensor.  These are
inference ops (no autograd formula registered); training goes through the fused block engine
(models/hip_unet.py), whose backward is one explicit schedule per block.
Reference semantics: model/unet_parts.py:10-13 (Conv2d 3x3 pad 1 + ReLU), :26 (MaxPool2d(2, 2)),
utils/utils.py:9-25 (BCE - log Dice, Dice global over the batch).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import kernels as K


def _to_nhwc_bf16(x: torch.Tensor, cpad: int) -> torch.Tensor:
    """NCHW (any float dtype / memory format) -> dense NHWC bf16 with channels zero-padded to ``cpad``."""
    N, C, H, W = x.shape
    out = torch.zeros(N, H, W, cpad, dtype=torch.bfloat16, device=x.device) if cpad != C else \
        torch.empty(N, H, W, C, dtype=torch.bfloat16, device=x.device)
    out[..., :C].copy_(x.permute(0, 2, 3, 1))
    return out


def _pack_conv3x3(w: torch.Tensor, cs: int) -> torch.Tensor:
    Cout, Cin = w.shape[:2]
    kpad = K.round_up(9 * cs, 32)
    wf = w.detach().float().contiguous()
    packed = torch.zeros(Cout * kpad, dtype=torch.bfloat16, device=w.device)
    d = K.PackDesc(wf.data_ptr(), 0, 0, Cout, Cin, cs, Cout, kpad)
    descs = torch.frombuffer(bytearray(bytes(d)), dtype=torch.uint8).to(w.device)
    # (wf may be freed on return: the caching allocator reuses its block only in stream order,
    # after the pack kernel enqueued here)
    K.pack_weights(packed, descs, 1, Cout * kpad)
    return packed


@torch.library.custom_op("dpa::conv3x3", mutates_args=())
def conv3x3(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], relu: bool) -> torch.Tensor:
    """y = relu?(conv2d(x, weight, bias, stride 1, padding 1)); weight [Cout, Cin, 3, 3]."""
    if not x.is_cuda:
        y = F.conv2d(x, weight.to(x.dtype), None if bias is None else bias.to(x.dtype), padding=1)
        return F.relu(y) if relu else y
    N, Cin, H, W = x.shape
    Cout = weight.shape[0]
    assert weight.shape == (Cout, Cin, 3, 3) and Cout % 32 == 0, "dpa::conv3x3 on HIP: Cout % 32 == 0"
    cs = K.round_up(Cin, 8)
    xh = _to_nhwc_bf16(x, cs)
    packed = _pack_conv3x3(weight, cs)
    y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=x.device)
    b = None if bias is None else bias.detach().float().contiguous()
    K.igemm(xh, packed, y, Ngemm=Cout, Kpad=K.round_up(9 * cs, 32), KH=3, KW=3, stride=1, pad=1, Cs=cs,
            out_grid=(N, H, W), bias=b, relu=relu)
    return y.permute(0, 3, 1, 2)


def _fake_out(x, shape):
    """Fake output with the REAL op's strides: on the GPU the kernels return a channels_last bf16
    view (NHWC memory), on the CPU a contiguous tensor of the input dtype."""
    if x.is_cuda:
        return x.new_empty(shape, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    return x.new_empty(shape, dtype=x.dtype)


@conv3x3.register_fake
def _(x, weight, bias, relu):
    N, _, H, W = x.shape
    return _fake_out(x, (N, weight.shape[0], H, W))


@torch.library.custom_op("dpa::max_pool2x2", mutates_args=())
def max_pool2x2(x: torch.Tensor) -> torch.Tensor:
    """2x2 / stride 2 max-pool, floor semantics (nn.MaxPool2d(2, 2))."""
    if not x.is_cuda:
        return F.max_pool2d(x, 2, 2)
    N, C, H, W = x.shape
    assert C % 8 == 0, "dpa::max_pool2x2 on HIP: C % 8 == 0"
    xh = x.permute(0, 2, 3, 1)
    if not (x.dtype == torch.bfloat16 and x.is_contiguous(memory_format=torch.channels_last)):
        xh = _to_nhwc_bf16(x, C)
    y = torch.empty(N, H // 2, W // 2, C, dtype=torch.bfloat16, device=x.device)
    K.maxpool2(xh, y)
    return y.permute(0, 3, 1, 2)


@max_pool2x2.register_fake
def _(x):
    N, C, H, W = x.shape
    return _fake_out(x, (N, C, H // 2, W // 2))


@torch.library.custom_op("dpa::bce_dice_loss", mutates_args=())
def bce_dice_loss(probs: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Reference loss on probabilities: BCE(mean, log clamped at -100) - log(2 I / (P + T + 1e-15)),
    Dice global over the batch, fp32 (the four partial sums + loss tail of compute.py)."""
    from ..compute import loss_from_partials, loss_partials_from_probs
    p, t = probs.float(), target.float()
    return loss_from_partials(loss_partials_from_probs(p, t), t.numel()).reshape(())


@bce_dice_loss.register_fake
def _(probs, target):
    return probs.new_empty((), dtype=torch.float32)


__all__ = ["conv3x3", "max_pool2x2", "bce_dice_loss"]
