"""fp32 training engine on the hand-written fp32 kernels (csrc/fp32.hip, ops/fp32.py).

The reference trains in fp32 (``/root/reference/utils/train_utils.py:60-61``: fp32 model and inputs,
no autocast; model ``model/unet_parts.py`` / ``unet_model.py``).  The bf16 engine
(:class:`.hip_unet.HipBlocks`) stores bf16 activations; this engine keeps every activation, gradient
and weight in fp32 and runs every conv-shaped product on fp32 MFMA (v_mfma_f32_16x16x4_f32):

* conv3x3 + bias + ReLU forward, its dgrad (flipped weights) and weight / bias gradient;
* ConvTranspose2d(k2, s2) forward (GEMM + 2x2 scatter), dgrad (stride-2 gather GEMM) and weight /
  bias gradient;
* 2x2 max-pool with window codes and its backward, the segmentation head (1x1 conv + sigmoid +
  BCE / Dice partial sums, ``utils/utils.py:9-25``) and its backward, the NCHW -> NHWC input pass.

Granularity is one autograd Function per op, except a DoubleConv's two convs (one Function: the inner
ReLU backward is the mask epilogue of the second conv's dgrad); the bf16 engine's other cross-op fusions
are not replicated (fp32 is the parity / precision path, bf16 the fast one).  Activations are NHWC
tensors handed between blocks as logical-NCHW channels_last views, as in the bf16 engine.  Supported:
the reference UNet family without BatchNorm and with transposed-conv up-sampling, channel widths
divisible by 32 (other configurations take the stock torch path, ``compute.resolve_backend``).
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops import fp32 as F32
from .unet import Up


def supported(model) -> bool:
    cfg = model.cfg
    if getattr(cfg, "batchnorm", False) or any(isinstance(m, Up) for m in model.decoder.ups()):
        return False
    convs = [c for b in model.encoder.blocks() for c in b.convs()] + list(model.mid.convs()) + \
            [c for b in model.decoder.blocks() for c in b.convs()]
    return all(c.out_channels % 32 == 0 for c in convs) and model.encoder.blocks()[0].convs()[0].in_channels <= 4 \
        and model.segmap.out_channels == 1 and model.segmap.in_channels in (8, 16, 32, 64)


def _v(t: torch.Tensor) -> torch.Tensor:
    """logical-NCHW channels_last -> NHWC view (copies only if the layout is something else)."""
    if t.dim() == 4 and t.stride(1) != 1:
        t = t.contiguous(memory_format=torch.channels_last)
    return t.permute(0, 2, 3, 1)


def _o(t: torch.Tensor) -> torch.Tensor:
    return t.permute(0, 3, 1, 2)


def _dense(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous() else t.contiguous()


def _conv_fwd(x, weight, bias, cs: int):
    """relu(conv3x3(x) + b), NHWC fp32; ``cs`` = channels of x the kernel reads (>= Cin, zero weights for
    the padding channels of the network input)."""
    N, H, W = x.shape[:3]
    co = weight.shape[0]
    wp, kpad = F32.pack_conv_fwd(weight, cs)
    y = torch.empty(N, H, W, co, dtype=torch.float32, device=x.device)
    F32.igemm(x, wp, y, Ngemm=co, Kpad=kpad, KH=3, KW=3, stride=1, pad=1, Cs=cs, out_grid=(N, H, W),
              bias=bias.detach(), relu=True)
    return y


def _conv_dgrad(ge, weight, cs: int, mask=None):
    """dL/dx of a conv3x3 from the pre-activation gradient ``ge``; ``mask`` = the input's own ReLU output
    (its backward applied in the epilogue)."""
    co, ci = weight.shape[:2]
    N, H, W = ge.shape[:3]
    wd, kd = F32.pack_conv_dgrad(weight)
    ng = F32.round_up(cs, 32)          # GEMM-N multiple of 32: zero rows for the padding channels
    if ng != ci:
        wd = torch.cat([wd, wd.new_zeros(ng - ci, kd)]).contiguous()
    gx = torch.empty(N, H, W, ng, dtype=torch.float32, device=ge.device)
    F32.igemm(ge, wd, gx, Ngemm=ng, Kpad=kd, KH=3, KW=3, stride=1, pad=1, Cs=co, out_grid=(N, H, W), mask=mask)
    return gx[..., :cs] if ng != cs else gx


def _conv_wgrad(ge, x, weight, cs: int):
    co, ci = weight.shape[:2]
    gw = torch.zeros(co, cs, 3, 3, dtype=torch.float32, device=x.device)
    gb = torch.zeros(co, dtype=torch.float32, device=x.device)
    F32.wgrad(ge, x, gw, gb, KH=3, KW=3, s=1, pad=1)
    return (gw if cs == ci else gw[:, :ci].contiguous()), gb


class _ConvReLU(torch.autograd.Function):
    """y = relu(conv3x3(x) + b), NHWC fp32 (one conv: the halves of a DoubleConv cut by a pipeline stage
    boundary)."""

    @staticmethod
    def forward(ctx, x, weight, bias, cs: int):
        y = _conv_fwd(x, weight, bias, cs)
        ctx.cs = cs
        ctx.save_for_backward(x, weight, y)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, y = ctx.saved_tensors
        ge = F32.relu_bwd(_dense(gy), y)
        gx = _conv_dgrad(ge, weight, ctx.cs) if ctx.needs_input_grad[0] else None
        gw, gb = _conv_wgrad(ge, x, weight, ctx.cs)
        return gx, gw, gb, None


class _DoubleConvReLU(torch.autograd.Function):
    """relu(conv2(relu(conv1(x)))) (reference DoubleConv without BatchNorm, model/unet_parts.py:7-15) as one
    Function: the inner ReLU's backward is the mask epilogue of conv2's dgrad, so the inner gradient is
    written once, already masked."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, cs: int):
        a = _conv_fwd(x, w1, b1, cs)
        y = _conv_fwd(a, w2, b2, a.shape[3])
        ctx.cs = cs
        ctx.save_for_backward(x, w1, a, w2, y)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w1, a, w2, y = ctx.saved_tensors
        ge2 = F32.relu_bwd(_dense(gy), y)
        ge1 = _conv_dgrad(ge2, w2, a.shape[3], mask=a)
        gw2, gb2 = _conv_wgrad(ge2, a, w2, a.shape[3])
        gx = _conv_dgrad(ge1, w1, ctx.cs) if ctx.needs_input_grad[0] else None
        gw1, gb1 = _conv_wgrad(ge1, x, w1, ctx.cs)
        return gx, gw1, gb1, gw2, gb2, None


class _EncBlock(torch.autograd.Function):
    """Encoder block: DoubleConv + 2x2 max-pool (reference Encoder, model/unet_parts.py:20-40) -> (skip, pooled).
    Backward: the skip gradient, the pool backward and the last ReLU backward form the second conv's
    pre-activation gradient in one pass (F32.enc_out_bwd); the inner ReLU as in :class:`_DoubleConvReLU`."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, cs: int):
        a = _conv_fwd(x, w1, b1, cs)
        y = _conv_fwd(a, w2, b2, a.shape[3])
        pooled, code = F32.maxpool2(y)
        ctx.cs = cs
        ctx.save_for_backward(x, w1, a, w2, y, code)
        return y, pooled

    @staticmethod
    def backward(ctx, gs, gp):
        x, w1, a, w2, y, code = ctx.saved_tensors
        if gs is not None and not F32.nhwc_ok(gs):
            gs = gs.contiguous()
        ge2 = F32.enc_out_bwd(gs, None if gp is None else _dense(gp), code, y)
        ge1 = _conv_dgrad(ge2, w2, a.shape[3], mask=a)
        gw2, gb2 = _conv_wgrad(ge2, a, w2, a.shape[3])
        gx = _conv_dgrad(ge1, w1, ctx.cs) if ctx.needs_input_grad[0] else None
        gw1, gb1 = _conv_wgrad(ge1, x, w1, ctx.cs)
        return gx, gw1, gb1, gw2, gb2, None


class _Deconv(torch.autograd.Function):
    """y = ConvTranspose2d(k2, s2)(x) + b, NHWC fp32 (reference model/unet_parts.py:51-54)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        N, h, w, ci = x.shape
        co = weight.shape[1]
        y = torch.empty(N, 2 * h, 2 * w, co, dtype=torch.float32, device=x.device)
        F32.igemm(x, F32.pack_deconv_fwd(weight), y, Ngemm=4 * co, Kpad=ci, KH=1, KW=1, stride=1, pad=0, Cs=ci,
                  out_grid=(N, h, w), bias=bias.detach(), mode=1, Cout=co)
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        N, h, w, ci = x.shape
        co = weight.shape[1]
        gy = _dense(gy)
        gx = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty(N, h, w, ci, dtype=torch.float32, device=x.device)
            F32.igemm(gy, F32.pack_deconv_dgrad(weight), gx, Ngemm=ci, Kpad=4 * co, KH=2, KW=2, stride=2, pad=0, Cs=co,
                      out_grid=(N, h, w))
        gw = torch.zeros(ci, co, 2, 2, dtype=torch.float32, device=x.device)
        F32.wgrad(x, gy, gw, None, KH=2, KW=2, s=2, pad=0)
        gb = torch.zeros(co, dtype=torch.float32, device=x.device)
        F32.channel_sum(gy, gb)
        return gx, gw, gb


class _UpCat(torch.autograd.Function):
    """[skip ‖ ConvTranspose2d(k2, s2)(x) + b] in one NHWC buffer (reference concat order, skip first,
    model/unet_parts.py:58-59): the transposed conv's scatter epilogue stores straight into the upper
    channel half; the backward reads both gradient halves in place (no split copies)."""

    @staticmethod
    def forward(ctx, x, skip, weight, bias):
        N, h, w, ci = x.shape
        co, C = weight.shape[1], skip.shape[3]
        buf = torch.empty(N, 2 * h, 2 * w, C + co, dtype=torch.float32, device=x.device)
        buf[..., :C].copy_(skip)
        F32.igemm(x, F32.pack_deconv_fwd(weight), buf[..., C:], Ngemm=4 * co, Kpad=ci, KH=1, KW=1, stride=1, pad=0,
                  Cs=ci, out_grid=(N, h, w), bias=bias.detach(), mode=1, Cout=co)
        ctx.C = C
        ctx.save_for_backward(x, weight)
        return buf

    @staticmethod
    def backward(ctx, gbuf):
        x, weight = ctx.saved_tensors
        N, h, w, ci = x.shape
        co, C = weight.shape[1], ctx.C
        if not F32.nhwc_ok(gbuf):
            gbuf = gbuf.contiguous()
        gs, gy = gbuf[..., :C], gbuf[..., C:]
        gx = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty(N, h, w, ci, dtype=torch.float32, device=x.device)
            F32.igemm(gy, F32.pack_deconv_dgrad(weight), gx, Ngemm=ci, Kpad=4 * co, KH=2, KW=2, stride=2, pad=0, Cs=co,
                      out_grid=(N, h, w))
        gw = torch.zeros(ci, co, 2, 2, dtype=torch.float32, device=x.device)
        F32.wgrad(x, gy, gw, None, KH=2, KW=2, s=2, pad=0)
        gb = torch.zeros(co, dtype=torch.float32, device=x.device)
        F32.channel_sum(gy, gb)
        return gx, gs, gw, gb


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y, code = F32.maxpool2(x)
        ctx.hw = x.shape[1:3]
        ctx.save_for_backward(code)
        return y

    @staticmethod
    def backward(ctx, gy):
        (code,) = ctx.saved_tensors
        return F32.maxpool2_bwd(_dense(gy), code, *ctx.hw)


class _HeadLoss(torch.autograd.Function):
    """Partial sums S[4] of the reference loss from the last decoder output (1x1 conv + sigmoid)."""

    @staticmethod
    def forward(ctx, y, weight, bias, t):
        S, _ = F32.head_fwd(y, weight, bias, t)
        ctx.save_for_backward(y, weight, bias, t)
        return S

    @staticmethod
    def backward(ctx, dS):
        y, weight, bias, t = ctx.saved_tensors
        gy, gw, gb = F32.head_bwd(y, weight, bias, t, dS)
        return gy, gw.view_as(weight), gb.view_as(bias), None


class HipF32Blocks:
    """Block backend (models.blocks protocol) of the fp32 engine."""

    name = "hip"

    def __init__(self, model, device=None, owned=None):
        self.model = model
        self.device = torch.device(device) if device is not None else next(model.parameters()).device
        assert self.device.type == "cuda", "HipF32Blocks needs a GPU"
        assert supported(model), "fp32 HIP engine: reference UNet family without BatchNorm / bilinear, widths % 32 == 0"
        self.dense_skips = set()

    def prep(self, x):
        if x.dim() == 4 and x.shape[1] <= 4 and x.dtype == torch.float32 and x.stride(1) != 1:
            return _o(F32.input_nhwc4(x))
        if x.dim() == 4 and x.stride(1) == 1 and x.shape[1] == 4:
            return x          # already converted
        return _o(F32.input_nhwc4(x.float()))

    def _conv(self, conv, x, cs=None):
        return _ConvReLU.apply(x, conv.weight, conv.bias, cs or x.shape[3])

    def _double(self, c1, c2, x, cs=None):
        return _DoubleConvReLU.apply(x, c1.weight, c1.bias, c2.weight, c2.bias, cs or x.shape[3])

    def enc(self, l: int, x):
        c1, c2 = self.model.encoder.blocks()[l].convs()
        xv = _v(x)
        s, p = _EncBlock.apply(xv, c1.weight, c1.bias, c2.weight, c2.bias, 4 if l == 0 else xv.shape[3])
        return _o(s), _o(p)

    def mid(self, x):
        c1, c2 = self.model.mid.convs()
        return _o(self._double(c1, c2, _v(x)))

    def dec(self, i: int, x, skip):
        # transposed conv, reference CenterCrop of the skip (model/unet_parts.py:58-74), concat with the
        # skip first (:59), conv_block
        c1, c2 = self.model.decoder.blocks()[i].convs()
        return _o(self._double(c1, c2, self._up_cat(i, x, skip)))

    # halves of a block cut between its two convs (pipeline stage boundary inside a DoubleConv)
    def enc_a(self, l: int, x):
        c1 = self.model.encoder.blocks()[l].convs()[0]
        return _o(self._conv(c1, _v(x), 4 if l == 0 else None))

    def enc_b(self, l: int, a):
        c2 = self.model.encoder.blocks()[l].convs()[1]
        s = self._conv(c2, _v(a))
        return _o(s), _o(_MaxPool.apply(s))

    def mid_a(self, x):
        return _o(self._conv(self.model.mid.convs()[0], _v(x)))

    def mid_b(self, a):
        return _o(self._conv(self.model.mid.convs()[1], _v(a)))

    def _up_cat(self, i: int, x, skip):
        d = self.model.decoder.ups()[i]
        xv, sk = _v(x), _v(skip)
        if tuple(sk.shape[1:3]) == (2 * xv.shape[1], 2 * xv.shape[2]) and sk.shape[3] % 4 == 0:
            return _UpCat.apply(xv, sk, d.weight, d.bias)
        up = _Deconv.apply(xv, d.weight, d.bias)
        h2, w2 = up.shape[1:3]
        if tuple(sk.shape[1:3]) != (h2, w2):
            top, left = int(round((sk.shape[1] - h2) / 2.0)), int(round((sk.shape[2] - w2) / 2.0))
            sk = sk[:, top:top + h2, left:left + w2]
        return torch.cat([sk, up], dim=3)

    def dec_a(self, i: int, x, skip):
        c1 = self.model.decoder.blocks()[i].convs()[0]
        return _o(self._conv(c1, self._up_cat(i, x, skip)))

    def dec_b(self, i: int, a):
        return _o(self._conv(self.model.decoder.blocks()[i].convs()[1], _v(a)))

    def head_partials(self, x, t):
        seg = self.model.segmap
        return _HeadLoss.apply(_dense(_v(x)), seg.weight, seg.bias, t.float().contiguous())

    @torch.no_grad()
    def head_probs(self, x):
        seg = self.model.segmap
        y = _dense(_v(x))
        _, p = F32.head_fwd(y, seg.weight, seg.bias, None, want_probs=True)
        return p.view(y.shape[0], 1, y.shape[1], y.shape[2])
