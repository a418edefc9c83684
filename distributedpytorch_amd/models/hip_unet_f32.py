"""fp32 training engine on the hand-written fp32 kernels (csrc/fp32.hip, ops/fp32.py).

The reference trains in fp32 (``/root/reference/utils/train_utils.py:60-61``: fp32 model and inputs,
no autocast; model ``model/unet_parts.py`` / ``unet_model.py``).  The bf16 engine
(:class:`.hip_unet.HipBlocks`) stores bf16 activations; this engine keeps every activation, gradient
and weight in fp32 and runs every conv-shaped product on fp32 MFMA (v_mfma_f32_16x16x4_f32):

* conv3x3 + bias + ReLU forward, its dgrad (flipped weights) and weight / bias gradient;
* ConvTranspose2d(k2, s2) forward (GEMM + 2x2 scatter), dgrad (stride-2 gather GEMM) and weight /
  bias gradient;
* 2x2 max-pool with window codes and its backward, the segmentation head (1x1 conv + sigmoid +
  BCE / Dice partial sums, ``utils/utils.py:9-25``) and its backward, the NCHW -> NHWC input pass;
* the north-star variants (``model/modelsummary.txt:153-247``): Conv2d+BatchNorm+ReLU DoubleConvs (fp32 batch
  statistics, apply and backward kernels, csrc/norm_up.hip) and the bilinear Up path (x2 up-sampling
  kernels; its 1x1 projection is a plain GEMM at the low resolution).

Granularity is one autograd Function per block (a DoubleConv's two convs are one Function: the inner ReLU
backward is the mask epilogue of the second conv's dgrad).  As in the bf16 engine, parameters are not
autograd inputs: every layer's GEMM weight layouts are packed by one batched kernel per parameter update
(``ensure_packed``), and the weight / bias gradients are reduced straight into the flat fp32 gradient
buffer, each block announcing its finished parameters (``ready``: DDP buckets overlap the backward).  Activations are NHWC
tensors handed between blocks as logical-NCHW channels_last views, as in the bf16 engine.  Supported:
the reference UNet family with or without BatchNorm, transposed-conv or bilinear up-sampling, channel widths
divisible by 32 (other configurations take the stock torch path, ``compute.resolve_backend``).
"""
from __future__ import annotations

import weakref
from typing import Optional

import torch

from ..ops import fp32 as F32
from .unet import Up


def supported(model) -> bool:
    """The reference UNet family, with or without BatchNorm (Conv2d+BN+ReLU DoubleConv) and with transposed-
    conv or bilinear up-sampling, channel widths divisible by 32."""
    convs = [c for b in model.encoder.blocks() for c in b.convs()] + list(model.mid.convs()) + \
            [c for b in model.decoder.blocks() for c in b.convs()]
    ups_ok = all(isinstance(m, Up) or m.out_channels % 32 == 0 for m in model.decoder.ups())
    return all(c.out_channels % 32 == 0 for c in convs) and model.encoder.blocks()[0].convs()[0].in_channels <= 4 \
        and model.segmap.out_channels == 1 and model.segmap.in_channels in (8, 16, 32, 64) and ups_ok


def _v(t: torch.Tensor) -> torch.Tensor:
    """logical-NCHW channels_last -> NHWC view (copies only if the layout is something else)."""
    if t.dim() == 4 and t.stride(1) != 1:
        t = t.contiguous(memory_format=torch.channels_last)
    return t.permute(0, 2, 3, 1)


def _o(t: torch.Tensor) -> torch.Tensor:
    return t.permute(0, 3, 1, 2)


def _dense(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous() else t.contiguous()


def _grad(p: torch.nn.Parameter) -> torch.Tensor:
    """The parameter's gradient view in the flat fp32 buffer (optim.FlatParameterSpace): the engine's
    weight-gradient reductions accumulate straight into it (no zero-filled temporaries, no autograd add)."""
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    g = p.grad
    assert g.dtype == torch.float32 and g.is_contiguous()
    return g


class _L:
    """Packing bookkeeping of one conv3x3 / transposed-conv layer: offsets of its forward and dgrad GEMM
    weights in the engine's packed fp32 buffer."""

    def __init__(self, mod, kind: str, cs: int = 0, bn=None):
        self.mod, self.kind, self.bn = mod, kind, bn
        if kind == "conv":
            self.Cout, self.Cin = mod.out_channels, mod.in_channels
            self.Cs = cs or self.Cin
            self.Kf = F32.round_up(9 * self.Cs, 16)
            self.Nd = F32.round_up(self.Cin, 32)          # dgrad GEMM-N (zero rows for padding channels)
            self.Kd = F32.round_up(9 * self.Cout, 16)
        elif kind == "up":                                # bilinear Up: 1x1 projection (models/unet.py Up)
            self.Cin, self.Cout = mod.proj.in_channels, mod.proj.out_channels
            self.Cs, self.Kf, self.Nd, self.Kd = self.Cin, self.Cin, self.Cin, self.Cout
        else:                                             # ConvTranspose2d(k2, s2): weight [Cin, Cout, 2, 2]
            self.Cin, self.Cout = mod.in_channels, mod.out_channels
            self.Cs = self.Cin
            self.Kf, self.Nd, self.Kd = self.Cin, self.Cin, 4 * self.Cout
        self.off_f = self.off_d = -1


def _conv_fwd(B, c: _L, x, y=None, relu: bool = True):
    """relu(conv3x3(x) + b), NHWC fp32; x has ``c.Cs`` channels (>= Cin: zero weights for the padding
    channels of the network input); ``y``: the output (a channel slice allowed), else a new tensor.
    ``relu=False``: the pre-BatchNorm output z."""
    N, H, W = x.shape[:3]
    if y is None:
        y = torch.empty(N, H, W, c.Cout, dtype=torch.float32, device=x.device)
    F32.igemm(x, B.wf(c), y, Ngemm=c.Cout, Kpad=c.Kf, KH=3, KW=3, stride=1, pad=1, Cs=c.Cs, out_grid=(N, H, W),
              bias=c.mod.bias.detach(), relu=relu)
    return y


def _conv_bn_fwd(B, c: _L, x, y=None):
    """relu(bn(conv3x3(x) + b)): returns (y, z, saved) -- z the conv output, saved the BN batch statistics
    (None in eval mode: running statistics)."""
    z = _conv_fwd(B, c, x, relu=False)
    y, saved = F32.bn_fwd(z, c.bn, B.model.training, relu=True, y=y)
    return y, z, saved


def _bn_bwd(c: _L, g, z, saved):
    """dL/dz from g = dL/d(relu(bn(z))) with the ReLU mask already applied."""
    return F32.bn_bwd(_dense(g), z, saved, c.bn, _grad(c.bn.weight), _grad(c.bn.bias))


def _conv_dgrad(B, c: _L, ge, mask=None):
    """dL/dx of a conv3x3 from the pre-activation gradient ``ge``; ``mask`` = the input's own ReLU output
    (its backward applied in the epilogue)."""
    N, H, W = ge.shape[:3]
    gx = torch.empty(N, H, W, c.Nd, dtype=torch.float32, device=ge.device)
    F32.igemm(ge, B.wd(c), gx, Ngemm=c.Nd, Kpad=c.Kd, KH=3, KW=3, stride=1, pad=1, Cs=c.Cout, out_grid=(N, H, W),
              mask=mask)
    return gx[..., :c.Cs] if c.Nd != c.Cs else gx


def _conv_wgrad(B, c: _L, ge, x):
    gw, gb = _grad(c.mod.weight), _grad(c.mod.bias)
    B.side_launch(lambda: F32.wgrad(ge, x, gw, gb, KH=3, KW=3, s=1, pad=1, nreal=c.Cin), ge, x)


def _relu_masked(gy: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """ReLU backward of a block output y: a no-op for a gradient the head backward already masked by y > 0
    (the tensor carries ``_dpa_relu_masked``; any autograd accumulation returns a fresh, unmarked tensor)."""
    if getattr(gy, "_dpa_relu_masked", False):
        return gy
    return F32.relu_bwd(_dense(gy), y)


class _ConvReLU(torch.autograd.Function):
    """y = relu(conv3x3(x) + b), NHWC fp32 (one conv: the halves of a DoubleConv cut by a pipeline stage
    boundary)."""

    @staticmethod
    def forward(ctx, anchor, x, B, c):
        y = _conv_fwd(B, c, x)
        ctx.B, ctx.c = B, c
        ctx.save_for_backward(x, y)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y = ctx.saved_tensors
        B, c = ctx.B, ctx.c
        ge = _relu_masked(gy, y)
        _conv_wgrad(B, c, ge, x)
        gx = _conv_dgrad(B, c, ge) if ctx.needs_input_grad[1] else None
        B.join()
        B.ready([c.mod])
        return None, gx, None, None


class _DoubleConvReLU(torch.autograd.Function):
    """relu(conv2(relu(conv1(x)))) (reference DoubleConv without BatchNorm, model/unet_parts.py:7-15) as one
    Function: the inner ReLU's backward is the mask epilogue of conv2's dgrad, so the inner gradient is
    written once, already masked."""

    @staticmethod
    def forward(ctx, anchor, x, B, c1, c2):
        a = _conv_fwd(B, c1, x)
        y = _conv_fwd(B, c2, a)
        ctx.B, ctx.c = B, (c1, c2)
        ctx.save_for_backward(x, a, y)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, a, y = ctx.saved_tensors
        B, (c1, c2) = ctx.B, ctx.c
        ge2 = _relu_masked(gy, y)
        _conv_wgrad(B, c2, ge2, a)                 # side stream: overlaps the dgrad chain
        ge1 = _conv_dgrad(B, c2, ge2, mask=a)
        _conv_wgrad(B, c1, ge1, x)
        gx = _conv_dgrad(B, c1, ge1) if ctx.needs_input_grad[1] else None
        B.join()
        B.ready([c2.mod, c1.mod])
        return None, gx, None, None, None


class _EncBlock(torch.autograd.Function):
    """Encoder block: DoubleConv + 2x2 max-pool (reference Encoder, model/unet_parts.py:20-40) -> (skip, pooled).
    The second conv writes the skip straight into the first half of the decoder's [N,H,W,2C] concat buffer
    (registered with the engine by address; a skip leaving this pipeline stage stays dense), so the
    reference's torch.cat (unet_parts.py:59) costs no copy.  Backward: the skip gradient, the pool backward
    and the last ReLU backward form the second conv's pre-activation gradient in one pass
    (F32.enc_out_bwd); the inner ReLU as in :class:`_DoubleConvReLU`."""

    @staticmethod
    def forward(ctx, anchor, x, B, c1, c2, dense: bool):
        N, H, W = x.shape[:3]
        a = _conv_fwd(B, c1, x)
        if dense:
            own = y = torch.empty(N, H, W, c2.Cout, dtype=torch.float32, device=x.device)
        else:
            own = B.new_cat(N, H, W, c2.Cout)
            y = own[..., :c2.Cout]
        _conv_fwd(B, c2, a, y)
        pooled, code = F32.maxpool2(y)
        ctx.B, ctx.c, ctx.C = B, (c1, c2), c2.Cout
        # the concat buffer itself is saved: it keeps the engine's weak registry entry alive for the decoder
        ctx.save_for_backward(x, a, own, code)
        return y, pooled

    @staticmethod
    def backward(ctx, gs, gp):
        x, a, own, code = ctx.saved_tensors
        B, (c1, c2) = ctx.B, ctx.c
        y = own[..., :ctx.C]
        if gs is not None and not F32.nhwc_ok(gs):
            gs = gs.contiguous()
        ge2 = F32.enc_out_bwd(gs, None if gp is None else _dense(gp), code, y)
        _conv_wgrad(B, c2, ge2, a)
        ge1 = _conv_dgrad(B, c2, ge2, mask=a)
        _conv_wgrad(B, c1, ge1, x)
        gx = _conv_dgrad(B, c1, ge1) if ctx.needs_input_grad[1] else None
        B.join()
        B.ready([c2.mod, c1.mod])
        return None, gx, None, None, None, None


class _DoubleConvBN(torch.autograd.Function):
    """relu(bn2(conv2(relu(bn1(conv1(x)))))) -- the north-star DoubleConv = Conv2d+BN+ReLU twice
    (model/modelsummary.txt:153-247), training (batch statistics) or eval (running statistics).  Backward: the
    outer ReLU mask, BN2's backward, conv2's dgrad with the inner ReLU as its mask epilogue, BN1's backward,
    conv1's dgrad; weight gradients on the side stream."""

    @staticmethod
    def forward(ctx, anchor, x, B, c1, c2):
        y1, z1, s1 = _conv_bn_fwd(B, c1, x)
        y2, z2, s2 = _conv_bn_fwd(B, c2, y1)
        ctx.B, ctx.c = B, (c1, c2)
        ctx.st = (s1, s2)
        ctx.save_for_backward(x, z1, y1, z2, y2)
        return y2

    @staticmethod
    def backward(ctx, gy):
        x, z1, y1, z2, y2 = ctx.saved_tensors
        B, (c1, c2) = ctx.B, ctx.c
        s1, s2 = ctx.st
        dz2 = _bn_bwd(c2, _relu_masked(gy, y2), z2, s2)
        _conv_wgrad(B, c2, dz2, y1)
        g1 = _conv_dgrad(B, c2, dz2, mask=y1)
        dz1 = _bn_bwd(c1, g1, z1, s1)
        _conv_wgrad(B, c1, dz1, x)
        gx = _conv_dgrad(B, c1, dz1) if ctx.needs_input_grad[1] else None
        B.join()
        B.ready([c2.mod, c2.bn, c1.mod, c1.bn])
        ctx.st = None
        return None, gx, None, None, None


class _ConvBN(torch.autograd.Function):
    """relu(bn(conv3x3(x))) -- one half of a BN DoubleConv cut by a pipeline stage boundary."""

    @staticmethod
    def forward(ctx, anchor, x, B, c):
        y, z, s = _conv_bn_fwd(B, c, x)
        ctx.B, ctx.c, ctx.st = B, c, s
        ctx.save_for_backward(x, z, y)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, z, y = ctx.saved_tensors
        B, c = ctx.B, ctx.c
        dz = _bn_bwd(c, _relu_masked(gy, y), z, ctx.st)
        _conv_wgrad(B, c, dz, x)
        gx = _conv_dgrad(B, c, dz) if ctx.needs_input_grad[1] else None
        B.join()
        B.ready([c.mod, c.bn])
        ctx.st = None
        return None, gx, None, None


class _EncBlockBN(torch.autograd.Function):
    """Encoder block of the BN model: DoubleConv(+BN) + 2x2 max-pool -> (skip, pooled); the skip written into
    the decoder's concat buffer as in :class:`_EncBlock`; backward forms the last ReLU's masked gradient from
    the skip gradient and the pool backward in one pass (F32.enc_out_bwd), then the two BN + conv backwards."""

    @staticmethod
    def forward(ctx, anchor, x, B, c1, c2, dense: bool):
        N, H, W = x.shape[:3]
        y1, z1, s1 = _conv_bn_fwd(B, c1, x)
        if dense:
            own = y = torch.empty(N, H, W, c2.Cout, dtype=torch.float32, device=x.device)
        else:
            own = B.new_cat(N, H, W, c2.Cout)
            y = own[..., :c2.Cout]
        _, z2, s2 = _conv_bn_fwd(B, c2, y1, y=y)
        pooled, code = F32.maxpool2(y)
        ctx.B, ctx.c, ctx.C, ctx.st = B, (c1, c2), c2.Cout, (s1, s2)
        ctx.save_for_backward(x, z1, y1, z2, own, code)
        return y, pooled

    @staticmethod
    def backward(ctx, gs, gp):
        x, z1, y1, z2, own, code = ctx.saved_tensors
        B, (c1, c2) = ctx.B, ctx.c
        s1, s2 = ctx.st
        y = own[..., :ctx.C]
        if gs is not None and not F32.nhwc_ok(gs):
            gs = gs.contiguous()
        g2 = F32.enc_out_bwd(gs, None if gp is None else _dense(gp), code, y)
        dz2 = _bn_bwd(c2, g2, z2, s2)
        _conv_wgrad(B, c2, dz2, y1)
        g1 = _conv_dgrad(B, c2, dz2, mask=y1)
        dz1 = _bn_bwd(c1, g1, z1, s1)
        _conv_wgrad(B, c1, dz1, x)
        gx = _conv_dgrad(B, c1, dz1) if ctx.needs_input_grad[1] else None
        B.join()
        B.ready([c2.mod, c2.bn, c1.mod, c1.bn])
        ctx.st = None
        return None, gx, None, None, None, None


class _Up2(torch.autograd.Function):
    """Bilinear x2 up-sampling, align_corners=False (the variant ``Up``: models/unet.py), NHWC fp32."""

    @staticmethod
    def forward(ctx, x):
        return F32.up2_fwd(x)

    @staticmethod
    def backward(ctx, g):
        return F32.up2_bwd(_dense(g))


def _deconv_bwd(B, d: _L, x, gy, need_dx: bool):
    N, h, w, ci = x.shape
    gw, gb = _grad(d.mod.weight), _grad(d.mod.bias)

    def wgrad():
        F32.wgrad(x, gy, gw, None, KH=2, KW=2, s=2, pad=0)
        F32.channel_sum(gy, gb)

    B.side_launch(wgrad, x, gy)
    gx = None
    if need_dx:
        gx = torch.empty(N, h, w, ci, dtype=torch.float32, device=x.device)
        F32.igemm(gy, B.wd(d), gx, Ngemm=ci, Kpad=d.Kd, KH=2, KW=2, stride=2, pad=0, Cs=d.Cout, out_grid=(N, h, w))
    B.join()
    B.ready([d.mod])
    return gx


class _Deconv(torch.autograd.Function):
    """y = ConvTranspose2d(k2, s2)(x) + b, NHWC fp32 (reference model/unet_parts.py:51-54)."""

    @staticmethod
    def forward(ctx, anchor, x, B, d):
        N, h, w, ci = x.shape
        y = torch.empty(N, 2 * h, 2 * w, d.Cout, dtype=torch.float32, device=x.device)
        F32.igemm(x, B.wf(d), y, Ngemm=4 * d.Cout, Kpad=d.Kf, KH=1, KW=1, stride=1, pad=0, Cs=ci,
                  out_grid=(N, h, w), bias=d.mod.bias.detach(), mode=1, Cout=d.Cout)
        ctx.B, ctx.d = B, d
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        return None, _deconv_bwd(ctx.B, ctx.d, x, _dense(gy), ctx.needs_input_grad[1]), None, None


class _UpCat(torch.autograd.Function):
    """[skip ‖ ConvTranspose2d(k2, s2)(x) + b] in one NHWC buffer (reference concat order, skip first,
    model/unet_parts.py:58-59): the skip is already in the buffer's first half when this engine's encoder
    wrote it (one copy otherwise: a skip received from another pipeline stage); the transposed conv's
    scatter epilogue stores straight into the upper half; the backward reads both gradient halves in place."""

    @staticmethod
    def forward(ctx, anchor, x, skip, B, d):
        N, h, w, ci = x.shape
        C = skip.shape[3]
        buf = B.cat_for(skip, C + d.Cout)
        F32.igemm(x, B.wf(d), buf[..., C:], Ngemm=4 * d.Cout, Kpad=d.Kf, KH=1, KW=1, stride=1, pad=0,
                  Cs=ci, out_grid=(N, h, w), bias=d.mod.bias.detach(), mode=1, Cout=d.Cout)
        ctx.C, ctx.B, ctx.d = C, B, d
        ctx.save_for_backward(x)
        return buf

    @staticmethod
    def backward(ctx, gbuf):
        (x,) = ctx.saved_tensors
        C = ctx.C
        if not F32.nhwc_ok(gbuf):
            gbuf = gbuf.contiguous()
        gs, gy = gbuf[..., :C], gbuf[..., C:]
        gx = _deconv_bwd(ctx.B, ctx.d, x, gy, ctx.needs_input_grad[1])
        return None, gx, gs, None, None


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
    def forward(ctx, anchor, y, B, t):
        seg = B.model.segmap
        S, _ = F32.head_fwd(y, seg.weight, seg.bias, t)
        ctx.B = B
        ctx.save_for_backward(y, t)
        return S

    @staticmethod
    def backward(ctx, dS):
        y, t = ctx.saved_tensors
        seg = ctx.B.model.segmap
        # y is the last decoder block's ReLU output: its ReLU backward rides in the head backward, and the
        # block skips its relu_bwd pass for a gradient marked this way (_relu_masked)
        gy, _, _ = F32.head_bwd(y, seg.weight, seg.bias, t, dS, _grad(seg.weight).view(-1), _grad(seg.bias),
                                relu=True)
        gy._dpa_relu_masked = True
        ctx.B.ready([seg])
        return None, gy, None, None


class F32Engine:
    """Packed fp32 GEMM weights of a set of layers plus the readiness announcements: the state the
    block Functions use (``wf`` / ``wd`` / ``ready``).  :class:`HipF32Blocks` is the UNet's engine; the
    tests build one over single layers."""

    def __init__(self, layers, device, owned=None):
        self.device = torch.device(device)
        self._owned = owned
        # parameters enter no autograd graph: the Functions take this leaf so their outputs require grad,
        # and write the parameter gradients into the flat buffer themselves
        self.anchor = torch.zeros(1, device=self.device, requires_grad=True)
        self._build_packing(layers)
        self._packed_version = None
        # weight gradients on a second HIP stream (as in the bf16 engine): nothing in the backward reads
        # them, so they overlap the dgrad chain; a block's end joins the streams, then announces
        from ..ops import kernels as K
        self.side = torch.cuda.Stream(device=self.device, priority=K.SIDE_PRIORITY) if K.SIDE_WGRAD else None
        self._keep = []
        # concat buffers by the address of their first half (weak: a buffer whose skip another engine consumes
        # is not kept alive by this map)
        self._cats = weakref.WeakValueDictionary()
        self.dense_skips = set()

    def new_cat(self, N, H, W, C):
        cat = torch.empty(N, H, W, 2 * C, dtype=torch.float32, device=self.device)
        self._cats[cat.data_ptr()] = cat
        return cat

    def cat_for(self, skip: torch.Tensor, width: int) -> torch.Tensor:
        """[N,H,W,width] concat buffer whose first skip.shape[3] channels hold ``skip``: the encoder's own
        buffer when ``skip`` is its first half (zero-copy), else a new one with the skip copied in."""
        N, H, W, C = skip.shape
        cat = self._cats.pop(skip.data_ptr(), None)
        if cat is not None and tuple(cat.shape) == (N, H, W, width) and skip.stride(2) == width:
            return cat
        cat = torch.empty(N, H, W, width, dtype=torch.float32, device=self.device)
        cat[..., :C].copy_(skip)
        return cat

    def side_launch(self, fn, *keep):
        """Run ``fn`` (weight-gradient launches reading ``keep``) on the side stream; the operands stay
        referenced until :meth:`join`, so the caching allocator cannot hand their memory to the compute
        stream while the side stream still reads it."""
        if self.side is None:
            fn()
            return
        self.side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.side):
            fn()
        self._keep.extend(keep)

    def join(self):
        if self.side is not None and self._keep:
            torch.cuda.current_stream(self.device).wait_stream(self.side)
            self._keep = []

    def _build_packing(self, layers):
        """One descriptor per (layer, layout) of the layers on this device (a pipeline stage packs only its
        own); ONE batched kernel re-packs them whenever a parameter changed (``space.version``)."""
        from ..ops import kernels as K
        descs, off, max_elems, spaces = [], 0, 0, {}

        def add(mode, w, cout, cin, cs, ngemm, kpad):
            nonlocal off, max_elems
            assert w.dtype == torch.float32 and w.is_contiguous()
            descs.append(K.PackDesc(w.data_ptr(), off, mode, cout, cin, cs, ngemm, kpad))
            sp = getattr(w, "_dpa_space", None)
            if sp is not None:
                spaces[id(sp)] = sp
            start = off
            off = F32.round_up(off + ngemm * kpad, 64)
            max_elems = max(max_elems, ngemm * kpad)
            return start

        for c in layers:
            if c.kind == "up":                # bilinear Up: its 1x1 projection is a plain GEMM (torch.addmm)
                continue
            if c.mod.weight.device != self.device or (self._owned is not None and id(c.mod.weight) not in self._owned):
                continue
            if c.kind == "conv":
                c.off_f = add(0, c.mod.weight, c.Cout, c.Cin, c.Cs, c.Cout, c.Kf)
                c.off_d = add(1, c.mod.weight, c.Cout, c.Cin, c.Cout, c.Nd, c.Kd)
            else:
                c.off_f = add(2, c.mod.weight, c.Cout, c.Cin, c.Cin, 4 * c.Cout, c.Kf)
                c.off_d = add(3, c.mod.weight, c.Cout, c.Cin, c.Cout, c.Cin, c.Kd)
        self.packed = torch.zeros(max(off, 64), dtype=torch.float32, device=self.device)
        raw = bytes((K.PackDesc * len(descs))(*descs))
        # (a pipeline stage may own no conv at all, e.g. only the head: an empty table, no pack launch)
        self.descs_dev = (torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device) if raw
                          else torch.zeros(0, dtype=torch.uint8, device=self.device))
        self.ndesc, self.max_elems = len(descs), max_elems
        self.spaces = list(spaces.values())

    def ensure_packed(self):
        """Re-pack when a parameter changed (without a flat parameter space: every call)."""
        v = sum(s.version for s in self.spaces)
        if self._packed_version != v or not self.spaces:
            F32.pack_weights(self.packed, self.descs_dev, self.ndesc, self.max_elems)
            self._packed_version = v

    def wf(self, c: _L) -> torch.Tensor:
        assert c.off_f >= 0, "layer not packed on this engine's device"
        n = (4 * c.Cout if c.kind == "deconv" else c.Cout) * c.Kf
        return self.packed[c.off_f:c.off_f + n]

    def wd(self, c: _L) -> torch.Tensor:
        assert c.off_d >= 0, "layer not packed on this engine's device"
        return self.packed[c.off_d:c.off_d + c.Nd * c.Kd]

    def ready(self, mods):
        """Announce finished parameter gradients (DDP buckets start while the backward runs)."""
        by_space = {}
        for m in mods:
            if m is None:
                continue
            for p in (m.weight, m.bias):
                sp = getattr(p, "_dpa_space", None)
                if sp is not None:
                    by_space.setdefault(id(sp), (sp, []))[1].append(p)
        for sp, ps in by_space.values():
            sp.notify_ready(ps)


class HipF32Blocks(F32Engine):
    """Block backend (models.blocks protocol) of the fp32 engine."""

    name = "hip"

    def __init__(self, model, device=None, owned=None):
        from ..optim import FlatParameterSpace
        self.model = model
        device = torch.device(device) if device is not None else next(model.parameters()).device
        assert device.type == "cuda", "HipF32Blocks needs a GPU"
        assert supported(model), "fp32 HIP engine: reference UNet family (BN / bilinear variants too), widths % 32 == 0"
        if not any(hasattr(p, "_dpa_space") for p in model.parameters()):
            FlatParameterSpace(model, device=device)     # standalone use: flatten here

        def convs(b, first=False):
            bns = b.bns() if getattr(b, "batchnorm", False) else [None, None]
            return [_L(c, "conv", 4 if (first and j == 0) else 0, bn=bn) for j, (c, bn) in enumerate(zip(b.convs(), bns))]

        self.encc = [convs(b, l == 0) for l, b in enumerate(model.encoder.blocks())]
        self.midc = convs(model.mid)
        self.decc = [convs(b) for b in model.decoder.blocks()]
        self.ups = [_L(m, "up" if isinstance(m, Up) else "deconv") for m in model.decoder.ups()]
        layers = [c for cs in self.encc for c in cs] + self.midc + [c for cs in self.decc for c in cs] + self.ups
        super().__init__(layers, device, owned)

    # ------------------------------------------------------------------ block API
    def prep(self, x):
        if x.dim() == 4 and x.shape[1] <= 4 and x.dtype == torch.float32 and x.stride(1) != 1:
            return _o(F32.input_nhwc4(x))
        if x.dim() == 4 and x.stride(1) == 1 and x.shape[1] == 4:
            return x          # already converted
        return _o(F32.input_nhwc4(x.float()))

    def _conv(self, c, x):
        self.ensure_packed()
        if c.bn is not None:
            return _ConvBN.apply(self.anchor, x, self, c)
        return _ConvReLU.apply(self.anchor, x, self, c)

    def _double(self, c1, c2, x):
        self.ensure_packed()
        if c1.bn is not None:
            return _DoubleConvBN.apply(self.anchor, x, self, c1, c2)
        return _DoubleConvReLU.apply(self.anchor, x, self, c1, c2)

    def enc(self, l: int, x):
        self.ensure_packed()
        c1, c2 = self.encc[l]
        fn = _EncBlockBN if c1.bn is not None else _EncBlock
        s, p = fn.apply(self.anchor, _v(x), self, c1, c2, l in self.dense_skips)
        return _o(s), _o(p)

    def mid(self, x):
        return _o(self._double(*self.midc, _v(x)))

    def dec(self, i: int, x, skip):
        # transposed conv, reference CenterCrop of the skip (model/unet_parts.py:58-74), concat with the
        # skip first (:59), conv_block
        return _o(self._double(*self.decc[i], self._up_cat(i, x, skip)))

    # halves of a block cut between its two convs (pipeline stage boundary inside a DoubleConv)
    def enc_a(self, l: int, x):
        return _o(self._conv(self.encc[l][0], _v(x)))

    def enc_b(self, l: int, a):
        s = self._conv(self.encc[l][1], _v(a))
        return _o(s), _o(_MaxPool.apply(s))

    def mid_a(self, x):
        return _o(self._conv(self.midc[0], _v(x)))

    def mid_b(self, a):
        return _o(self._conv(self.midc[1], _v(a)))

    def _up_cat(self, i: int, x, skip):
        self.ensure_packed()
        d = self.ups[i]
        xv, sk = _v(x), _v(skip)
        if d.kind == "up":
            # bilinear Up: proj(up2(x)) == up2(proj(x)) (the interpolation weights sum to 1 and act per channel):
            # the 1x1 projection runs at the low resolution as a plain GEMM, then the up-sampling kernel
            N, h, w, ci = xv.shape
            wt = d.mod.proj.weight.view(d.mod.proj.out_channels, ci)
            low = torch.addmm(d.mod.proj.bias, _dense(xv).reshape(-1, ci), wt.t()).view(N, h, w, -1)
            up = _Up2.apply(low)
        elif tuple(sk.shape[1:3]) == (2 * xv.shape[1], 2 * xv.shape[2]) and sk.shape[3] % 4 == 0:
            return _UpCat.apply(self.anchor, xv, sk, self, d)
        else:
            up = _Deconv.apply(self.anchor, xv, self, d)
        h2, w2 = up.shape[1:3]
        if tuple(sk.shape[1:3]) != (h2, w2):
            top, left = int(round((sk.shape[1] - h2) / 2.0)), int(round((sk.shape[2] - w2) / 2.0))
            sk = sk[:, top:top + h2, left:left + w2]
        return torch.cat([sk, up], dim=3)

    def dec_a(self, i: int, x, skip):
        return _o(self._conv(self.decc[i][0], self._up_cat(i, x, skip)))

    def dec_b(self, i: int, a):
        return _o(self._conv(self.decc[i][1], _v(a)))

    def head_partials(self, x, t):
        return _HeadLoss.apply(self.anchor, _dense(_v(x)), self, t.float().contiguous())

    @torch.no_grad()
    def head_probs(self, x):
        seg = self.model.segmap
        y = _dense(_v(x))
        _, p = F32.head_fwd(y, seg.weight, seg.bias, None, want_probs=True)
        return p.view(y.shape[0], 1, y.shape[1], y.shape[2])
