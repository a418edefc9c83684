"""MI355X block backend: the UNet blocks on hand-written gfx950 kernels (NHWC bf16, fp32 accumulate).

Implements the block API of :mod:`.blocks` (``prep / enc / mid / dec / head_partials / head_probs``)
so every strategy (single device, DDP, DP, GPipe stages) runs the same kernels.  Each block is one
``torch.autograd.Function`` whose backward is an explicit, fused schedule:

* forward  conv3x3+bias+ReLU (``igemm``), the encoder's second conv writes straight into the first
  half of the decoder's concat buffer and the transposed conv into its second half, so the
  reference's ``torch.cat((skip, up), 1)`` (model/unet_parts.py:59-74) costs nothing;
* backward dgrad convs carry the ReLU-backward mask of their *input* in the epilogue, max-pool
  backward + skip-gradient add + mask is one kernel, weight gradients are split-K MFMA kernels that
  accumulate straight into the flat fp32 gradient buffer (:class:`..optim.FlatParameterSpace`) in
  PyTorch layout, and each block announces the parameters whose gradients are final
  (``space.notify_ready``) so the data-parallel all-reduce of that bucket starts while the rest of
  the backward runs.

Tensor interface: activations cross block boundaries as *logical NCHW, channels_last* bf16 tensors
(memory = NHWC), exactly what the stock-op backend produces, so the pipeline send/recv code and any
torch op work on them unchanged; internally the kernels see the NHWC view (``permute(0, 2, 3, 1)``).

Gradient convention between blocks: the gradient a block's backward *receives* for its (ReLU)
output is already multiplied by the ReLU mask (the consumer applies it in its own fused epilogue);
for the encoder skip, whose two consumers (pool, decoder concat) add up, the mask is applied once in
the fused pool-backward kernel.  Parameters stay fp32 (master weights); a single batched kernel
repacks them to bf16 GEMM layouts whenever they changed (``space.version``).

Fusions across block boundaries: the last decoder conv computes the segmentation head and the loss
partial sums in its epilogue when the segment ends in the head (``expect_target``); the
full-resolution transposed convs run their dgrad and weight gradient in one pass.

Variants (north-star DoubleConv / Up): a conv followed by BatchNorm writes its raw output z with the
batch statistics from its epilogue; the BN output relu(bn(z)) is materialised (``bn_fwd``) only where
its consumer is an LDS-DMA GEMM.  Every other consumer forms it on load from z and the per-channel
(scale, shift): the second conv of a 32/64-channel DoubleConv (``bn_on_load``), the next decoder block's
transposed conv (``_zx`` hand-over, forward and backward), the dual-input decoder conv for a skip kept as
z, and the segmentation head (forward and backward).  Backward: the BN's partial sums (sum g, sum g*y)
come from whichever kernel produces g (dx epilogues, the head / max-pool / transposed-conv backwards;
``hand_stats`` / ``take_stats``), and dz = a g + b z + c is formed in the consumer's loader (fused conv
backward, the first conv's weight gradient) -- a separate ``bn_bwd`` pass remains only in front of the
deep GEMMs.  The bilinear Up path runs its 1x1 projection at the low resolution and up-samples into the
concat half (``_Up``).
"""
from __future__ import annotations

import ctypes
import weakref
from typing import List

import torch

from ..ops import kernels as K
from ..optim import FlatParameterSpace
from .unet import UNet, Up


class _Conv:
    """Packing bookkeeping for one Conv2d(3x3, pad 1) layer (+ the BatchNorm2d that follows it in
    the BN variant: then the conv writes its raw output z and BN+ReLU is a separate fused pass)."""

    def __init__(self, mod: torch.nn.Conv2d, cin_pad: int, need_dgrad: bool, bn=None):
        self.mod = mod
        self.bn = bn
        self.Cout, self.Cin = mod.out_channels, mod.in_channels
        self.Cs = cin_pad
        self.Kf = K.round_up(9 * self.Cs, 32)        # fwd: K = 9*Cs
        self.Kd = K.round_up(9 * self.Cout, 32)      # dgrad: K = 9*Cout
        self.need_dgrad = need_dgrad
        self.off_f = self.off_d = 0


class _Deconv:
    def __init__(self, mod: torch.nn.ConvTranspose2d):
        self.mod = mod
        self.Cin, self.Cout = mod.in_channels, mod.out_channels
        self.Kf = K.round_up(self.Cin, 32)
        self.Kd = K.round_up(4 * self.Cout, 32)
        self.off_f = self.off_d = 0


class _Up:
    """Bilinear x2 + 1x1 projection (``models.unet.Up``).  Both are linear and the interpolation
    weights sum to 1, so proj(up(x)) == up(proj(x)) including the bias: the 1x1 conv runs at the LOW
    resolution (4x fewer MACs and bytes) and the up-sampling writes straight into the concat half."""

    def __init__(self, mod):
        self.mod = mod.proj
        self.Cin, self.Cout = self.mod.in_channels, self.mod.out_channels
        self.Kf = K.round_up(self.Cin, 32)
        self.Kd = K.round_up(self.Cout, 32)
        self.off_f = self.off_d = 0


class HipBlocks:
    name = "hip"

    def __init__(self, model: UNet, dtype: str = "bf16", device=None, owned=None):
        """``owned``: ids of the parameters this engine computes with (a pipeline stage's share when
        several stages live on one device); None = every parameter on ``device``."""
        cfg = model.cfg
        self._owned = owned
        if dtype != "bf16":
            raise NotImplementedError("hip backend computes in bf16 (fp32 accumulate); use --backend torch for fp32")
        self.model = model
        self.cfg = cfg
        self.depth = cfg.depth
        self.device = torch.device(device) if device is not None else next(model.parameters()).device
        assert self.device.type == "cuda", "HipBlocks needs a GPU"
        if not any(hasattr(p, "_dpa_space") for p in model.parameters()):
            FlatParameterSpace(model, device=self.device)     # standalone use: flatten here
        self.anchor = torch.zeros(1, device=self.device, requires_grad=True)
        def bns(b):
            return b.bns() if cfg.batchnorm else [None] * len(b.convs())

        self.enc_convs = [[_Conv(c, K.round_up(c.in_channels, 8) if (l == 0 and j == 0) else c.in_channels,
                                 need_dgrad=not (l == 0 and j == 0), bn=bn)
                           for j, (c, bn) in enumerate(zip(b.convs(), bns(b)))]
                          for l, b in enumerate(model.encoder.blocks())]
        self.mid_convs = [_Conv(c, c.in_channels, True, bn) for c, bn in zip(model.mid.convs(), bns(model.mid))]
        self.dec_convs = [[_Conv(c, c.in_channels, True, bn) for c, bn in zip(b.convs(), bns(b))]
                          for b in model.decoder.blocks()]
        self.deconvs = [_Up(m) if isinstance(m, Up) else _Deconv(m) for m in model.decoder.ups()]
        for convs in self.enc_convs + [self.mid_convs] + self.dec_convs:
            for c in convs:
                assert c.Cout % 32 == 0 and c.Cs % 8 == 0, "hip backend needs channel widths divisible by 32"
        self._build_packing()
        self._packed_version = None
        # concat buffers by the address of their first half; weak, so a buffer whose skip is consumed
        # by another engine (pipeline stage boundary) is not kept alive by this map
        self._cats: "weakref.WeakValueDictionary[int, torch.Tensor]" = weakref.WeakValueDictionary()
        self._target = None        # (target as given, fp32 flat copy) announced by run_segment
        self._head_cache = None    # (y ptr, target ptr, S) from the fused head epilogue
        # conv weight gradients on a second HIP stream: nothing in the backward consumes them, so a
        # block's wgrads overlap its dgrad chain (filling each kernel's tail); the block's end joins
        # the streams and only then announces its gradients (DDP buckets see finished values)
        self.side = (torch.cuda.Stream(device=self.device, priority=K.SIDE_PRIORITY)
                     if K.SIDE_WGRAD else None)
        self._side_pending = False
        self._ready_pending = []
        self._keep = []
        self._fold_cache = {}      # eval-mode BN folds: id(conv) -> (key, packed weights, bias)
        self._bn_stats_version = 0
        # encoder levels whose skip leaves this engine (pipeline stage boundary): the second conv writes
        # that skip into a dense tensor, which then goes on the wire as is (no concat-half copy)
        self.dense_skips = set()
        self._fusable = {}
        self._head_pending = None   # (placeholder grad, y, target, dS): head backward deferred to the decoder
        # gradients whose producer also wrote the consumer BatchNorm's backward partial sums (the head and
        # the fused transposed-conv backward): data_ptr -> (shape, stride, (slab, rows)); see take_stats
        self._stats_hand = {}
        # decoder outputs handed to the next decoder block as their BatchNorm input z (run_segment sets
        # next_dec_local when that block follows in the same segment): z data_ptr -> (z, coef)
        # skip_z_levels: encoder levels whose skip may be kept as that BN's input z (run_segment: the
        # consuming decoder level runs in the same call and the skip is not sent)
        self.next_dec_local = False
        self.skip_z_levels = set()
        self._zx = {}
        # pipeline microbatches: the side-stream conv weight gradients of every microbatch are deferred
        # and run as ONE launch per layer over all microbatches' images (K.wgrad_multi) -- one split-K
        # slab set and reduction per step instead of one per microbatch.  Flushed at the end of the
        # autograd backward (queue_callback), or by the pipeline when it opened a window (GPipeDist
        # back-propagates microbatch by microbatch); readiness announcements wait for the flush.
        self.defer_wgrad = 0          # microbatches per step whose weight gradients are merged (0/1: off)
        self._defer_window = False
        self._deferred = {}
        self._deferred_ready = []
        self._flush_queued = False
        # early_ready (set by a strategy whose reducer listens): per-module announcement as soon as the last
        # microbatch's contribution is issued, instead of all at flush_wgrad
        self.early_ready = False
        self._ready_count, self._seen_mods, self._announced = {}, {}, set()
        self.side2 = None             # stream of the merged (all-microbatch) weight-gradient launches
        self._keep2 = []              # (event after the launch, its operands): released once the event is done
        # memory bound of the deferral: a layer's deferred gradients and inputs stay alive
        # until its merged launch, so when the not-yet-launched operands of all layers exceed this many
        # bytes, the layer that crossed it launches over the microbatches it has (a partial merge)
        self.defer_cap_bytes = 8 << 30
        self._deferred_bytes = 0
        self.n_multi_launches = 0     # merged weight-gradient launches so far (tests / tools/defer_mem.py)
        self.peak_deferred_bytes = 0

    # ------------------------------------------------------------------ weight packing
    def _build_packing(self):
        """One descriptor per (layer, layout) for the layers whose weights live on this device (a
        pipeline stage packs only its own); the pack kernel reads the fp32 weights in place."""
        descs: List[K.PackDesc] = []
        off = 0
        max_elems = 0
        spaces = {}

        def add(mode, w, cout, cin, cs, ngemm, kpad):
            nonlocal off, max_elems
            assert w.dtype == torch.float32 and w.is_contiguous()
            descs.append(K.PackDesc(w.data_ptr(), off, mode, cout, cin, cs, ngemm, kpad))
            sp = getattr(w, "_dpa_space", None)
            if sp is not None:
                spaces[id(sp)] = sp
            start = off
            off = K.round_up(off + ngemm * kpad, 64)
            max_elems = max(max_elems, ngemm * kpad)
            return start

        here = lambda m: (m.weight.device == self.device   # noqa: E731
                          and (self._owned is None or id(m.weight) in self._owned))
        for c in [c for cs in self.enc_convs for c in cs] + self.mid_convs + [c for cs in self.dec_convs for c in cs]:
            if not here(c.mod):
                continue
            c.off_f = add(0, c.mod.weight, c.Cout, c.Cin, c.Cs, c.Cout, c.Kf)
            if c.need_dgrad:
                c.off_d = add(1, c.mod.weight, c.Cout, c.Cin, c.Cout, c.Cin, c.Kd)
        for d in self.deconvs:
            if not here(d.mod):
                continue
            if isinstance(d, _Up):
                d.off_f = add(4, d.mod.weight, d.Cout, d.Cin, d.Cin, d.Cout, d.Kf)
                d.off_d = add(5, d.mod.weight, d.Cout, d.Cin, d.Cout, d.Cin, d.Kd)
            else:
                d.off_f = add(2, d.mod.weight, d.Cout, d.Cin, d.Cin, 4 * d.Cout, d.Kf)
                d.off_d = add(3, d.mod.weight, d.Cout, d.Cin, d.Cout, d.Cin, d.Kd)
        self.packed = torch.zeros(max(off, 64), dtype=torch.bfloat16, device=self.device)
        raw = bytes((K.PackDesc * len(descs))(*descs))
        # (a pipeline stage may own no conv at all, e.g. only the head: an empty table, no pack launch)
        self.descs_dev = (torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device) if raw
                          else torch.zeros(0, dtype=torch.uint8, device=self.device))
        self.ndesc = len(descs)
        self.max_elems = max_elems
        self.spaces = list(spaces.values())
        # parameter data pointers the descriptors captured (re-pack layout if a param is re-bound)
        self._ptrs = [d.src for d in descs]

    def ensure_packed(self):
        v = sum(s.version for s in self.spaces)
        if self._packed_version != v:
            K.pack_weights(self.packed, self.descs_dev, self.ndesc, self.max_elems)
            self._packed_version = v

    def wf(self, c):
        return self.packed[c.off_f:c.off_f + (4 * c.Cout if isinstance(c, _Deconv) else c.Cout) * c.Kf]

    def wd(self, c):
        return self.packed[c.off_d:c.off_d + c.Cin * c.Kd]

    # ------------------------------------------------------------------ primitive launches
    def bn_on_load(self, c1: _Conv, c2: _Conv, H: int, W: int) -> bool:
        """DoubleConv conv1 -> BN -> ReLU -> conv2 -> BN at the 32/64-channel levels (training): conv1
        stops at its pre-BN output z (statistics from its epilogue, :meth:`conv_bn_z`) and conv2 forms
        relu(bn(z)) in its row-streaming loader, forward and fused backward (``xbn``).  The BN output
        of conv1 -- a full-resolution tensor per DoubleConv -- is never written, read or kept."""
        if not (K.USE_BN_ON_LOAD and K.USE_STREAM and K.USE_FUSED_BN and self.model.training):
            return False
        if c1.bn is None or c2.bn is None or not (c2.Cs == c2.Cin == c1.Cout and c2.Cin in (32, 64)
                                                  and c2.Cout in (32, 64)):
            return False
        # the row-streaming conv binds one image per block: z's image within the 32-bit buffer range
        return H * W * c2.Cin * 2 < K._MAX_BYTES and self.fusable(c2, c1, W)

    def conv_bn_z(self, c: _Conv, x: torch.Tensor, st: list, xbn: torch.Tensor = None, x2: torch.Tensor = None):
        """Training conv + BatchNorm statistics without the normalise pass: returns (z, coef) with the
        consumer's on-load transform relu(z * coef[c] + coef[C + c]); ``st`` receives (z, saved, coef).
        ``xbn``: x is itself a pre-BN output, read as relu(bn(x)) (:meth:`conv_fwd`); ``x2``: dual input."""
        N, H, W = x.shape[:3]
        z = torch.empty(N, H, W, c.Cout, dtype=torch.bfloat16, device=x.device)
        self._bn_stats_version += 1
        stats = []
        K.igemm(x, self.wf(c), z, Ngemm=c.Cout, Kpad=c.Kf, KH=3, KW=3, stride=1, pad=1, Cs=c.Cs, out_grid=(N, H, W),
                bias=c.mod.bias, relu=False, bn_stats=stats, xbn=xbn, x2=x2)
        coef = []
        saved = K.bn_fwd(z, None, c.bn, train=True, stats=stats, coef_out=coef)
        st.append((z, saved, coef[0]))
        return z, coef[0]

    def conv_bn_z_pool(self, c: _Conv, x: torch.Tensor, st: list, pool: torch.Tensor, pcode: torch.Tensor,
                       xbn: torch.Tensor = None):
        """:meth:`conv_bn_z` that also writes the 2x2 max-pool of relu(bn(z)) and its window codes (one
        normalise pass over z that stores only the pooled quarter): returns (z, coef)."""
        N, H, W = x.shape[:3]
        z = torch.empty(N, H, W, c.Cout, dtype=torch.bfloat16, device=x.device)
        self._bn_stats_version += 1
        stats = []
        K.igemm(x, self.wf(c), z, Ngemm=c.Cout, Kpad=c.Kf, KH=3, KW=3, stride=1, pad=1, Cs=c.Cs, out_grid=(N, H, W),
                bias=c.mod.bias, relu=False, bn_stats=stats, xbn=xbn)
        coef = []
        saved = K.bn_fwd(z, None, c.bn, train=True, stats=stats, pool=pool, pcode=pcode, coef_out=coef)
        st.append((z, saved, coef[0]))
        return z, coef[0]

    def conv_fwd(self, c: _Conv, x: torch.Tensor, y: torch.Tensor = None, pool: torch.Tensor = None,
                 pcode: torch.Tensor = None, st: list = None, x2: torch.Tensor = None, xbn: torch.Tensor = None):
        """relu(conv(x)) -> y (and its 2x2 max-pool + window codes).  BN variant: the conv writes z,
        then one statistics pass + one normalise/ReLU pass; ``st`` receives (z, saved, coef) for the backward.
        ``x2``: dual input, the conv reads [x | x2] (:meth:`dual_level`).  ``xbn``: ``x`` is the layer
        below's pre-BN output and the conv reads relu(bn(x)) (:meth:`bn_on_load`)."""
        if self._stats_hand:                 # a forward: last backward's unconsumed hand-overs go
            self._stats_hand.clear()
        N, H, W = x.shape[:3]
        if y is None:
            y = torch.empty(N, H, W, c.Cout, dtype=torch.bfloat16, device=x.device)
        if c.bn is None:
            K.igemm(x, self.wf(c), y, Ngemm=c.Cout, Kpad=c.Kf, KH=3, KW=3, stride=1, pad=1, Cs=c.Cs,
                    out_grid=(N, H, W), bias=c.mod.bias, relu=True, pool=pool, pcode=pcode, x2=x2)
            return y
        assert x2 is None or self.model.training, "dual input with BatchNorm: training forward (dual_level)"
        assert xbn is None or self.model.training, "BN-on-load: training forward"
        if not self.model.training and K.FOLD_BN_EVAL and c.bn.track_running_stats and c.bn.running_mean is not None:
            # inference: BatchNorm with running statistics is a per-channel affine map -> folded into
            # the conv's weights and bias, so Conv2d+BN+ReLU(+pool) is ONE fused kernel, as without BN
            wpk, bias = self._folded(c)
            K.igemm(x, wpk, y, Ngemm=c.Cout, Kpad=c.Kf, KH=3, KW=3, stride=1, pad=1, Cs=c.Cs,
                    out_grid=(N, H, W), bias=bias, relu=True, pool=pool, pcode=pcode)
            return y
        z = torch.empty(N, H, W, c.Cout, dtype=torch.bfloat16, device=x.device)
        if self.model.training:
            self._bn_stats_version += 1                 # running statistics move (eval fold cache)
        stats = [] if self.model.training else None    # batch statistics from the conv epilogue
        K.igemm(x, self.wf(c), z, Ngemm=c.Cout, Kpad=c.Kf, KH=3, KW=3, stride=1, pad=1, Cs=c.Cs, out_grid=(N, H, W),
                bias=c.mod.bias, relu=False, bn_stats=stats, xbn=xbn, x2=x2)
        coef = [] if self.model.training else None     # (scale, shift): consumers may re-form y from z
        saved = K.bn_fwd(z, y, c.bn, train=self.model.training, stats=stats, pool=pool, pcode=pcode, coef_out=coef)
        if st is not None:
            st.append((z, saved, coef[0] if coef else None))
        return y

    @torch.no_grad()
    def _folded(self, c: _Conv):
        """(packed bf16 weights, fp32 bias) of conv ``c`` with its eval-mode BatchNorm folded in:
        W' = W * s, b' = (b - running_mean) * s + beta, s = gamma / sqrt(running_var + eps).  Recomputed
        Cached until the weights (flat-space version), the running statistics (a training-mode forward
        of this engine, or an in-place write such as load_state_dict) or the affine parameters change."""
        bn = c.bn
        key = (self._packed_version, self._bn_stats_version, bn.running_mean._version, bn.running_var._version,
               bn.weight._version, bn.bias._version)
        hit = self._fold_cache.get(id(c))
        if hit is not None and hit[0] == key:
            return hit[1], hit[2]
        scale = bn.weight.float() / torch.sqrt(bn.running_var.float() + bn.eps)
        w = (c.mod.weight.float() * scale.view(-1, 1, 1, 1)).contiguous()
        b0 = c.mod.bias.float() if c.mod.bias is not None else torch.zeros_like(scale)
        bias = ((b0 - bn.running_mean.float()) * scale + bn.bias.float()).contiguous()
        packed = torch.zeros(c.Cout * c.Kf, dtype=torch.bfloat16, device=w.device)
        d = K.PackDesc(w.data_ptr(), 0, 0, c.Cout, c.Cin, c.Cs, c.Cout, c.Kf)
        descs = torch.frombuffer(bytearray(bytes(d)), dtype=torch.uint8).to(w.device)
        K.pack_weights(packed, descs, 1, c.Cout * c.Kf)
        self._fold_cache[id(c)] = (key, packed, bias)
        return packed, bias

    def hand_stats(self, g: torch.Tensor, stats):
        """``g`` (about to be returned to autograd) comes with the partial sums (sum g, sum g*y) of the
        BatchNorm whose output y it is the gradient of: the consumer's backward takes them (take_stats).
        The entry holds ``g`` itself, so its memory cannot be reused by another tensor that would then
        match; entries left unconsumed (e.g. a gradient sent to another pipeline stage) are dropped at the
        next forward (conv_fwd)."""
        if stats:
            self._stats_hand[g.data_ptr()] = (g, stats)

    def take_stats(self, g: torch.Tensor):
        """The partial sums handed over with this very tensor (same storage, shape and strides), or None."""
        e = self._stats_hand.pop(g.data_ptr(), None)
        return e[1] if e is not None and e[0].shape == g.shape and e[0].stride() == g.stride() else None

    def bn_bwd(self, c: _Conv, g: torch.Tensor, st, stats: list = None):
        """gradient w.r.t. the conv output: identity without BN, BatchNorm backward with it (``stats``:
        the (sum g, sum g*y) partials the dgrad producing g computed in its epilogue, if any)."""
        if c.bn is None:
            return g
        z, saved = st[:2]
        return K.bn_bwd(g, z, saved, c.bn, _grad(c.bn.weight), _grad(c.bn.bias), stats=stats)

    def conv_dgrad(self, c: _Conv, g: torch.Tensor, mask: torch.Tensor = None, out: torch.Tensor = None,
                   below: _Conv = None):
        """dgrad of ``c`` (ReLU-masked by ``mask``).  ``below``: the conv whose output ``mask`` is; if it
        has a BatchNorm, returns (dx, stats) with that BN's backward partial sums from the epilogue."""
        N, H, W = g.shape[:3]
        if out is None:
            out = torch.empty(N, H, W, c.Cin, dtype=torch.bfloat16, device=g.device)
        stats = [] if (below is not None and below.bn is not None) else None
        # a persistent GEMM grid assumes it owns every CU; with side-stream weight gradients in flight
        # it would wait for them (profiles/hip_b256_512_timeline_r02_end.txt: 3.0-3.3 ms vs 0.4-0.8 alone)
        K.igemm(g, self.wd(c), out, Ngemm=c.Cin, Kpad=c.Kd, KH=3, KW=3, stride=1, pad=1, Cs=c.Cout,
                out_grid=(N, H, W), mask=mask, bn_stats=stats, persistent=not self._side_busy())
        return out if below is None else (out, stats)

    def conv_dgrad_split(self, c: _Conv, g: torch.Tensor, split: int):
        """dgrad of a conv over a concat input, written as two dense tensors (channels < split, >= split):
        the skip gradient and the up-path gradient are then read at full cache-line efficiency by the
        max-pool backward and the transposed-conv backward (interleaved halves cost ~1.6x there)."""
        N, H, W = g.shape[:3]
        lo = torch.empty(N, H, W, split, dtype=torch.bfloat16, device=g.device)
        hi = torch.empty(N, H, W, c.Cin - split, dtype=torch.bfloat16, device=g.device)
        K.igemm(g, self.wd(c), lo, Ngemm=c.Cin, Kpad=c.Kd, KH=3, KW=3, stride=1, pad=1, Cs=c.Cout,
                out_grid=(N, H, W), y2=hi, split=split, persistent=not self._side_busy())
        return lo, hi

    def _side_busy(self) -> bool:
        """Weight gradients may be in flight on a side stream: the per-block one, or the merged
        (all-microbatch) launches of a pipeline stage on ``side2`` (held in ``_keep2`` until flushed)."""
        return self._side_pending or bool(self._keep2)

    def _side_launch(self, fn, *keep: torch.Tensor):
        """Run ``fn`` (a weight-gradient launch reading ``keep``) on the side stream when there is one:
        weight gradients are off the critical path (nothing in the backward reads them before the
        optimizer), so they overlap the dgrad chain of the compute stream."""
        if self.side is None:
            fn()
            return
        self.side.wait_stream(torch.cuda.current_stream(self.device))    # the operands are ready
        with torch.cuda.stream(self.side):
            fn()
        # keep the operands alive until join(): once the compute stream has waited for the side stream
        # their memory is reused in order (record_stream would instead hold the blocks out of the
        # caching allocator until an event query, forcing fresh allocations every step: measured 8x slower)
        self._keep.extend(keep)
        self._side_pending = True

    def fusable(self, c: _Conv, below, W: int, whole: bool = False) -> bool:
        """The fused backward (dgrad + weight/bias gradient in one pass, csrc/bwd_stream.hip) serves
        this conv: 32/64 channels in and out, image rows a multiple of the kernel's pixel strip.  A
        BatchNorm after the conv (its backward formed on load) or below it (its statistics from the dx
        epilogue) needs the plain modes (:meth:`bwd_conv`); the pool / head folds (``whole``) do not
        combine with BatchNorm."""
        if not (K.USE_FUSED_BWD and bn_combo_ok(c.bn is not None, None if below is None else below.bn is not None,
                                                K.USE_FUSED_BN_BWD and not whole) and c.Cs == c.Cin):
            return False
        key = (c.Cin, c.Cout, W, whole)
        ok = self._fusable.get(key)
        if ok is None:
            ok = self._fusable[key] = K.bwd_fused_eligible(c.Cin, c.Cout, W, whole=whole)
        return ok

    def conv_bwd(self, c: _Conv, g, x: torch.Tensor, mask: bool, split: int = 0, head=None, pool=None, first=None,
                 sink=None):
        """Fused backward of ``c``: returns dx (ReLU-masked by ``x`` when ``mask``; with ``split`` the
        two dense halves of a concat gradient) and accumulates the weight and bias gradients.
        ``head``: ``g`` is the conv output and the segmentation-head backward is folded in; ``pool``:
        ``g`` is the skip gradient and the max-pool backward is folded in; ``first`` = (conv c1, its
        input x1): ``x = relu(c1(x1))`` and x1 needs no gradient, so dx is consumed in-kernel by
        c1's weight/bias gradient and never stored (returns None).  ``sink`` (:class:`K.SlabSink`): the weight
        gradient slab rows go there, reduced by the sink's owner."""
        if first is not None:
            c1, x1 = first
            w1 = (x1, _grad(c1.mod.weight).view(-1), _grad(c1.mod.bias))
            return K.conv_bwd_fused(g, x, self.wd(c), c.Kd, _grad(c.mod.weight).view(-1), _grad(c.mod.bias),
                                    mask=True, pool=pool, w1=w1)
        gw, gb = _grad(c.mod.weight).view(-1), _grad(c.mod.bias)
        if split:
            N, H, W = x.shape[:3]
            hi = torch.empty(N, H, W, c.Cin - split, dtype=torch.bfloat16, device=x.device)
            return K.conv_bwd_fused(g, x, self.wd(c), c.Kd, gw, gb, mask=False, dx2=hi, split=split)
        return K.conv_bwd_fused(g, x, self.wd(c), c.Kd, gw, gb, mask=mask, head=head, pool=pool, sink=sink)

    def bwd_conv(self, c: _Conv, g: torch.Tensor, x: torch.Tensor, st, *, mask: bool, below: _Conv = None,
                 stats: list = None, split: int = 0, x2: torch.Tensor = None, xbn: torch.Tensor = None):
        """Fused backward of ``c`` (:meth:`fusable`) when ``g`` is the gradient of its output -- of its
        BatchNorm+ReLU output if it has one (``st`` = that BN's saved (z, mean/invstd), ``stats`` = the
        BN's backward partial sums from whoever produced ``g``, if any): the BN backward is formed in the
        kernel's loader from per-channel coefficients, so neither dz nor a BN pass over HBM exists.
        Returns (dx -- or the (lo, hi) halves with ``split`` --, st_g) with st_g the BatchNorm partial
        sums of ``below`` (its ReLU output is ``x``, the dx mask) or None."""
        gw, gb = _grad(c.mod.weight).view(-1), _grad(c.mod.bias)
        bn = None
        if c.bn is not None:
            z, saved = st[:2]
            bn = (z, K.bn_bwd_coef(g, z, saved, c.bn, _grad(c.bn.weight), _grad(c.bn.bias), stats=stats))
        want = below is not None and below.bn is not None
        dx2 = None
        if split:
            N, H, W = x.shape[:3]
            dx2 = torch.empty(N, H, W, c.Cin - split, dtype=torch.bfloat16, device=x.device)
        res = K.conv_bwd_fused(g, x, self.wd(c), c.Kd, gw, gb, mask=mask, dx2=dx2, split=split, bn=bn, bn_stats=want,
                               x2=x2, xbn=xbn)
        return res if want else (res, None)

    def bwd_conv_head_bn(self, c: _Conv, z: torch.Tensor, x: torch.Tensor, st, t, dS, hprob, ycoef, *,
                         xbn: torch.Tensor = None, stats: list = None):
        """Fused backward of the last decoder conv of a BN model with the head folded in: ``z`` is its BN
        input (= st[0]), ``ycoef`` that BN's forward (scale, shift); the kernel forms the head gradient of
        relu(bn(z)) from ``hprob`` / ``t`` / ``dS`` and the BN backward (partial sums ``stats`` from the head
        statistics pass) on load.  Returns (dx, BN partial sums of the layer below)."""
        gw, gb = _grad(c.mod.weight).view(-1), _grad(c.mod.bias)
        z = st[0]                          # the saved BN input (the head's copy of it is the same storage)
        coef3 = K.bn_bwd_coef(z, z, st[1], c.bn, _grad(c.bn.weight), _grad(c.bn.bias), stats=stats)
        seg = self.model.segmap
        return K.conv_bwd_fused(z, x, self.wd(c), c.Kd, gw, gb, mask=True,
                                head=(t, seg.weight, seg.bias, dS, None, None, hprob), bn=(z, coef3), bn_stats=True,
                                xbn=xbn, ybn=ycoef)

    def halves_fusable(self, c: _Conv, C: int, W: int) -> bool:
        """A conv over a concat of two C-channel halves whose fused backward does not exist at 2C input
        channels but does at C (the 256^2 decoder conv 128 -> 64): conv(cat) = conv_lo(skip) +
        conv_hi(up), so its backward is two fused passes, one per half."""
        if not (K.USE_FUSED_HALVES and (c.bn is None or (K.BN_HALVES and K.USE_FUSED_BN_BWD))
                and c.Cs == c.Cin == 2 * C):
            return False
        key = ("halves", C, c.Cout, W)
        ok = self._fusable.get(key)
        if ok is None:
            ok = self._fusable[key] = K.bwd_fused_eligible(C, c.Cout, W)
        return ok

    def dual_level(self, l: int, H: int, W: int) -> bool:
        """Encoder level ``l`` and its decoder conv run WITHOUT a concat buffer: the skip and the
        up-sampled half are two dense [N,H,W,32] tensors and the decoder's first conv (forward: the
        row-streaming kernel; backward: the fused one) reads its 64 input channels from both (their
        ``x2`` dual input).  Every write of either half is then a whole-cache-line store -- the skip
        from the encoder conv's epilogue, the up half from the transposed conv -- instead of a 64-B half
        of each 128-B concat pixel (the full-resolution level's stores ran at ~2/3 of the HBM rate)."""
        if not (K.USE_STREAM and K.USE_DUAL_INPUT):
            return False
        d = len(self.dec_convs)
        if not 0 <= l < d:
            return False
        c1 = self.dec_convs[d - 1 - l][0]
        if not ((c1.bn is None or (K.BN_DUAL and self.model.training)) and c1.Cs == c1.Cin == 64
                and self.enc_convs[l][1].Cout == 32):
            return False
        # both kernels bind one image per block: each [H,W,32] image within the 32-bit buffer range
        return W >= 16 and H * W * 32 * 2 < K._MAX_BYTES and self.fusable(c1, None, W)

    def conv_bwd_halves(self, c: _Conv, g: torch.Tensor, cat: torch.Tensor, C: int, bn=None):
        """Backward of a conv over ``cat = [lo | hi]`` (C channels each) as two fused passes: each
        writes its half's dense input gradient and its half of the weight gradient (the dgrad rows of
        the packed weights and the input-channel columns of dW belonging to that half); the bias
        gradient comes with the first.  Replaces one 2C-channel dgrad + a side-stream weight gradient
        that together did ~1.7x the work at a third of the MFMA rate (profiles/kbench_halo_b256_r02.txt).
        ``bn`` = (z, coef3): the conv is followed by BatchNorm + ReLU and ``g`` is the gradient of its
        output; both passes form dz on load (:func:`K.conv_bwd_fused` ``bn``)."""
        gw, gb = _grad(c.mod.weight).view(c.Cout, c.Cin, 9), _grad(c.mod.bias)
        wd = self.wd(c)
        outs = []
        for h in range(2):
            part = torch.zeros(c.Cout * C * 9, dtype=torch.float32, device=g.device)
            outs.append(K.conv_bwd_fused(g, cat[..., h * C:(h + 1) * C], wd[h * C * c.Kd:(h + 1) * C * c.Kd], c.Kd,
                                         part, gb if h == 0 else None, mask=False, bn=bn))
            gw[:, h * C:(h + 1) * C].add_(part.view(c.Cout, C, 9))
        return outs[0], outs[1]

    def head_bwd_foldable(self, W: int) -> bool:
        """The head backward can be folded into the last decoder conv's fused backward."""
        c1, c2 = self.dec_convs[-1]
        return (K.USE_FUSED_HEAD_BWD and c2.Cin == 32 and c2.Cout == 32 and self.model.segmap.out_channels == 1
                and self.fusable(c2, c1, W, whole=True))

    def conv_wgrad(self, c: _Conv, g: torch.Tensor, x: torch.Tensor, gbn=None, sink=None):
        """Weight + bias gradient of ``c`` (side stream).  ``gbn`` = (z, coef3): ``g`` is the gradient of
        c's BatchNorm+ReLU output and dz is formed on load (:func:`K.wgrad` ``abn``; first conv only).
        ``sink`` (:class:`K.SlabSink`): slab rows only; the caller reduces (:meth:`sink_reduce`)."""
        N, H, W = g.shape[:3]
        if sink is not None:
            gw, gb = _grad(c.mod.weight), _grad(c.mod.bias)
            self._side_launch(lambda: K.wgrad(g, x, kind=0, grid=(N, H, W), M=c.Cout, Nc=c.Cs, s=1, pad=1, KW=3,
                                              gw=gw.view(-1), gb=gb, Nreal=c.Cin, sink=sink), g, x)
            return
        if gbn is not None:
            gw, gb = _grad(c.mod.weight), _grad(c.mod.bias)
            self._side_launch(lambda: K.wgrad(g, x, kind=0, grid=(N, H, W), M=c.Cout, Nc=c.Cs, s=1, pad=1, KW=3,
                                              gw=gw.view(-1), gb=gb, Nreal=c.Cin, abn=gbn), g, x, *gbn)
            return
        if self.defer_wgrad > 1 and K.wgrad_multi_eligible(c.Cout, c.Cs, W):
            self._release_done()
            ent = self._deferred.setdefault(id(c), (c, [], []))
            ent[1].append(g)
            ent[2].append(x)
            self._deferred_bytes += _nbytes(g) + _nbytes(x)
            self.peak_deferred_bytes = max(self.peak_deferred_bytes, self._deferred_bytes)
            if len(ent[1]) >= self.defer_wgrad:
                # every microbatch of this layer is in: launch now, so it overlaps the rest of the backward
                self._launch_deferred(id(c))
            # memory cap: launch the layers holding the most deferred bytes until the total is
            # back under the cap -- not only the one that crossed it, which would leave the others over the
            # cap and turn every later weight gradient into a per-microbatch launch
            while self._deferred_bytes > self.defer_cap_bytes and self._deferred:
                self._launch_deferred(max(self._deferred, key=lambda k: sum(
                    _nbytes(t) for t in self._deferred[k][1] + self._deferred[k][2])))
            if not self._defer_window and not self._flush_queued:
                # end of this backward: leftovers, the merged stream's join, the readiness announcements
                torch.autograd.Variable._execution_engine.queue_callback(self.flush_wgrad)
                self._flush_queued = True
            return
        gw, gb = _grad(c.mod.weight), _grad(c.mod.bias)
        self._side_launch(lambda: K.wgrad(g, x, kind=0, grid=(N, H, W), M=c.Cout, Nc=c.Cs, s=1, pad=1, KW=3,
                                          gw=gw.view(-1), gb=gb, Nreal=c.Cin), g, x)

    def sink_reduce(self, sink):
        """Reduce a side-stream :class:`K.SlabSink` on the side stream (after every launch that fed it)."""
        self._side_launch(sink.reduce)

    def join(self):
        """End of a block's backward: the compute stream waits for the side-stream weight gradients,
        then the block's parameters are announced ready."""
        if self._side_pending:
            torch.cuda.current_stream(self.device).wait_stream(self.side)
            self._side_pending = False
            self._keep = []
        pending, self._ready_pending = self._ready_pending, []
        if pending:
            self._notify(pending)

    def deconv_fwd(self, d: _Deconv, x: torch.Tensor, out: torch.Tensor, xbn: torch.Tensor = None):
        """``xbn``: ``x`` is the level below's BatchNorm input z, read as relu(bn(z)) (fused shapes only)."""
        N, h, w = x.shape[:3]
        if xbn is not None:
            K.deconv_fwd_fused(x, self.wf(d), d.mod.bias, out, xbn=xbn)
            return
        if isinstance(d, _Up):
            low = torch.empty(N, h, w, d.Cout, dtype=torch.bfloat16, device=x.device)
            K.igemm(x, self.wf(d), low, Ngemm=d.Cout, Kpad=d.Kf, KH=1, KW=1, stride=1, pad=0, Cs=d.Cin,
                    out_grid=(N, h, w), bias=d.mod.bias)
            K.up2_fwd(low, out)
            return
        if K.USE_FUSED_DECONV and (d.Cin, d.Cout) in K.DECONV_BWD_SHAPES:
            K.deconv_fwd_fused(x, self.wf(d), d.mod.bias, out)
            return
        K.igemm(x, self.wf(d), out, Ngemm=4 * d.Cout, Kpad=d.Kf, KH=1, KW=1, stride=1, pad=0, Cs=d.Cin,
                out_grid=(N, h, w), bias=d.mod.bias, mode=1, Cout=d.Cout)

    def deconv_dgrad(self, d: _Deconv, gup: torch.Tensor, x: torch.Tensor):
        N, h, w = x.shape[:3]
        dx = torch.empty(N, h, w, d.Cin, dtype=torch.bfloat16, device=x.device)
        if isinstance(d, _Up):   # gup is the low-resolution gradient here (see _DecFn.backward)
            K.igemm(gup, self.wd(d), dx, Ngemm=d.Cin, Kpad=d.Kd, KH=1, KW=1, stride=1, pad=0, Cs=d.Cout,
                    out_grid=(N, h, w), mask=x)
            return dx
        K.igemm(gup, self.wd(d), dx, Ngemm=d.Cin, Kpad=d.Kd, KH=2, KW=2, stride=2, pad=0, Cs=d.Cout,
                out_grid=(N, h, w), mask=x, persistent=not self._side_busy())
        return dx

    def deconv_wgrad(self, d: _Deconv, gup: torch.Tensor, x: torch.Tensor):
        N, h, w = x.shape[:3]
        gw, gb = _grad(d.mod.weight).view(-1), _grad(d.mod.bias)
        if isinstance(d, _Up):
            self._side_launch(lambda: K.wgrad(gup, x, kind=2, grid=(N, h, w), M=d.Cout, Nc=d.Cin, s=1, pad=0, KW=1,
                                              gw=gw, gb=gb, Nreal=d.Cin), gup, x)
            return
        self._side_launch(lambda: K.wgrad(gup, x, kind=1, grid=(N, h, w), M=d.Cout, Nc=d.Cin, s=2, pad=0, KW=2,
                                          gw=gw, gb=gb, Nreal=d.Cin), gup, x)

    def deconv_bwd(self, d, gup: torch.Tensor, x: torch.Tensor, xbn: torch.Tensor = None) -> torch.Tensor:
        """dgrad + weight gradient of the up-path layer; the full-resolution transposed convs run
        both in one pass over (gup, x) (csrc/deconv.hip).  Elsewhere the weight gradient goes to the
        side stream first, then the dgrad runs on the compute stream.  ``xbn``: as :meth:`deconv_fwd`."""
        if isinstance(d, _Deconv) and K.USE_FUSED_DECONV and (d.Cin, d.Cout) in K.DECONV_BWD_SHAPES:
            # x is the BatchNorm+ReLU output of the level below (a BN model): its BN's backward partial sums
            # come from this kernel's dx epilogue
            stats = [] if (xbn is not None or (self.enc_convs[0][1].bn is not None and K.BN_SUMS_DECONV)) else None
            dx = K.deconv_bwd_fused(gup, x, self.wd(d), _grad(d.mod.weight).view(-1), _grad(d.mod.bias),
                                    bn_stats=stats, xbn=xbn)
            self.hand_stats(dx, stats)
            return dx
        self.deconv_wgrad(d, gup, x)
        return self.deconv_dgrad(d, gup, x)

    def ready(self, mods):
        if self.defer_wgrad > 1 and (self._deferred or self._defer_window or self._flush_queued):
            if not self.early_ready:
                self._deferred_ready.extend(mods)   # final only after flush_wgrad
                return
            # a data-parallel reducer listens (pipelines x replicas): announce a module as soon as its last
            # microbatch's contribution is issued -- its buckets' all-reduces then overlap the rest of the
            # stage's backward instead of following it
            final = []
            for m in mods:
                if m is None or id(m) in self._announced:
                    continue
                n = self._ready_count.get(id(m), 0) + 1
                self._ready_count[id(m)] = n
                self._seen_mods[id(m)] = m
                if n >= self.defer_wgrad and not any(e[0].mod is m for e in self._deferred.values()):
                    final.append(m)
            if final:
                self._announce_now(final)
            return
        if self._side_pending:          # some of these gradients may still be in flight on the side stream
            self._ready_pending.extend(mods)
            return
        self._notify(mods)

    def _announce_now(self, mods):
        """Announce final gradients produced on any of this engine's streams: the announcement (and the
        collective a listener launches from it) is issued on the merged-launch stream after it has caught up
        with the compute and side streams -- the compute stream itself never waits."""
        for m in mods:
            self._announced.add(id(m))
        if self.side2 is None:
            self.side2 = torch.cuda.Stream(device=self.device, priority=K.SIDE_PRIORITY)
        self.side2.wait_stream(torch.cuda.current_stream(self.device))
        if self.side is not None:
            self.side2.wait_stream(self.side)
        with torch.cuda.stream(self.side2):
            self._notify(mods)

    def open_defer_window(self):
        """Pipeline stage backward over several microbatches begins: defer until close_defer_window()."""
        self._defer_window = self.defer_wgrad > 1

    def close_defer_window(self):
        self._defer_window = False
        self.flush_wgrad()

    def _launch_deferred(self, key):
        c, gs, xs = self._deferred.pop(key)
        self._deferred_bytes -= sum(_nbytes(t) for t in gs + xs)
        self.n_multi_launches += 1
        self._launch_multi(c, gs, xs)

    def _launch_multi(self, c, gs, xs):
        """One weight-gradient launch over the deferred microbatches of conv ``c``, on a stream of its
        own: the per-block joins (side stream) must not wait for it, only flush_wgrad does."""
        gw, gb = _grad(c.mod.weight), _grad(c.mod.bias)
        if self.side2 is None:
            self.side2 = torch.cuda.Stream(device=self.device, priority=K.SIDE_PRIORITY)
        self.side2.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.side2):
            K.wgrad_multi(gs, xs, M=c.Cout, Nc=c.Cs, gw=gw.view(-1), gb=gb, Nreal=c.Cin)
            ev = torch.cuda.Event()
            ev.record(self.side2)
        self._keep2.append((ev, list(gs) + list(xs)))

    def _release_done(self):
        """Drop the operands of merged weight-gradient launches that have finished (an event query, no
        sync): their memory returns to the caching allocator during the backward instead of at
        flush_wgrad.  Safe without record_stream: the kernel reading them is complete."""
        while self._keep2 and self._keep2[0][0].query():
            self._keep2.pop(0)

    def flush_wgrad(self):
        """Run the deferred weight gradients still waiting for microbatches (one launch per layer over
        the ones that arrived), join the side stream, announce the gradients."""
        self._flush_queued = False
        for key in list(self._deferred):
            self._launch_deferred(key)
        self._deferred_bytes = 0
        if self._keep2:
            torch.cuda.current_stream(self.device).wait_stream(self.side2)
            self._keep2 = []
        self.join()
        mods, self._deferred_ready = self._deferred_ready, []
        if self.early_ready:
            # the modules not yet announced (a layer whose merged launch waited for the flush)
            mods = [m for k, m in self._seen_mods.items() if k not in self._announced]
            self._ready_count, self._seen_mods, self._announced = {}, {}, set()
        if mods:
            self._notify(mods)

    def _notify(self, mods):
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

    # ------------------------------------------------------------------ block API
    def prep(self, x: torch.Tensor) -> torch.Tensor:
        self._zx.clear()
        if x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] == 8:
            return x   # already converted (logical NCHW8, channels_last)
        return _o(K.input_nhwc8(x.float()))

    def enc(self, l: int, x):
        self.ensure_packed()
        return _EncFn.apply(self.anchor, x, self, l)

    def mid(self, x):
        self.ensure_packed()
        return _MidFn.apply(self.anchor, x, self)

    def dec(self, i: int, x, skip):
        self.ensure_packed()
        return _DecFn.apply(self.anchor, x, skip, self, i)

    # halves of a block cut between its two convs (a pipeline stage boundary inside a DoubleConv,
    # models/blocks.py): the tensor between them is the first conv's (BN+)ReLU output, materialised;
    # the fusions that span the two convs (BN-on-load, the first conv's BN statistics from the second
    # conv's dgrad epilogue) do not cross the cut
    def enc_a(self, l: int, x):
        self.ensure_packed()
        return _ConvHalfFn.apply(self.anchor, x, self, self.enc_convs[l][0], l > 0, None)

    def enc_b(self, l: int, a):
        self.ensure_packed()
        return _EncBFn.apply(self.anchor, a, self, l)

    def mid_a(self, x):
        self.ensure_packed()
        return _ConvHalfFn.apply(self.anchor, x, self, self.mid_convs[0], True, None)

    def mid_b(self, a):
        self.ensure_packed()
        return _ConvHalfFn.apply(self.anchor, a, self, self.mid_convs[1], True, self.mid_convs[0])

    def dec_a(self, i: int, x, skip):
        self.ensure_packed()
        return _DecAFn.apply(self.anchor, x, skip, self, i)

    def dec_b(self, i: int, a):
        self.ensure_packed()
        c1, c2 = self.dec_convs[i]
        return _ConvHalfFn.apply(self.anchor, a, self, c2, True, c1)

    def expect_target(self, t):
        """The segment being run ends in the head: the last decoder conv may compute the head and the
        loss partial sums in its epilogue (one pass less over the full-resolution activation)."""
        self._target = None if t is None else (t, t.float().reshape(-1).contiguous())

    def head_partials(self, x, t):
        if self._target is not None and self._target[0] is t:
            tf = self._target[1].view(t.shape)
        else:
            tf = t.float().contiguous()
        self._target = None
        return _HeadFn.apply(self.anchor, x, tf, self)

    @torch.no_grad()
    def head_probs(self, x):
        seg = self.model.segmap
        _, probs = K.head_fwd(_v(x), seg.weight, seg.bias, None, want_probs=True)
        return probs.unsqueeze(1)

    # concat buffers: the encoder allocates [N,H,W,2C] and returns its first half as the skip
    def new_cat(self, N, H, W, C):
        cat = torch.empty(N, H, W, 2 * C, dtype=torch.bfloat16, device=self.device)
        self._cats[cat.data_ptr()] = cat
        return cat

    def cat_for(self, skip: torch.Tensor) -> torch.Tensor:
        """NHWC concat buffer whose first half holds ``skip`` (an NHWC view): zero-copy when ``skip``
        came from this engine's encoder, one copy when it arrived from elsewhere (pipeline recv)."""
        N, H, W, C = skip.shape
        cat = self._cats.pop(skip.data_ptr(), None)
        if cat is not None and tuple(cat.shape) == (N, H, W, 2 * C) and skip.stride(2) == 2 * C:
            return cat
        cat = torch.empty(N, H, W, 2 * C, dtype=torch.bfloat16, device=self.device)
        cat[..., :C].copy_(skip)
        return cat


def bn_combo_ok(conv_bn: bool, below_bn, bn_fusable: bool) -> bool:
    """BatchNorm combinations the fused backward kernel (csrc/bwd_stream.hip) implements.  ``below_bn``
    is None when the dx is not ReLU-masked by a layer below (no ``below``), else whether that layer has a
    BatchNorm.  Without BN anywhere: always.  With BN: only when fusing it is allowed and, for a masked dx,
    the conv and the layer below agree -- the kernel's BN modes pair the loader's BN backward (this conv)
    with the dx epilogue's BN partial sums (the layer below); a BN on one side only has no instantiation
    (mixed models must take the unfused path, not fail an assert / InvalidValue)."""
    if not conv_bn and not below_bn:
        return True
    if not bn_fusable:
        return False
    return below_bn is None or below_bn == conv_bn


def _v(t: torch.Tensor) -> torch.Tensor:
    """logical-NCHW channels_last -> NHWC view (copies only if the layout is something else)."""
    if t.dim() == 4 and t.stride(1) != 1:
        t = t.contiguous(memory_format=torch.channels_last)
    return t.permute(0, 2, 3, 1)


def _o(t: torch.Tensor) -> torch.Tensor:
    """NHWC -> logical-NCHW view (channels_last strides)."""
    return t.permute(0, 3, 1, 2)


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


def _grad(p: torch.nn.Parameter) -> torch.Tensor:
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    g = p.grad
    assert g.dtype == torch.float32 and g.is_contiguous()
    return g


class _EncFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, x, B: HipBlocks, l: int):
        c1, c2 = B.enc_convs[l]
        x = _v(x)
        N, H, W = x.shape[:3]
        st1, st2 = [], []
        xbn1 = None
        if B.bn_on_load(c1, c2, H, W):
            a, xbn1 = B.conv_bn_z(c1, x, st1)         # a = conv1's pre-BN output; conv2 applies BN + ReLU
        else:
            a = B.conv_fwd(c1, x, st=st1)
        if l in B.dense_skips or B.dual_level(l, H, W):
            cat = None
            skip = torch.empty(N, H, W, c2.Cout, dtype=torch.bfloat16, device=x.device)
        else:
            cat = B.new_cat(N, H, W, c2.Cout)
            skip = cat[..., :c2.Cout]
        pooled = torch.empty(N, H // 2, W // 2, c2.Cout, dtype=torch.bfloat16, device=x.device)
        # window codes (argmax + ReLU masks) for the backward: it then never re-reads the skip
        code = (torch.empty(N, H // 2, W // 2, c2.Cout, dtype=torch.uint8, device=x.device)
                if H % 2 == 0 and W % 2 == 0 else None)
        if (cat is None and code is not None and c2.bn is not None and K.BN_SKIP_Z and l in B.skip_z_levels
                and B.model.training and K.BN_SUMS_POOL and K.BN_SUMS_POOL_Z and l not in B.dense_skips
                and B.dual_level(l, H, W) and B.bn_on_load(*B.dec_convs[len(B.dec_convs) - 1 - l], H, W)):
            # the skip's consumer (the decoder conv's dual input) forms relu(bn(z)) on load: the skip IS z and
            # the BN pass writes only the pooled quarter + codes (the full-resolution y is never stored)
            skip, coef2 = B.conv_bn_z_pool(c2, a, st2, pooled, code, xbn=xbn1)
            B._zx[skip.data_ptr()] = (skip, coef2)
        else:
            B.conv_fwd(c2, a, skip, pool=pooled, pcode=code, st=st2, xbn=xbn1)   # pool fused into the conv epilogue when streaming
        ctx.B, ctx.l = B, l
        ctx.xbn1 = xbn1
        ctx.x_needs_grad = l > 0
        ctx.has_code = code is not None
        ctx.st = (st1[0] if st1 else None, st2[0] if st2 else None)
        ctx.dense = cat is None
        # the concat buffer itself is saved (not its half): it keeps the engine's weak cat map entry alive
        own = skip if cat is None else cat
        ctx.save_for_backward(x, a, own, code if code is not None else own)
        return _o(skip), _o(pooled)

    @staticmethod
    def backward(ctx, dskip, dpooled):
        B, l = ctx.B, ctx.l
        x, a, own, code = ctx.saved_tensors
        st1, st2 = ctx.st
        c1, c2 = B.enc_convs[l]
        C = c2.Cout
        skip = own if ctx.dense else own[..., :C]
        if dpooled is None:
            dpooled = torch.zeros(x.shape[0], x.shape[1] // 2, x.shape[2] // 2, C, dtype=torch.bfloat16, device=x.device)
        else:
            dpooled = _v(dpooled)
        dskip = None if dskip is None else _v(dskip)
        W = a.shape[2]
        pool_fold = (ctx.has_code and K.USE_FUSED_POOL_BWD and B.fusable(c2, c1, W, whole=True)
                     and K.bwd_pool_foldable(c2.Cin, c2.Cout))
        if pool_fold and not ctx.x_needs_grad and K.USE_FUSED_W1 and c1.bn is None and c1.Cs == 8 \
                and c1.Cout == 32 and x.is_contiguous():
            # first level: conv2's fused backward also forms conv1's weight/bias gradient from its
            # (never stored) input gradient -- the level's whole backward in one pass
            B.conv_bwd(c2, dskip, a, mask=True, pool=(code, dpooled), first=(c1, x))
            B.ready([c2.mod, c2.bn])
            B.ready([c1.mod, c1.bn])
            B.join()
            ctx.st = None
            return None, None, None, None
        N = a.shape[0]
        chunks = K.ENC0_CHUNKS if (pool_fold and not ctx.x_needs_grad and c1.bn is None and dskip is not None
                                   and B.side is not None and B.defer_wgrad <= 1) else 1
        if chunks > 1 and N >= chunks:
            # the first level: conv1 needs only its weight gradient, which reads conv2's whole input gradient
            # -- launched after the last fused backward it would run alone at the end of the step (1.1 ms
            # at b256).  Image chunks: conv1's weight gradient of chunk i (side stream) overlaps the fused
            # backward of chunk i + 1, leaving only the last chunk's exposed
            bounds = [N * i // chunks for i in range(chunks + 1)]
            H = a.shape[1]
            sink2 = sink1 = None
            if K.CHUNK_SINK and K.wgrad_multi_eligible(c1.Cout, c1.Cs, W) and not K._ABLATE:
                # one weight-gradient reduction per conv after the chunks instead of one per chunk per stream
                # (each a presum + reduce; the side stream's waited ~0.45 ms for dispatch behind the next
                # chunk's fused backward)
                sizes = [n1 - n0 for n0, n1 in zip(bounds, bounds[1:])]
                sink2 = K.SlabSink(sum(K.bwd_fused_rows(n, H, W, c2.Cin, c2.Cout) for n in sizes), c2.Cout, c2.Cin,
                                   _grad(c2.mod.weight).view(-1), _grad(c2.mod.bias), c2.Cin)
                sink1 = K.SlabSink(sum(K.wgrad_stream_rows(n, H, W, c1.Cout, c1.Cs) for n in sizes), c1.Cout, c1.Cs,
                                   _grad(c1.mod.weight).view(-1), _grad(c1.mod.bias), c1.Cin)
            for n0, n1 in zip(bounds, bounds[1:]):
                g1c = B.conv_bwd(c2, dskip[n0:n1], a[n0:n1], mask=True, pool=(code[n0:n1], dpooled[n0:n1]), sink=sink2)
                B.conv_wgrad(c1, g1c, x[n0:n1], sink=sink1)
            if sink2 is not None:
                sink2.reduce()
                B.sink_reduce(sink1)
            B.ready([c2.mod, c2.bn])
            B.ready([c1.mod, c1.bn])
            B.join()
            ctx.st = None
            return None, None, None, None
        if pool_fold:
            # max-pool backward folded into the conv's fused backward: the gradient is formed from
            # (skip gradient, pooled gradient, window codes) on load and never stored
            g1, st_g = B.conv_bwd(c2, dskip, a, mask=True, pool=(code, dpooled)), None
        else:
            g2 = torch.empty(a.shape[:3] + (C,), dtype=torch.bfloat16, device=a.device)
            # a BatchNorm after conv2 (skip = its ReLU output): the pool backward also writes that BN's backward
            # partial sums (sum g, sum g*skip) -- no statistics pass over (g, z)
            g_stats = [] if (c2.bn is not None and ctx.has_code and K.BN_SUMS_POOL) else None
            if ctx.has_code:
                # the sums read y = relu(bn(z)) re-formed from the dense z (the skip is a strided concat half)
                zc = (st2[0], st2[2]) if (g_stats is not None and K.BN_SUMS_POOL_Z and st2[2] is not None) else (skip, None)
                K.pool_bwd_code(code, dskip, dpooled, g2, y=zc[0], bn_stats=g_stats, coef=zc[1])
            else:
                K.pool_bwd(skip, dskip, dpooled, g2)
            g_stats = g_stats or None
            if B.fusable(c2, c1, W):
                g1, st_g = B.bwd_conv(c2, g2, a, st2, mask=True, below=c1, xbn=ctx.xbn1, stats=g_stats)
            else:
                assert ctx.xbn1 is None, "BN-on-load forward needs the fused backward"
                g2 = B.bn_bwd(c2, g2, st2, stats=g_stats)
                B.conv_wgrad(c2, g2, a)              # side stream: overlaps the dgrad chain
                g1, st_g = B.conv_dgrad(c2, g2, mask=a, below=c1)
            g2 = None                    # dead: freed before conv1's backward allocates
        st2 = None                       # conv2's BN input z, likewise
        ctx.st = (st1, None)
        ctx.xbn1 = None
        B.ready([c2.mod, c2.bn])
        if ctx.x_needs_grad and B.fusable(c1, None, W):
            # the pool backward below applies the ReLU mask
            gx, _ = B.bwd_conv(c1, g1, x, st1, mask=False, stats=st_g)
        elif (not ctx.x_needs_grad and c1.bn is not None and K.BN_WGRAD_ON_LOAD and B.defer_wgrad <= 1
              and K.wgrad_bn_eligible(c1.Cout, c1.Cs, W) and g1.is_contiguous() and st1[0].is_contiguous()):
            # the first conv (no input gradient): its BN backward is formed in the weight gradient's loader from
            # per-channel coefficients -- the full-resolution dz pass (write + read) never happens
            z1, saved1 = st1[:2]
            coef3 = K.bn_bwd_coef(g1, z1, saved1, c1.bn, _grad(c1.bn.weight), _grad(c1.bn.bias), stats=st_g)
            B.conv_wgrad(c1, g1, x, gbn=(z1, coef3))
            gx = None
        else:
            g1 = B.bn_bwd(c1, g1, st1, stats=st_g)
            B.conv_wgrad(c1, g1, x)
            gx = B.conv_dgrad(c1, g1) if ctx.x_needs_grad else None
        B.ready([c1.mod, c1.bn])
        B.join()
        ctx.st = None
        return None, (None if gx is None else _o(gx)), None, None


class _MidFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, x, B: HipBlocks):
        c1, c2 = B.mid_convs
        x = _v(x)
        st1, st2 = [], []
        a = B.conv_fwd(c1, x, st=st1)
        y = B.conv_fwd(c2, a, st=st2)
        ctx.B = B
        ctx.st = (st1[0] if st1 else None, st2[0] if st2 else None)
        ctx.save_for_backward(x, a)
        return _o(y)

    @staticmethod
    def backward(ctx, g2):
        B = ctx.B
        x, a = ctx.saved_tensors
        st1, st2 = ctx.st
        c1, c2 = B.mid_convs
        g2 = _v(g2)
        g2 = B.bn_bwd(c2, g2, st2, stats=B.take_stats(g2))
        B.conv_wgrad(c2, g2, a)
        g1, st_g = B.conv_dgrad(c2, g2, mask=a, below=c1)
        B.ready([c2.mod, c2.bn])
        g1 = B.bn_bwd(c1, g1, st1, stats=st_g)
        B.conv_wgrad(c1, g1, x)
        gx = B.conv_dgrad(c1, g1)
        B.ready([c1.mod, c1.bn])
        B.join()
        ctx.st = None
        return None, _o(gx), None


class _DecFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, x, skip, B: HipBlocks, i: int):
        d = B.deconvs[i]
        c1, c2 = B.dec_convs[i]
        C = d.Cout
        x = _v(x)
        skip = _v(skip)
        # x may be the previous decoder block's BatchNorm input z (see below): the transposed conv reads
        # relu(bn(z)) on load, forward and backward
        zx = B._zx.pop(x.data_ptr(), None)
        dxbn = zx[1] if (zx is not None and zx[0].shape == x.shape and zx[0].stride() == x.stride()) else None
        skip_xbn = None
        local_next, B.next_dec_local = B.next_dec_local, False
        Ns, Hs, Ws, _ = skip.shape
        h2, w2 = 2 * x.shape[1], 2 * x.shape[2]
        ctx.crop = None
        if (Hs, Ws) != (h2, w2):
            # reference CenterCrop of the skip to the up-sampled size (model/unet_parts.py:58-74):
            # H, W not divisible by 2**depth -- the cropped skip is copied into a fresh concat buffer
            top, left = int(round((Hs - h2) / 2.0)), int(round((Ws - w2) / 2.0))
            cat = torch.empty(Ns, h2, w2, 2 * C, dtype=torch.bfloat16, device=x.device)
            cat[..., :C].copy_(skip[:, top:top + h2, left:left + w2])
            ctx.crop = (Hs, Ws, top, left)
            up = None
        elif (skip.is_contiguous() and B.dual_level(len(B.deconvs) - 1 - i, h2, w2)):
            # dual input: skip and up stay two dense tensors, the conv reads both (no concat buffer)
            cat = skip
            up = torch.empty(Ns, h2, w2, C, dtype=torch.bfloat16, device=x.device)
            sz = B._zx.pop(skip.data_ptr(), None)
            if sz is not None and sz[0].shape == skip.shape and sz[0].stride() == skip.stride():
                # the skip is the encoder BN's input z: conv1 reads relu(bn(z)) for its first 32 channels
                skip_xbn = sz[1]
        else:
            cat = B.cat_for(skip)
            up = None
        B.deconv_fwd(d, x, cat[..., C:] if up is None else up, xbn=dxbn)
        st1, st2 = [], []
        xbn1 = None
        if skip_xbn is not None:
            assert B.bn_on_load(c1, c2, h2, w2), "skip kept as z: the decoder conv must be a BN-statistics stream conv"
        if B.bn_on_load(c1, c2, h2, w2):
            # a = conv1's pre-BN output; conv2 applies BN + ReLU
            a, xbn1 = B.conv_bn_z(c1, cat, st1, x2=up, xbn=skip_xbn)
        else:
            a = B.conv_fwd(c1, cat, st=st1, x2=up)
        N, H, W = a.shape[:3]
        tgt = B._target[1] if (B._target is not None and i == len(B.deconvs) - 1) else None
        seg = B.model.segmap
        if (tgt is not None and c2.bn is None and seg.out_channels == 1 and tgt.numel() == N * H * W
                and K.head_fusable(N, H, W, c2.Cin, c2.Cout)):
            # last decoder conv + segmap + sigmoid + BCE/Dice partial sums in one kernel
            y = torch.empty(N, H, W, c2.Cout, dtype=torch.bfloat16, device=a.device)
            # the per-pixel probability is kept for the head backward folded into this conv's backward
            hprob = torch.empty(N * H * W, dtype=torch.float32, device=a.device)
            S = K.igemm(a, B.wf(c2), y, Ngemm=c2.Cout, Kpad=c2.Kf, KH=3, KW=3, stride=1, pad=1, Cs=c2.Cs,
                        out_grid=(N, H, W), bias=c2.mod.bias, relu=True,
                        head=(seg.weight.view(-1), seg.bias, tgt, hprob))
            B._head_cache = (y.data_ptr(), tgt.data_ptr(), S, hprob)
        elif (local_next and tgt is None and c2.bn is not None and K.BN_DECONV_ON_LOAD and B.model.training
              and i + 1 < len(B.deconvs) and isinstance(B.deconvs[i + 1], _Deconv) and K.USE_FUSED_DECONV
              and (B.deconvs[i + 1].Cin, B.deconvs[i + 1].Cout) in K.DECONV_BWD_SHAPES
              and B.deconvs[i + 1].Cin == c2.Cout):
            # BatchNorm model: the next decoder block's transposed conv reads relu(bn(z)) on load (forward and
            # backward), so this BN output is never written; the returned tensor is z, recognised there
            y, coef = B.conv_bn_z(c2, a, st2, xbn=xbn1)
            B._zx[y.data_ptr()] = (y, coef)
        elif (tgt is not None and c2.bn is not None and K.BN_HEAD_ON_LOAD and B.model.training and seg.out_channels == 1
              and tgt.numel() == N * H * W and c2.Cout in (32, 64)):
            # BatchNorm model: the head reads relu(bn(z)) on load (forward and backward), so the last decoder
            # conv's BN output is never written: the returned tensor is z, which _HeadFn recognises
            y, coef = B.conv_bn_z(c2, a, st2, xbn=xbn1)
            # the per-pixel probability is kept for the head backward folded into conv2's (K.BN_HEAD_FOLD)
            S, probs = K.head_fwd(y, seg.weight, seg.bias, tgt, coef=coef, want_probs=K.BN_HEAD_FOLD)
            B._head_cache = (y.data_ptr(), tgt.data_ptr(), S, None if probs is None else probs.view(-1), coef)
        else:
            y = B.conv_fwd(c2, a, st=st2, xbn=xbn1)
        ctx.xbn1 = xbn1
        ctx.dxbn = dxbn
        ctx.skip_xbn = skip_xbn
        ctx.B, ctx.i = B, i
        ctx.st = (st1[0] if st1 else None, st2[0] if st2 else None)
        ctx.dual = up is not None
        ctx.save_for_backward(x, cat, a, up if up is not None else cat)
        return _o(y)

    @staticmethod
    def backward(ctx, g2):
        B, i = ctx.B, ctx.i
        x, cat, a, up = ctx.saved_tensors
        st1, st2 = ctx.st
        d = B.deconvs[i]
        c1, c2 = B.dec_convs[i]
        C = d.Cout
        pend = B._head_pending
        formed = folded = False
        if (pend is not None and len(pend) > 5 and g2.data_ptr() == pend[0].data_ptr()
                and g2.stride() == pend[0].stride()):
            # BatchNorm model, head on load: its gradient (and that BN's backward partial sums) is formed here
            # from (z, coef) rather than in _HeadFn.backward, so the full-resolution gy is a local that dies
            # after this conv's backward instead of an autograd buffer held to the end of this function
            B._head_pending = None
            _, z2, t, dS, hprob, coef = pend
            pend = None
            seg = B.model.segmap
            hs = []
            W = z2.shape[2]
            if (hprob is not None and K.BN_HEAD_FOLD and c1.bn is not None and c2.Cin == c2.Cout == 32
                    and B.fusable(c2, c1, W) and W % 64 == 0
                    and z2.is_contiguous() and st2[0].data_ptr() == z2.data_ptr() and st2[0].stride() == z2.stride()):
                # head + BN folded into conv2's fused backward: a statistics pass (the segmap gradients and the
                # BN's partial sums), then the kernel forms gy from z and the stored probability and dz from gy
                # on load -- the head gradient is never stored
                K.head_bwd(z2, seg.weight, seg.bias, t, dS, _grad(seg.weight).view(-1), _grad(seg.bias), bn_stats=hs,
                           coef=coef, store=False)
                B.ready([seg])
                g1, st_g = B.bwd_conv_head_bn(c2, z2, a, st2, t, dS, hprob, coef, xbn=ctx.xbn1, stats=hs)
                folded = True
            else:
                g2 = K.head_bwd(z2, seg.weight, seg.bias, t, dS, _grad(seg.weight).view(-1), _grad(seg.bias),
                                bn_stats=hs, coef=coef)
                B.ready([seg])
                head_stats, formed = hs or None, True
            del z2
        if folded:
            pass
        elif (pend is not None and len(pend) == 5 and g2.data_ptr() == pend[0].data_ptr()
                and g2.stride() == pend[0].stride()):
            # the head's gradient was deferred (_HeadFn.backward): it is formed from y inside this
            # conv's fused backward instead of being materialised (saves a write + read of it)
            B._head_pending = None
            _, y, t, dS, hprob = pend
            seg = B.model.segmap
            W = y.shape[2]
            g1, st_g = B.conv_bwd(c2, y, a, mask=True, head=(t, seg.weight, seg.bias, dS,
                                                             _grad(seg.weight).view(-1), _grad(seg.bias), hprob)), None
            B.ready([seg])
        else:
            if not formed:
                g2 = _v(g2)
                head_stats = B.take_stats(g2)    # from the head's or the next level's transposed-conv backward
            if pend is not None:
                # the head's deferred gradient reached us in another form (summed with another
                # gradient, or materialised by a hook): form it now and add it, never drop it
                B._head_pending = None
                ph, y, t, dS = pend[:4]
                coef = pend[5] if len(pend) > 5 else None      # BN head on load: y is the BN input z
                seg = B.model.segmap
                gy = K.head_bwd(y, seg.weight, seg.bias, t, dS, _grad(seg.weight).view(-1), _grad(seg.bias),
                                bn_stats=[] if coef is not None else None, coef=coef)
                B.ready([seg])
                g2 = (gy.float() + g2.float()).to(torch.bfloat16).contiguous()
                head_stats = None            # partial sums of the summed gradient: the BN backward forms them
            W = g2.shape[2]
            if B.fusable(c2, c1, W):
                g1, st_g = B.bwd_conv(c2, g2, a, st2, mask=True, below=c1, xbn=ctx.xbn1, stats=head_stats)
            else:
                assert ctx.xbn1 is None, "BN-on-load forward needs the fused backward"
                g2 = B.bn_bwd(c2, g2, st2, stats=head_stats)
                B.conv_wgrad(c2, g2, a)
                g1, st_g = B.conv_dgrad(c2, g2, mask=a, below=c1)
        B.ready([c2.mod, c2.bn])
        # dead from here: the gradient and conv2's saved BN input z (the step's peak is reached just below, in
        # conv1's backward at full resolution; autograd would hold them to the end of this function)
        g2 = st2 = None
        ctx.st = (st1, None)
        if ctx.dual:
            # the forward checked fusable() (dual_level): the fused backward reads [skip | up] too
            (dskip, gup), _ = B.bwd_conv(c1, g1, cat, st1, mask=False, stats=st_g, split=C, x2=up, xbn=ctx.skip_xbn)
            ctx.skip_xbn = None
        elif B.fusable(c1, None, W):
            (dskip, gup), _ = B.bwd_conv(c1, g1, cat, st1, mask=False, stats=st_g, split=C)
        elif c1.bn is not None and B.halves_fusable(c1, C, W) and g1.stride() == st1[0].stride():
            # BatchNorm conv over a 2C-channel concat: one fused pass per half, each forming the BN backward
            # on load (the dz pass, the split dgrad GEMM and the side-stream weight gradient all go)
            z1, saved1 = st1[:2]
            coef3 = K.bn_bwd_coef(g1, z1, saved1, c1.bn, _grad(c1.bn.weight), _grad(c1.bn.bias), stats=st_g)
            dskip, gup = B.conv_bwd_halves(c1, g1, cat, C, bn=(z1, coef3))
        else:
            g1 = B.bn_bwd(c1, g1, st1, stats=st_g)
            if B.halves_fusable(c1, C, W):
                dskip, gup = B.conv_bwd_halves(c1, g1, cat, C)
            else:
                B.conv_wgrad(c1, g1, cat)
                dskip, gup = B.conv_dgrad_split(c1, g1, C)
        B.ready([c1.mod, c1.bn])
        g1 = None
        if isinstance(d, _Up):
            gup = K.up2_bwd(gup)          # to the projection's (low) resolution
        dx = B.deconv_bwd(d, gup, x, xbn=ctx.dxbn)
        ctx.dxbn = None
        B.ready([d.mod])
        B.join()
        ctx.st = None
        if ctx.crop is not None:     # gradient of the crop: zero outside the kept window
            Hs, Ws, top, left = ctx.crop
            full = torch.zeros(dskip.shape[0], Hs, Ws, C, dtype=dskip.dtype, device=dskip.device)
            full[:, top:top + dskip.shape[1], left:left + dskip.shape[2]] = dskip
            dskip = full
        return None, _o(dx), _o(dskip), None, None


class _ConvHalfFn(torch.autograd.Function):
    """One conv (+BN) + ReLU of a split DoubleConv.  ``below``: the conv whose output ``x`` is (the
    first conv, for a second half) -- x is then a ReLU output and the dgrad is masked by it; without
    ``below`` (a first half) the dgrad is not masked (the pool backward / concat split upstream masks
    it), and ``x_grad`` False skips it (the network input)."""

    @staticmethod
    def forward(ctx, anchor, x, B: "HipBlocks", c: _Conv, x_grad: bool, below):
        x = _v(x)
        st = []
        y = B.conv_fwd(c, x, st=st)
        ctx.B, ctx.c, ctx.below, ctx.x_grad = B, c, below, x_grad
        ctx.st = st[0] if st else None
        ctx.save_for_backward(x)
        return _o(y)

    @staticmethod
    def backward(ctx, g):
        B, c, below = ctx.B, ctx.c, ctx.below
        (x,) = ctx.saved_tensors
        g = _v(g)
        W = g.shape[2]
        mask = below is not None
        if ctx.x_grad and B.fusable(c, below, W):
            gx, _ = B.bwd_conv(c, g, x, ctx.st, mask=mask, below=below)
        else:
            g = B.bn_bwd(c, g, ctx.st)
            B.conv_wgrad(c, g, x)
            gx = None
            if ctx.x_grad:
                gx = B.conv_dgrad(c, g, mask=x if mask else None, below=below)
                if below is not None:
                    gx = gx[0]
        B.ready([c.mod, c.bn])
        B.join()
        ctx.st = None
        return None, (None if gx is None else _o(gx)), None, None, None, None


class _EncBFn(torch.autograd.Function):
    """Second half of an encoder block: conv2 (+BN) + ReLU + max-pool (fused when streaming)."""

    @staticmethod
    def forward(ctx, anchor, a, B: "HipBlocks", l: int):
        c1, c2 = B.enc_convs[l]
        a = _v(a)
        N, H, W = a.shape[:3]
        skip = torch.empty(N, H, W, c2.Cout, dtype=torch.bfloat16, device=a.device)   # dense: it may leave the stage
        pooled = torch.empty(N, H // 2, W // 2, c2.Cout, dtype=torch.bfloat16, device=a.device)
        code = (torch.empty(N, H // 2, W // 2, c2.Cout, dtype=torch.uint8, device=a.device)
                if H % 2 == 0 and W % 2 == 0 else None)
        st2 = []
        B.conv_fwd(c2, a, skip, pool=pooled, pcode=code, st=st2)
        ctx.B, ctx.l = B, l
        ctx.st = st2[0] if st2 else None
        ctx.has_code = code is not None
        ctx.save_for_backward(a, skip, code if code is not None else skip)
        return _o(skip), _o(pooled)

    @staticmethod
    def backward(ctx, dskip, dpooled):
        B, l = ctx.B, ctx.l
        a, skip, code = ctx.saved_tensors
        c1, c2 = B.enc_convs[l]
        C = c2.Cout
        dpooled = (torch.zeros(a.shape[0], a.shape[1] // 2, a.shape[2] // 2, C, dtype=torch.bfloat16, device=a.device)
                   if dpooled is None else _v(dpooled))
        dskip = None if dskip is None else _v(dskip)
        W = a.shape[2]
        if (ctx.has_code and K.USE_FUSED_POOL_BWD and B.fusable(c2, c1, W, whole=True)
                and K.bwd_pool_foldable(c2.Cin, c2.Cout)):
            g1 = B.conv_bwd(c2, dskip, a, mask=True, pool=(code, dpooled))
        else:
            g2 = torch.empty(a.shape[:3] + (C,), dtype=torch.bfloat16, device=a.device)
            if ctx.has_code:
                K.pool_bwd_code(code, dskip, dpooled, g2)
            else:
                K.pool_bwd(skip, dskip, dpooled, g2)
            if B.fusable(c2, c1, W):
                g1, _ = B.bwd_conv(c2, g2, a, ctx.st, mask=True, below=c1)
            else:
                g2 = B.bn_bwd(c2, g2, ctx.st)
                B.conv_wgrad(c2, g2, a)
                g1, _ = B.conv_dgrad(c2, g2, mask=a, below=c1)
        B.ready([c2.mod, c2.bn])
        B.join()
        ctx.st = None
        return None, _o(g1), None, None


class _DecAFn(torch.autograd.Function):
    """First half of a decoder block: transposed conv, crop, concat (or the dual input), conv1 (+BN) + ReLU."""

    @staticmethod
    def forward(ctx, anchor, x, skip, B: "HipBlocks", i: int):
        d = B.deconvs[i]
        c1, c2 = B.dec_convs[i]
        C = d.Cout
        x = _v(x)
        skip = _v(skip)
        Ns, Hs, Ws, _ = skip.shape
        h2, w2 = 2 * x.shape[1], 2 * x.shape[2]
        ctx.crop = None
        up = None
        if (Hs, Ws) != (h2, w2):
            top, left = int(round((Hs - h2) / 2.0)), int(round((Ws - w2) / 2.0))
            cat = torch.empty(Ns, h2, w2, 2 * C, dtype=torch.bfloat16, device=x.device)
            cat[..., :C].copy_(skip[:, top:top + h2, left:left + w2])
            ctx.crop = (Hs, Ws, top, left)
        elif skip.is_contiguous() and B.dual_level(len(B.deconvs) - 1 - i, h2, w2):
            cat = skip
            up = torch.empty(Ns, h2, w2, C, dtype=torch.bfloat16, device=x.device)
        else:
            cat = B.cat_for(skip)
        B.deconv_fwd(d, x, cat[..., C:] if up is None else up)
        st1 = []
        a = B.conv_fwd(c1, cat, st=st1, x2=up)
        ctx.B, ctx.i = B, i
        ctx.st = st1[0] if st1 else None
        ctx.dual = up is not None
        ctx.save_for_backward(x, cat, up if up is not None else cat)
        return _o(a)

    @staticmethod
    def backward(ctx, g1):
        B, i = ctx.B, ctx.i
        x, cat, up = ctx.saved_tensors
        d = B.deconvs[i]
        c1, c2 = B.dec_convs[i]
        C = d.Cout
        g1 = _v(g1)
        W = g1.shape[2]
        if ctx.dual:
            (dskip, gup), _ = B.bwd_conv(c1, g1, cat, ctx.st, mask=False, split=C, x2=up)
        elif B.fusable(c1, None, W):
            (dskip, gup), _ = B.bwd_conv(c1, g1, cat, ctx.st, mask=False, split=C)
        else:
            g1 = B.bn_bwd(c1, g1, ctx.st)
            if B.halves_fusable(c1, C, W):
                dskip, gup = B.conv_bwd_halves(c1, g1, cat, C)
            else:
                B.conv_wgrad(c1, g1, cat)
                dskip, gup = B.conv_dgrad_split(c1, g1, C)
        B.ready([c1.mod, c1.bn])
        if isinstance(d, _Up):
            gup = K.up2_bwd(gup)
        dx = B.deconv_bwd(d, gup, x)
        B.ready([d.mod])
        B.join()
        ctx.st = None
        if ctx.crop is not None:
            Hs, Ws, top, left = ctx.crop
            full = torch.zeros(dskip.shape[0], Hs, Ws, C, dtype=dskip.dtype, device=dskip.device)
            full[:, top:top + dskip.shape[1], left:left + dskip.shape[2]] = dskip
            dskip = full
        return None, _o(dx), _o(dskip), None, None


class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, y, t, B: HipBlocks):
        seg = B.model.segmap
        y = _v(y)
        B._stats_hand.clear()                # a previous step's unconsumed hand-overs go now
        cache, B._head_cache = B._head_cache, None
        hit = cache is not None and cache[0] == y.data_ptr() and cache[1] == t.data_ptr()
        if hit:
            S = cache[2]                     # computed by the last decoder conv's epilogue
        else:
            S, _ = K.head_fwd(y, seg.weight, seg.bias, t)
        ctx.B = B
        # BN model with the head formed on load: y is the last BN's input z, relu(bn(z)) = relu(z*coef[:C]+coef[C:])
        ctx.coef = cache[4] if hit and len(cache) > 4 else None
        # fused forward => y is this engine's last decoder conv output and its backward runs next
        ctx.fold = hit and ctx.coef is None and B.head_bwd_foldable(y.shape[2])
        # the forward's probabilities, for the folded backward (plain, or BN head on load)
        ctx.hprob = cache[3] if (ctx.fold or ctx.coef is not None) else None
        ctx.save_for_backward(y, t)
        return S.clone()

    @staticmethod
    def backward(ctx, dS):
        B = ctx.B
        y, t = ctx.saved_tensors
        seg = B.model.segmap
        if ctx.fold and t.is_contiguous():
            # defer: hand the decoder a zero-stride placeholder of y's gradient; _DecFn.backward
            # recognises it and folds the head backward into the last conv's fused backward
            ph = torch.zeros((), dtype=y.dtype, device=y.device).expand(y.shape[0], y.shape[3], y.shape[1], y.shape[2])
            B._head_pending = (ph, y, t.reshape(-1), dS, ctx.hprob)
            ctx.hprob = None
            return None, ph, None, None
        # a BatchNorm after the last decoder conv: the head backward also writes that BN's backward partial
        # sums (sum gy, sum gy*y), handed to the decoder's backward with gy (no statistics pass over gy, z)
        coef, ctx.coef = ctx.coef, None
        if coef is not None and t.is_contiguous() and K.BN_HEAD_DEFER:
            # BN head on load: defer to the decoder's backward (see _DecFn.backward), like the fold above
            ph = torch.zeros((), dtype=y.dtype, device=y.device).expand(y.shape[0], y.shape[3], y.shape[1], y.shape[2])
            B._head_pending = (ph, y, t.reshape(-1), dS, ctx.hprob, coef)
            ctx.hprob = None
            return None, ph, None, None
        stats = [] if B.dec_convs[-1][1].bn is not None else None
        gy = K.head_bwd(y, seg.weight, seg.bias, t, dS, _grad(seg.weight).view(-1), _grad(seg.bias), bn_stats=stats,
                        coef=coef)
        B.ready([seg])
        B.hand_stats(gy, stats)
        return None, _o(gy), None, None
