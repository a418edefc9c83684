"""ctypes bindings of the gfx950 kernels in ``csrc/*.hip`` (``_C/libdpa_hip.so``).

Every wrapper takes torch tensors (NHWC bf16 activations, fp32 parameters/gradients), checks the
shape/stride/alignment assumptions its kernel makes on the host *before* launching (a bad launch
can fault the GPU), and launches on the current HIP stream of the tensor's device.  There is no
fallback: on a GPU the library must be present (``_lib.lib()`` raises otherwise).

Kernel map:  conv3x3 fwd / dgrad, convT fwd / dgrad -> ``igemm``;  conv / convT
weight gradients -> ``wgrad`` + ``wgrad_reduce``;  max-pool (K5) -> ``maxpool2`` / ``pool_bwd``;
segmap + sigmoid + BCE + Dice (K8-K11) -> ``head_fwd`` / ``head_bwd``;  Adam (K13) -> ``adam_step``.
Variant blocks (north-star DoubleConv with BatchNorm, bilinear Up): ``bn_fwd`` / ``bn_bwd``,
``up2_fwd`` / ``up2_bwd`` (csrc/norm_up.hip) and the 1x1 projection through ``igemm`` / ``wgrad(kind=2)``.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib
from . import config as _config

c_int, c_ll, c_void_p = ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p


class IgemmArgs(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("w", c_void_p), ("bias", c_void_p), ("y", c_void_p), ("mask", c_void_p)] + \
               [(n, c_int) for n in ("ldx", "ldy", "ldm", "mask_ch", "N", "Ho", "Wo", "Hs", "Ws", "Cs", "KH", "KW",
                                     "stride", "pad", "Ngemm", "Kpad", "mode", "relu", "accumulate", "Cout")] + \
               [("xbytes", ctypes.c_uint), ("pool", c_void_p), ("ldp", c_int), ("pcode", c_void_p), ("y2", c_void_p),
                ("ldy2", c_int), ("split", c_int), ("hw", c_void_p), ("hb", c_void_p), ("tgt", c_void_p),
                ("hslab", c_void_p), ("bnslab", c_void_p), ("korder", c_int), ("ximg", ctypes.c_uint),
                ("hprob", c_void_p), ("x2", c_void_p), ("xbn", c_void_p)]


class WgradArgs(ctypes.Structure):
    _fields_ = [("A", c_void_p), ("B", c_void_p), ("slab", c_void_p), ("bslab", c_void_p)] + \
               [(n, c_int) for n in ("lda", "ldb", "N", "Hg", "Wg", "HA", "WA", "HB", "WB", "M", "Nc", "s", "pad",
                                     "KW", "pix_per_split", "splits")] + \
               [("abytes", ctypes.c_uint), ("bbytes", ctypes.c_uint), ("atab", c_void_p), ("btab", c_void_p),
                ("az", c_void_p), ("abn", c_void_p)]


class BwdArgs(ctypes.Structure):
    _fields_ = [("g", c_void_p), ("x", c_void_p), ("wd", c_void_p), ("y", c_void_p), ("y2", c_void_p),
                ("slab", c_void_p), ("bslab", c_void_p)] + \
               [(n, c_int) for n in ("ldg", "ldx", "ldy", "ldy2", "split", "Kd", "N", "H", "W", "rh", "ipb")] + \
               [("gbytes", ctypes.c_uint), ("xbytes", ctypes.c_uint)] + \
               [("tgt", c_void_p), ("hw", c_void_p), ("hb", c_void_p), ("dS", c_void_p), ("hslab", c_void_p)] + \
               [("pcode", c_void_p), ("dpool", c_void_p), ("ldp", c_int)] + \
               [("x1", c_void_p), ("slab1", c_void_p), ("bslab1", c_void_p), ("x1bytes", ctypes.c_uint)] + \
               [("z", c_void_p), ("bncoef", c_void_p), ("bnslab", c_void_p), ("hprob", c_void_p), ("x2", c_void_p),
                                                                                      ("xbn", c_void_p), ("ybn", c_void_p)]


class PackDesc(ctypes.Structure):
    _fields_ = [("src", c_ll), ("dst", c_ll), ("mode", c_int), ("Cout", c_int), ("Cin", c_int), ("Cs", c_int),
                ("Ngemm", c_int), ("Kpad", c_int)]


def _p(t: Optional[torch.Tensor]):
    return None if t is None else c_void_p(t.data_ptr())


def _stream(t: torch.Tensor):
    return c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _check(err, name):
    _lib.check(int(err), name)


def _nhwc(t: torch.Tensor, name: str):
    """(N, H, W, C, ld) of an NHWC bf16 tensor whose channel slice may be strided (concat halves)."""
    assert t.dtype == torch.bfloat16 and t.dim() == 4 and t.is_cuda, f"{name}: need cuda bf16 NHWC, got {t.dtype} {tuple(t.shape)}"
    N, H, W, C = t.shape
    sN, sH, sW, sC = t.stride()
    ld = sW
    assert sC == 1 and sH == W * ld and (N == 1 or sN == H * W * ld), f"{name}: unsupported strides {t.stride()}"
    assert ld % 8 == 0 and t.data_ptr() % 16 == 0, f"{name}: ld {ld} / pointer not 16-byte aligned"
    return N, H, W, C, ld


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


_MAX_BYTES = 2 ** 31 - 1024   # kernels address activations through 32-bit buffer offsets
# dispatch switches: ONE table, read once from the documented DPA_* variables (ops/config.py)
CFG = _config.KernelConfig.from_env()
USE_HALO = CFG.halo                    # row-halo kernels (csrc/halo.hip)
USE_STREAM = CFG.stream                # row-streaming conv3x3 (weights resident, row ring)
USE_GLDS = CFG.glds                    # LDS-DMA GEMMs (csrc/igemm_glds.hip)
# 128-output-channel layers on rows of <= 128 pixels: the slice-staged 128 x 512 GEMM (cfg 18), 3-16 %
# faster than the 128-channel row-block kernel (profiles/kbench_sl_b256_r04.txt)
USE_GLDS_SL = CFG.glds_sl
# 64-output-channel convs over >= 64 input channels (the 256^2 decoder conv 128 -> 64, the 128^2 dgrads into 64
# channels): the slice-staged ping-pong 64 x 512 GEMM (cfg 19) instead of the row-halo conv
USE_SLP64 = CFG.slp64
BN_SUMS_POOL = CFG.bn_sums_pool        # BN backward partial sums from the pool backward (models/hip_unet.py)
BN_SUMS_DECONV = CFG.bn_sums_deconv    # ... from the fused transposed-conv backward
BN_SUMS_POOL_Z = CFG.bn_sums_pool_z    # ... reading the dense z (relu(bn(z)) re-formed) instead of the skip
BN_HEAD_ON_LOAD = CFG.bn_head_on_load  # the head reads the last decoder BN's input z (relu(bn(z)) on load)
BN_WGRAD_ON_LOAD = CFG.bn_wgrad_on_load  # the first conv's BN backward in its weight gradient's loader
BN_DECONV_ON_LOAD = CFG.bn_deconv_on_load  # a decoder block's output BN applied by the next transposed conv
BN_DUAL = CFG.bn_dual                  # BN model: dual-input (no concat buffer) full-resolution decoder level
BN_HALVES = CFG.bn_halves              # BN model: two-pass fused backward of the concat-input decoder conv
BN_SKIP_Z = CFG.bn_skip_z              # BN model: the dual-level skip kept as its BN input z
BN_HEAD_FOLD = CFG.bn_head_fold        # BN model: head backward folded into the last conv's fused backward
BN_HEAD_DEFER = CFG.bn_head_defer      # ... with its backward deferred into the decoder's (memory)
# 128-channel convs on the row-block ping-pong GEMM (cfg 15) instead of the row-halo conv: 10-15 % faster
# on every 128-output-channel 3x3 conv / dgrad of the 512^2 UNet (profiles/kbench_glds_rowblock128_b256_r03.txt)
USE_GLDS128 = CFG.glds128
USE_GLDS_BN = CFG.glds_bn              # BatchNorm partial sums in the row-block GEMM epilogue
SIDE_WGRAD = CFG.side_wgrad            # weight gradients on a side stream (models/hip_unet.py)
SIDE_PRIORITY = CFG.side_priority      # its HIP priority (torch convention: lower = higher, 0 = default)
ENC0_CHUNKS = CFG.enc0_chunks          # first-level backward in image chunks (models/hip_unet.py _EncFn)
CHUNK_SINK = CFG.chunk_sink            # ... with one weight-gradient reduction per conv after the chunks (SlabSink)
WGRAD_STREAM_CFG = 0                   # row-streaming weight-gradient tile override (kbench A/B; 0 = auto)
HALO_CFG = CFG.halo_cfg                # row-halo conv tile override (A/B; 0 = auto)
USE_FUSED_HEAD = CFG.fused_head        # segmentation head + loss partials in the last decoder conv
USE_FUSED_BN = CFG.fused_bn            # BatchNorm statistics in the producing streaming conv
FOLD_BN_EVAL = CFG.fold_bn_eval        # eval-mode BatchNorm folded into the conv weights
# fused conv backward (dgrad + weight/bias gradient in one row-streaming pass, csrc/bwd_stream.hip) for
# the full-resolution 32/64-channel convs, and its modes: the head backward folded in, concat convs as
# one fused pass per half, the max-pool backward folded in, BatchNorm backward formed in the loader
USE_FUSED_BWD = CFG.fused_bwd
USE_FUSED_HEAD_BWD = CFG.fused_head_bwd
USE_FUSED_HALVES = CFG.fused_halves
USE_FUSED_POOL_BWD = CFG.fused_pool_bwd
USE_FUSED_BN_BWD = CFG.fused_bn_bwd
# the first encoder conv's weight gradient folded into the pool-mode backward of the second: opt-in,
# slower at batch 256 (6.05 ms vs 5.3 ms for the two kernels it replaces; see csrc/bwd_stream.hip)
USE_FUSED_W1 = CFG.fused_w1
# the 32-channel level without a concat buffer: dense skip + dense up half, read by the decoder conv's
# row-streaming forward and fused backward through their dual input (x2)
USE_DUAL_INPUT = CFG.dual_input
# DoubleConv with BatchNorm at the 32/64-channel levels: conv2 reads conv1's pre-BN output z and forms
# relu(bn(z)) in its loader (forward and fused backward) -- no normalise pass, no stored BN output
USE_BN_ON_LOAD = CFG.bn_on_load

# TIMING ABLATION ONLY (numerically wrong results): the listed kernel families are skipped so a bench
# run measures what they cost end to end.  Never read from the environment: set_timing_ablation() is
# called explicitly by bench.py --timing-ablation and tools/block_times.py.  Categories: stream, halo,
# glds, wgrad, wgrad_deep, bwd, deconv
_ABLATE = frozenset()
ABLATE_CATEGORIES = frozenset({"stream", "halo", "glds", "wgrad", "wgrad_deep", "bwd", "deconv"})


def set_timing_ablation(categories) -> None:
    global _ABLATE
    cats = frozenset(categories or ())
    unknown = cats - ABLATE_CATEGORIES
    assert not unknown, f"unknown ablation categories {sorted(unknown)}"
    _ABLATE = cats


def _extent_bytes(N, H, W, C, ld):
    return ((N * H * W - 1) * ld + C) * 2


def _image_chunks(N: int, per_image_bytes: int):
    """Split a batch so every launch addresses < 2 GiB per tensor (buffer-descriptor range), in equal
    chunks: 255 + 1 images would leave a one-image launch that cannot fill the chip (~35 us for ~5 us
    of work, several per step at b256)."""
    per = max(1, _MAX_BYTES // max(per_image_bytes, 1))
    n = -(-N // per)
    per = -(-N // n)
    return [(i, min(N, i + per)) for i in range(0, N, per)]


# ------------------------------------------------------------------------------------------ igemm
def igemm(x: torch.Tensor, wpacked: torch.Tensor, y: torch.Tensor, *, Ngemm: int, Kpad: int, KH: int, KW: int,
          stride: int, pad: int, Cs: int, out_grid, bias: Optional[torch.Tensor] = None, relu: bool = False,
          mask: Optional[torch.Tensor] = None, mode: int = 0, Cout: int = 0, accumulate: bool = False, cfg: int = 0,
          path: str = "auto", pool: Optional[torch.Tensor] = None, variant: int = 0,
          pcode: Optional[torch.Tensor] = None, y2: Optional[torch.Tensor] = None, split: int = 0, head=None,
          bn_stats: Optional[list] = None, persistent: bool = True, x2: Optional[torch.Tensor] = None,
          xbn: Optional[torch.Tensor] = None):
    """Implicit-GEMM conv.  ``out_grid`` = (N, Ho, Wo) pixel grid of GEMM-M.

    ``path``: ``auto`` picks, for a conv3x3, the row-streaming kernel (Ngemm, Cs in {32, 64}), then the
    row-halo kernel (Cs % 32 == 0, Ngemm <= 128), then the generic gather kernel (csrc/igemm.hip);
    ``stream`` / ``halo`` / ``glds`` / ``generic`` force one (tests, A/B).  ``glds`` (csrc/igemm_glds.hip,
    LDS-DMA staged, 8 waves, Cs % 64 == 0) serves the deep layers before the generic kernel.  ``pool``: also produce the 2x2/s2
    max-pool of ``y`` (fused into the streaming kernel's epilogue, else a separate pass); ``pcode``: with
    ``pool``, the per-window codes (argmax + ReLU masks, uint8 [N, Ho/2, Wo/2, Ngemm]) that
    :func:`pool_bwd_code` consumes.  ``y2``/``split``: output channels >= ``split`` go to the dense
    tensor ``y2`` (channel ``co - split``) -- the two halves of a concat gradient.  ``head`` =
    (segmap weight, segmap bias, target [N*Ho*Wo] fp32): the streaming kernel also computes the fused
    segmap + sigmoid + BCE/Dice partial sums of its (bf16) output; returns them as S[4].
    ``bn_stats`` (an empty list): when the streaming kernel runs, its epilogue also writes per-block
    channel partial sums and the list receives (slab [rows][2][Ngemm] fp32, rows); left empty
    otherwise.  Without ``mask`` (conv followed by BatchNorm): sum y, sum y^2 for :func:`bn_fwd`;
    with ``mask`` = the BN layer's output (dgrad into it): sum g, sum g*mask for :func:`bn_bwd`.
    ``persistent=False``: the LDS-DMA path never picks its persistent (one workgroup per CU) kernel --
    the backward passes it while side-stream weight gradients hold CUs, which a persistent grid
    sized for the whole chip would otherwise wait for.  ``x2``: dual input -- the conv input is the
    channel concat [x | x2] of two tensors of identical layout (32 channels each, ``Cs`` = 64), read
    by the row-streaming kernel from both (a decoder conv over [skip | up] without a concat buffer).
    ``xbn`` (fp32 [2 Cs], :func:`bn_fwd` ``coef_out``): ``x`` is the pre-BatchNorm output z of the layer
    below and the conv's input is relu(z * xbn[c] + xbn[Cs + c]), formed in the row-streaming loader
    (BN-statistics epilogue launches only: a conv followed by BN, ``bn_stats`` given)."""
    N, Hs, Ws, Cx, ldx = _nhwc(x, "igemm.x")
    if x2 is not None:
        assert _nhwc(x2, "igemm.x2") == (N, Hs, Ws, Cx, ldx) and Cx == 32 and Cs == 64, "dual input: two [N,H,W,32]"
        assert mode == 0 and pool is None and head is None and path in ("auto", "stream"), "dual input: plain stream conv"
        Cx = Cs
    _, _, _, Cy, ldy = _nhwc(y, "igemm.y")
    No, Ho, Wo = out_grid
    assert No == N and Cs <= Cx and Cs % 8 == 0 and Kpad % 32 == 0 and Ngemm % 32 == 0
    assert wpacked.dtype == torch.bfloat16 and wpacked.numel() >= Ngemm * Kpad
    assert Kpad >= KH * KW * Cs
    if mode == 0:
        assert tuple(y.shape[:3]) == (N, Ho, Wo) and (Cy >= Ngemm or y2 is not None), (tuple(y.shape), out_grid, Ngemm)
    else:
        assert tuple(y.shape[:3]) == (N, 2 * Ho, 2 * Wo) and Cy >= Cout and Ngemm == 4 * Cout
    # gathered source extent must stay inside x
    assert (Ho - 1) * stride + KH - 1 - pad <= Hs - 1 + pad and (Wo - 1) * stride + KW - 1 - pad <= Ws - 1 + pad
    ldm = mch = 0
    if mask is not None:
        Nm, Hm, Wm, Cm, ldm = _nhwc(mask, "igemm.mask")
        assert (Nm, Hm, Wm) == (N, Ho, Wo) and mode == 0
        mch = min(Cm, Ngemm)
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous() and bias.numel() >= (Cout or Ngemm)
    ldp = 0
    if pool is not None:
        Np, Hp, Wp, Cp, ldp = _nhwc(pool, "igemm.pool")
        assert (Np, Hp, Wp) == (N, Ho // 2, Wo // 2) and Cp >= Ngemm and mode == 0
    if pcode is not None:
        assert pool is not None and y2 is None and pcode.dtype == torch.uint8 and pcode.is_contiguous()
        assert tuple(pcode.shape) == (N, Ho // 2, Wo // 2, Ngemm)
    ldy2 = 0
    if y2 is not None:
        N2, H2, W2, C2, ldy2 = _nhwc(y2, "igemm.y2")
        assert mode == 0 and not accumulate and (N2, H2, W2) == (N, Ho, Wo) and split % 16 == 0
        assert 0 < split < Ngemm and C2 >= Ngemm - split and Cy >= split
    L = _lib.lib()
    st = _stream(y)
    hslab = None
    bslab = None
    want_bn = False
    if bn_stats is not None and USE_FUSED_BN and mode == 0 and pool is None and y2 is None and head is None \
            and not accumulate and not relu and path == "auto" and (mask is None or mch == Ngemm):
        bslab = torch.empty(N * -(-Ho // 16) * -(-Wo // 64) * 2 * Ngemm, dtype=torch.float32, device=y.device)
    if xbn is not None:
        # with a dual input only x (channels < 32) is formed on load: xbn = [scale 32 | shift 32]
        assert bslab is not None and mask is None and Cs != 8, "BN-on-load: the BN-statistics stream conv"
        assert xbn.dtype == torch.float32 and xbn.is_contiguous() and xbn.numel() == (64 if x2 is not None else 2 * Cs)
    hprob = None
    if head is not None:
        hw, hb, tgt = head[:3]
        hprob = head[3] if len(head) > 3 else None
        assert hprob is None or (hprob.dtype == torch.float32 and hprob.is_contiguous() and hprob.numel() == N * Ho * Wo)
        assert mode == 0 and Ngemm == 32 and Cs == 32 and pool is None and y2 is None and mask is None
        assert hw.dtype == torch.float32 and hw.is_contiguous() and hw.numel() == 32 and hb.numel() == 1
        assert tgt.dtype == torch.float32 and tgt.is_contiguous() and tgt.numel() == N * Ho * Wo
        hslab = torch.empty((N * -(-Ho // 16) * -(-Wo // 64) + 1) * 4, dtype=torch.float32, device=y.device)
    def args(n0, n1, per_image):
        xs, ys = x[n0:n1], y[n0:n1]
        nb = n1 - n0
        a = IgemmArgs(xs.data_ptr(), _p(wpacked).value, None if bias is None else bias.data_ptr(), ys.data_ptr(),
                      None if mask is None else mask[n0:n1].data_ptr(), ldx, ldy, ldm, mch, nb, Ho, Wo, Hs, Ws, Cs,
                      KH, KW, stride, pad, Ngemm, Kpad, mode, int(relu), int(accumulate), Cout,
                      0 if per_image else _extent_bytes(nb, Hs, Ws, Cx, ldx), None, 0, None,
                      None if y2 is None else y2[n0:n1].data_ptr(), ldy2, split)
        if x2 is not None:
            a.x2 = x2[n0:n1].data_ptr()
            a.ximg = _extent_bytes(1, Hs, Ws, 32, ldx)
        else:
            a.ximg = _extent_bytes(1, Hs, Ws, Cx, ldx)
        return a

    conv3 = mode == 0 and KH == 3 and stride == 1 and cfg == 0
    stream_ok = (Ngemm in (32, 64) and Cs in (32, 64)) or (Ngemm in (32, 64) and Cs == 8 and pool is None)
    # ---- per-image kernels (row-streaming, row-halo): each block binds one image, so ONE launch
    # covers the whole batch (no 2 GiB chunks, no chunk tails)
    per_image_ok = Hs * Ws * ldx * 2 < _MAX_BYTES
    a = args(0, N, True) if per_image_ok else None
    if head is not None:
        rows = L.dpa_igemm_stream_blocks(ctypes.byref(a)) if a is not None else 0
        assert conv3 and stream_ok and 0 < rows and (rows + 1) * 4 <= hslab.numel() and path in ("auto", "stream"), \
            "fused head needs the stream kernel"
        a.hw, a.hb, a.tgt, a.hslab = hw.data_ptr(), hb.data_ptr(), tgt.data_ptr(), hslab.data_ptr()
        a.hprob = None if hprob is None else hprob.data_ptr()
        _check(L.dpa_igemm_stream(ctypes.byref(a), c_int(0), st), "igemm_stream+head")
        S = hslab[hslab.numel() - 4:]
        _check(L.dpa_slab_sum(_p(hslab), c_int(rows), c_int(4), _p(S), st), "slab_sum")
        return S
    done = False
    if bslab is not None:
        if a is not None and conv3 and stream_ok and USE_STREAM and (Cs != 8 or xbn is None):
            rows = L.dpa_igemm_stream_blocks(ctypes.byref(a))
            if rows > 0 and rows * 2 * Ngemm <= bslab.numel():
                a.bnslab = bslab.data_ptr()
                a.xbn = None if xbn is None else xbn.data_ptr()
                err = L.dpa_igemm_stream(ctypes.byref(a), c_int(0), st)
                if err == 0:
                    bn_stats.extend([bslab, rows])
                    return
                if xbn is not None:
                    _check(err, "igemm_stream(BN-on-load)")
                a.bnslab = a.xbn = None
        assert xbn is None, "BN-on-load: only the row-streaming BN-statistics conv forms the input on load"
        # not fusable here: the BN pass computes the statistics (the same epilogue in the row-halo
        # kernel measured 4% slower end to end: its extra registers cost more than the pass it saves),
        # unless the row-block GEMM (below) takes the conv: its epilogue writes one slab row per tile
        bslab = None
        want_bn = True
    if _ABLATE and path == "auto":
        fam = ("stream" if (a is not None and USE_STREAM and conv3 and stream_ok) else
               "halo" if (a is not None and USE_HALO and conv3 and Cs % 32 == 0 and Ngemm <= 128) else
               "glds" if (USE_GLDS and cfg == 0 and Cs % 64 == 0 and Kpad % 64 == 0 and Ngemm % 128 == 0) else "generic")
        if fam in _ABLATE:
            return
    if a is not None and (path == "stream" or (path == "auto" and USE_STREAM and conv3 and stream_ok)):
        if pool is not None:
            a.pool, a.ldp = pool.data_ptr(), ldp
            a.pcode = None if pcode is None else pcode.data_ptr()
        err = L.dpa_igemm_stream(ctypes.byref(a), c_int(variant), st)
        if err == 0:
            return
        a.pool, a.ldp, a.pcode = None, 0, None
        if path == "stream" or x2 is not None:
            _check(err, "igemm_stream")
    assert x2 is None, "dual input: only the row-streaming kernel reads it"
    # measured at batch 128 (tools/kbench.py, profiles/kbench_b128_512.txt): the two-row halo kernel
    # beats the LDS-DMA kernel on every shape both accept (128-channel dgrads: 837 vs 1042 us at
    # 128^2, 2542 vs 2948 us at 256^2); the LDS-DMA kernel takes what the halo kernel cannot
    # (64^2 and smaller grids, > 128 output channels)
    # whole-row 256-pixel tiles, slice-major K, N % 256 != 0 (N % 256 == 0 takes cfg 14's 256-channel form)
    rb128 = (path == "auto" and USE_GLDS128 and USE_GLDS and conv3 and pad == 1 and
             (Hs, Ws) == (Ho, Wo) and Kpad == 9 * Cs and Cs % 64 == 0 and (Wo in (32, 64, 128) or Wo % 256 == 0) and
             (Ho * Wo) % 256 == 0 and Ngemm % 128 == 0 and Ngemm % 256 != 0)
    # 64 output channels from >= 64 (not the row-streaming shapes): whole-row 512-pixel tiles, slice-major K
    slp64 = (path == "auto" and USE_SLP64 and USE_GLDS and conv3 and pad == 1 and (Hs, Ws) == (Ho, Wo) and
             Kpad == 9 * Cs and Cs % 32 == 0 and Cs >= 64 and Ngemm == 64 and Wo in (32, 64, 128, 256) and
             (Ho * Wo) % 512 == 0 and xbn is None)
    if (a is not None and not rb128 and not slp64 and
            (path == "halo" or (path == "auto" and USE_HALO and conv3 and Cs % 32 == 0 and Ngemm <= 128))):
        err = L.dpa_igemm_halo(ctypes.byref(a), c_int(variant if path == "halo" else HALO_CFG), st)
        if err == 0:
            done = True
        elif path == "halo":
            _check(err, "igemm_halo")
    # ---- chunked kernels (LDS-DMA GEMM, generic gather): 32-bit offsets over the whole chunk
    glds_ok = USE_GLDS and cfg == 0 and Cs % 64 == 0 and Kpad % 64 == 0 and Ngemm % 128 == 0
    # BatchNorm partial sums from the row-block GEMM's epilogue (csrc/igemm_glds.hip glds_epilogue_bns):
    # bnslab[M / 256][2][Ngemm]; the kernel refuses shapes it cannot take (then the BN pass computes them)
    gslab = None
    if want_bn and not done and path == "auto" and glds_ok and (Ho * Wo) % 256 == 0 and USE_GLDS_BN:
        gslab = torch.empty(N * Ho * Wo // 256 * 2 * Ngemm, dtype=torch.float32, device=y.device)
    for n0, n1 in ([] if done else _image_chunks(N, max(Hs * Ws * ldx, (4 if mode else 1) * Ho * Wo * ldy) * 2)):
        a = args(n0, n1, False)
        if gslab is not None:
            a.bnslab = gslab[n0 * Ho * Wo // 256 * 2 * Ngemm:].data_ptr()
            if L.dpa_igemm_glds(ctypes.byref(a), c_int(variant), st) == 0:
                continue
            assert n0 == 0, "row-block BN statistics refused after the first chunk"
            a.bnslab, gslab = None, None
        if slp64:
            _check(L.dpa_igemm_glds(ctypes.byref(a), c_int(524288), st), "igemm_slp<64>")
            continue
        if path == "glds" or (path == "auto" and glds_ok):
            no_pers = not persistent
            # 128 output channels: the slice-staged 128 x 512 kernel (cfg 18) on rows of <= 128 pixels,
            # the 128-channel row-block kernel (15) otherwise; else the library's auto choice
            sl = USE_GLDS_SL and Wo in (32, 64, 128) and (Ho * Wo) % 512 == 0 and Cs % 32 == 0
            auto_cfg = (262144 if sl else 15) if rb128 else 32 * no_pers + (0 if USE_GLDS_SL else 1048576)
            err = L.dpa_igemm_glds(ctypes.byref(a), c_int(variant if path == "glds" else auto_cfg), st)
            if err == 0:
                continue
            if path == "glds":
                _check(err, "igemm_glds")
        _check(L.dpa_igemm(ctypes.byref(a), c_int(cfg), st), "igemm")
    if gslab is not None:
        bn_stats.extend([gslab, N * Ho * Wo // 256])
    if pool is not None:
        maxpool2(y, pool, pcode)


def head_fusable(N: int, H: int, W: int, Cin: int, Cout: int) -> bool:
    """Can the last decoder conv (Cin -> Cout = 32) carry the segmentation head in its epilogue?"""
    return USE_STREAM and USE_FUSED_HEAD and Cin == 32 and Cout == 32 and W >= 16 and H * W * Cin * 2 < _MAX_BYTES


# ------------------------------------------------------------------------------------------ wgrad
def wgrad_splits(P: int, tiles: int, target_blocks: int = 1024, min_pix: int = 512):
    splits = max(1, min(target_blocks // max(tiles, 1), P // min_pix))
    pps = round_up(-(-P // splits), 32)
    splits = -(-P // pps)
    return splits, pps


def wgrad_bn_eligible(M: int, Nc: int, W: int) -> bool:
    """Can :func:`wgrad` form a BatchNorm backward on load of its gradient (``abn``)?  The first conv
    (8-padded RGB input) on the row-streaming kernel."""
    return USE_STREAM and Nc == 8 and M % 32 == 0 and W >= 8 and "wgrad" not in _ABLATE


def wgrad(A: torch.Tensor, B: torch.Tensor, *, kind: int, grid, M: int, Nc: int, s: int, pad: int, KW: int,
          gw: torch.Tensor, gb: Optional[torch.Tensor], Nreal: int, cfg: int = 0, target_blocks: int = 1024,
          path: str = "auto", abn=None, sink: Optional["SlabSink"] = None):
    """Weight (+bias) gradient of a conv3x3 (kind 0), transposed conv 2x2/s2 (kind 1) or conv1x1
    (kind 2); accumulates into gw/gb.

    ``path``: ``auto`` = row-streaming kernel when W % 64 == 0, else row-halo (W % 32 == 0), else the
    generic per-tap gather kernel; ``stream`` / ``halo`` / ``generic`` force one.
    ``abn`` = (z, coef3): ``A`` is the ReLU-masked gradient of a BatchNorm output whose input is ``z``; the
    GEMM uses dz = coef3[m] A + coef3[M + m] z + coef3[2M + m] formed on load (:func:`bn_bwd_coef`), so the
    dz pass over HBM never happens (:func:`wgrad_bn_eligible` shapes).  ``sink`` (:class:`SlabSink`): the
    row-streaming kernel writes its slab rows there and the reduction is left to the sink (row-streaming
    shapes only: :func:`wgrad_multi_eligible`)."""
    if sink is not None:
        assert abn is None and kind == 0 and cfg == 0 and path == "auto" and not _ABLATE
        assert wgrad_multi_eligible(M, Nc, grid[2]) and not wgrad_band_eligible(M, Nc, grid) and \
            not wgrad_band128_eligible(M, Nc, grid) and not wgrad_gemm_eligible(M, Nc, grid), "sink: stream shapes"
        return _wgrad_stream(A, B, grid=grid, M=M, Nc=Nc, gw=gw, gb=gb, Nreal=Nreal, sink=sink)
    if abn is not None:
        assert kind == 0 and cfg == 0 and path in ("auto", "stream") and wgrad_bn_eligible(M, Nc, grid[2])
        return _wgrad_stream(A, B, grid=grid, M=M, Nc=Nc, gw=gw, gb=gb, Nreal=Nreal, abn=abn)
    if _ABLATE and ("wgrad" in _ABLATE or ("wgrad_deep" in _ABLATE and (M >= 128 or Nc >= 128))):
        return
    if (path == "band" or (path == "auto" and wgrad_band_eligible(M, Nc, grid))) and kind == 0 and cfg == 0 \
            and A.shape[1:3] == B.shape[1:3] == tuple(grid[1:]):
        return _wgrad_band(A, B, grid=grid, M=M, Nc=Nc, gw=gw, gb=gb, Nreal=Nreal)
    if (path == "band128" or (path == "auto" and wgrad_band128_eligible(M, Nc, grid))) and kind == 0 and cfg == 0 \
            and A.shape[1:3] == B.shape[1:3] == tuple(grid[1:]):
        return _wgrad_band128(A, B, grid=grid, M=M, Nc=Nc, gw=gw, gb=gb, Nreal=Nreal)
    if (path == "gemm" or (path == "auto" and wgrad_gemm_eligible(M, Nc, grid))) and kind == 0 and cfg == 0 \
            and A.shape[1:3] == B.shape[1:3] == tuple(grid[1:]):
        return _wgrad_gemm(A, B, grid=grid, M=M, Nc=Nc, gw=gw, gb=gb, Nreal=Nreal)
    if (path == "up" or (path == "auto" and wgrad_up_eligible(M, Nc, grid))) and kind == 1 and cfg == 0 \
            and A.shape[1:3] == (2 * grid[1], 2 * grid[2]) and Nreal == Nc:
        return _wgrad_up(A, B, grid=grid, M=M, Nc=Nc, gw=gw, gb=gb, Nreal=Nreal)
    if path in ("auto", "stream") and kind == 0 and cfg == 0 and (USE_STREAM or path == "stream") \
            and grid[2] >= 8 and M % 32 == 0 and (Nc % 32 == 0 or Nc == 8):
        return _wgrad_stream(A, B, grid=grid, M=M, Nc=Nc, gw=gw, gb=gb, Nreal=Nreal)
    if path == "stream":
        raise RuntimeError("wgrad stream path not eligible for this shape")
    NA, HA, WA, CA, lda = _nhwc(A, "wgrad.A")
    NB, HB, WB, CB, ldb = _nhwc(B, "wgrad.B")
    N, Hg, Wg = grid
    assert NA == NB == N and CA >= M and CB >= Nc and M % 32 == 0
    T = {0: 9, 1: 4, 2: 1}[kind]
    if kind in (0, 2):
        assert (HA, WA) == (Hg, Wg) and (HB, WB) == (Hg, Wg)
    else:
        assert (HA, WA) == (2 * Hg, 2 * Wg) and (HB, WB) == (Hg, Wg)
    halo = ((USE_HALO or path == "halo") and path != "generic" and kind == 0 and cfg == 0 and Wg % 32 == 0
            and Nc % 32 == 0 and M % 32 == 0)
    if halo:
        hcfg = 2 if M % 64 == 0 else (3 if Nc % 64 == 0 else 1)
        bm, bn = {1: (32, 32), 2: (64, 32), 3: (32, 64), 4: (64, 64)}[hcfg]
    else:
        if cfg == 0:
            if kind == 0:
                cfg = 1 if Nc <= 16 else (3 if M % 64 == 0 else 2)
            elif kind == 1:
                cfg = 14 if (M % 64 == 0 and Nc % 128 == 0) else (12 if (M % 64 == 0 and Nc >= 64) else 11)
            else:
                cfg = 22 if (M % 64 == 0 and Nc >= 64) else 21
        bm, bn = {1: (32, 16), 2: (32, 32), 3: (64, 32), 4: (64, 64), 11: (32, 32), 12: (64, 64), 13: (128, 64),
                  14: (64, 128), 21: (32, 32), 22: (64, 64)}[cfg]
    tiles = (M // bm) * (-(-Nc // bn))
    assert gw.dtype == torch.float32 and gw.is_contiguous() and gw.numel() == M * Nreal * T
    L = _lib.lib()
    st = _stream(A)
    for n0, n1 in _image_chunks(N, max(HA * WA * lda, HB * WB * ldb) * 2):
        nb = n1 - n0
        P = nb * Hg * Wg
        splits, pps = wgrad_splits(P, tiles, target_blocks)
        slab = torch.empty(splits * T * M * Nc + splits * M, dtype=torch.float32, device=A.device)
        bslab = slab[splits * T * M * Nc:] if gb is not None else None
        a = WgradArgs(A[n0:n1].data_ptr(), B[n0:n1].data_ptr(), slab.data_ptr(),
                      None if bslab is None else bslab.data_ptr(), lda, ldb, nb, Hg, Wg, HA, WA, HB, WB, M, Nc, s,
                      pad, KW, pps, splits, _extent_bytes(nb, HA, WA, CA, lda), _extent_bytes(nb, HB, WB, CB, ldb))
        if kind == 2:
            assert s == 1 and pad == 0 and KW == 1
        if halo:
            _check(L.dpa_wgrad_halo(ctypes.byref(a), c_int(hcfg), st), "wgrad_halo")
        else:
            _check(L.dpa_wgrad(ctypes.byref(a), c_int(kind), c_int(cfg), st), "wgrad")
        _check(L.dpa_wgrad_reduce(_p(slab), _p(bslab), _p(gw), _p(gb), c_int(splits), c_int(T), c_int(M), c_int(Nc),
                                  c_int(Nreal), c_int(1 if kind == 1 else 0), st), "wgrad_reduce")


WGRAD_STREAM_BLOCKS = CFG.wgrad_stream_blocks


def wgrad_multi_eligible(M: int, Nc: int, W: int) -> bool:
    """Can :func:`wgrad_multi` take this conv3x3 weight gradient (row-streaming or row kernels)?"""
    return USE_STREAM and W >= 8 and M % 32 == 0 and (Nc % 32 == 0 or Nc == 8) and "wgrad" not in _ABLATE


# deep-layer weight gradients as a dense 256x256 LDS-DMA GEMM on the ping-pong schedule
# (csrc/wgrad_gemm.hip); DPA_NO_WGRAD_GEMM=1 falls back to the row-streaming kernel
USE_WGRAD_GEMM = CFG.wgrad_gemm
WGRAD_GEMM_BLOCKS = CFG.wgrad_gemm_blocks


def wgrad_gemm_eligible(M: int, Nc: int, grid) -> bool:
    N, H, W = grid
    return (USE_WGRAD_GEMM and M % 256 == 0 and Nc % 8 == 0 and Nc >= 64 and (W % 64 == 0 or W == 32)
            and (H * W) % 64 == 0)


def _wgrad_gemm(A, B, *, grid, M, Nc, gw, gb, Nreal, blocks: int = 0, tabs=None, group: int = 0):
    """conv3x3 weight (+bias) gradient of the deep layers (M = Cout % 256 == 0): one workgroup per
    (group of images, 256 x 256 tile of dW[co][tap, ci]); split-K slabs over the image groups.
    ``tabs`` = per-image pointer tables (the images of ``group``-image tensors: every split stays
    inside one of them)."""
    NA, HA, WA, CA, lda = _nhwc(A, "wgrad_gemm.A")
    NB, HB, WB, CB, ldb = _nhwc(B, "wgrad_gemm.B")
    N, Hg, Wg = grid
    assert (HA, WA) == (Hg, Wg) == (HB, WB) and CA >= M and CB >= Nc
    assert (NA == NB == N) or (tabs is not None and tabs[0].numel() == tabs[1].numel() == N and group > 0
                               and N % group == 0)
    assert gw.dtype == torch.float32 and gw.is_contiguous() and gw.numel() == M * Nreal * 9
    tiles = (M // 256) * -(-9 * Nc // 256)
    spi = Hg * Wg // 64
    ips = max(1, -(-N * tiles // (blocks or WGRAD_GEMM_BLOCKS)), -(-2 // spi))
    # 32-bit offsets inside one split's images
    ips = max(1, min(ips, _MAX_BYTES // (Hg * Wg * max(lda, ldb) * 2)))
    if tabs is not None:
        while group % ips:        # a split never straddles two tensors
            ips -= 1
        assert ips * spi >= 2
    splits = -(-N // ips)
    slab = torch.empty(splits * 9 * M * Nc + splits * M, dtype=torch.float32, device=A.device)
    bslab = slab[splits * 9 * M * Nc:] if gb is not None else None
    a = WgradArgs(A.data_ptr(), B.data_ptr(), slab.data_ptr(), None if bslab is None else bslab.data_ptr(), lda, ldb,
                  N, Hg, Wg, HA, WA, HB, WB, M, Nc, 1, 1, 3, ips, splits, ips * Hg * Wg * lda * 2,
                  ips * Hg * Wg * ldb * 2)
    if tabs is not None:
        a.atab, a.btab = tabs[0].data_ptr(), tabs[1].data_ptr()
    L = _lib.lib()
    st = _stream(A)
    _check(L.dpa_wgrad_gemm(ctypes.byref(a), st), "wgrad_gemm")
    _check(L.dpa_wgrad_reduce(_p(slab), _p(bslab), _p(gw), _p(gb), c_int(splits), c_int(9), c_int(M), c_int(Nc),
                              c_int(Nreal), c_int(0), st), "wgrad_reduce(gemm)")


# transposed-conv (k2 s2) weight gradients on the dense LDS-DMA GEMM (csrc/wgrad_gemm.hip up mode) instead of the
# register-staged split-K kernel; DPA_NO_WGRAD_UP=1 falls back
USE_WGRAD_UP = CFG.wgrad_up


def wgrad_up_eligible(Cout: int, Cin: int, grid) -> bool:
    """Can the transposed conv Cin -> Cout on the low-resolution ``grid`` take :func:`_wgrad_up`?"""
    N, h, w = grid
    spi = h * w // 64
    # one workgroup per (image, tile) at most: with fewer than 128 of them the split-K kernel is faster
    # (UNet-XL 1024^2 b16, 256 -> 128: 32 workgroups, 409 vs 209 us; profiles/kbench_deconv_wgrad_up_r06.txt)
    tiles = (Cin // 256) * (4 * Cout // 256) if Cin % 256 == 0 and (4 * Cout) % 256 == 0 else 0
    return (USE_WGRAD_UP and tiles > 0 and N * tiles >= 128 and Cout % 8 == 0 and (h * w) % 64 == 0
            and (w % 64 == 0 or (w < 64 and 64 % w == 0)) and spi >= 2)


def _wgrad_up(A, B, *, grid, M, Nc, gw, gb, Nreal):
    """Weight (+bias) gradient of a transposed conv k2 s2 (``A`` = output gradient [N, 2h, 2w, >= M], M = Cout;
    ``B`` = layer input [N, h, w, >= Nc], Nc = Cin) as the dense GEMM dW[ci][tap][co] = sum_p x[p][ci] *
    g[2p + tap][co] (wgrad_gemm.hip up mode: the input is the GEMM's A operand, the gradient the 4-tap B
    operand); slab rows [split][tap][Cin][Cout] reduced straight into the ConvTranspose2d layout.  The bias
    gradient (no bias column in that kernel) is a per-channel sum of the gradient (dpa_chan_sum_bf16)."""
    NA, HA, WA, CA, lda = _nhwc(A, "wgrad_up.A")
    NB, HB, WB, CB, ldb = _nhwc(B, "wgrad_up.B")
    N, h, w = grid
    assert NA == NB == N and (HA, WA) == (2 * h, 2 * w) and (HB, WB) == (h, w) and CA >= M and CB >= Nc
    assert Nreal == Nc and gw.dtype == torch.float32 and gw.is_contiguous() and gw.numel() == M * Nc * 4
    tiles = (Nc // 256) * (4 * M // 256)
    spi = h * w // 64
    ips = max(1, -(-N * tiles // WGRAD_GEMM_BLOCKS), -(-2 // spi))
    ips = max(1, min(ips, _MAX_BYTES // (4 * h * w * max(lda, ldb) * 2)))
    splits = -(-N // ips)
    slab = torch.empty(splits * 4 * Nc * M, dtype=torch.float32, device=A.device)
    a = WgradArgs(B.data_ptr(), A.data_ptr(), slab.data_ptr(), None, ldb, lda, N, h, w, h, w, 2 * h, 2 * w, Nc, M,
                  2, 0, 2, ips, splits, ips * h * w * ldb * 2, ips * 4 * h * w * lda * 2)
    L = _lib.lib()
    st = _stream(A)
    _check(L.dpa_wgrad_gemm(ctypes.byref(a), st), "wgrad_gemm(up)")
    _check(L.dpa_wgrad_reduce(_p(slab), None, _p(gw), None, c_int(splits), c_int(4), c_int(Nc), c_int(M), c_int(M),
                              c_int(0), st), "wgrad_reduce(up)")
    if gb is not None:
        P = N * 4 * h * w
        nblk = max(1, min(1024, P * (M // 8) // 4096))
        part = torch.empty(nblk * M, dtype=torch.float32, device=A.device)
        _check(L.dpa_chan_sum_bf16(_p(A), ctypes.c_longlong(P), c_int(M), c_int(lda), _p(part), c_int(nblk), _p(gb),
                                   st), "chan_sum_bf16")


# deep-layer weight gradients with the input band staged once for all nine taps (csrc/wgrad_band.hip):
# 256 output channels x (9 taps x 32 input channels) per workgroup; DPA_NO_WGRAD_BAND=1 -> wgrad_gemm
USE_WGRAD_BAND = CFG.wgrad_band


def wgrad_band_eligible(M: int, Nc: int, grid) -> bool:
    N, H, W = grid
    return USE_WGRAD_BAND and M % 256 == 0 and Nc % 32 == 0 and W in (32, 64) and H % (64 // W) == 0


def wgrad_band_ips(N: int, H: int, W: int, M: int, Nc: int, group: int = 0, cus: int = 256,
                   min_blocks: int = 512) -> int:
    """Images per split of a band launch: the fewest rounds of workgroups over the CUs (one 140-KB workgroup
    per CU) times the work per workgroup, plus the fp32 slab traffic of the split-K partials; at least
    ``min_blocks`` workgroups when the batch allows (room to interleave with the other stream's kernels).
    ``group``: splits stay inside ``group``-image tensors (per-image tables)."""
    tiles = (M // 256) * (Nc // 32)
    steps = H * W // 64
    t_step, bw = 1.6e-6, 4e12                     # ~60 % MFMA per K-step (9.4 MFLOP); slab write + read
    best = None
    for ips in range(1, N + 1):
        if group and group % ips:
            continue
        splits = -(-N // ips)
        blocks = splits * tiles
        cost = -(-blocks // cus) * ips * steps * t_step + splits * 9 * M * Nc * 8 / bw
        key = (blocks < min(min_blocks, N * tiles), cost)
        if best is None or key < best[0]:
            best = (key, ips)
    return best[1]


def wgrad_band128_eligible(M: int, Nc: int, grid) -> bool:
    """The 128-output-channel band kernel (csrc/wgrad_band.hip wgrad_band128_kernel): W % 64 == 0 grids
    the 256-channel form does not take (the 128^2 level of the UNet)."""
    N, H, W = grid
    return (USE_WGRAD_BAND and M % 128 == 0 and Nc % 64 == 0 and W % 64 == 0 and W >= 64
            and not wgrad_band_eligible(M, Nc, grid))


def wgrad_band128_steps(N: int, H: int, W: int, M: int, Nc: int, group: int = 0, cus: int = 256,
                        min_blocks: int = 512) -> int:
    """K-steps (64 pixels) per split of a 128-channel band launch: whole images or an image's 1/2 .. 1/32
    (splits may start inside an image); the cost model of :func:`wgrad_band_ips`.  ``group``: whole-image
    splits inside ``group``-image tensors."""
    tiles = (M // 128) * (Nc // 64)
    spi = H * W // 64
    total = N * spi
    cands = {spi * i for i in range(1, N + 1) if not group or group % i == 0}
    if not group:
        cands |= {spi // k for k in (2, 4, 8, 16, 32) if spi % k == 0}
    t_step, bw = 1.6e-6, 4e12
    best = None
    for sps in sorted(cands):
        splits = -(-total // sps)
        blocks = splits * tiles
        cost = -(-blocks // cus) * sps * t_step + splits * 9 * M * Nc * 8 / bw
        key = (blocks < min(min_blocks, total * tiles), cost)
        if best is None or key < best[0]:
            best = (key, sps)
    return best[1]


def _wgrad_band128(A, B, *, grid, M, Nc, gw, gb, Nreal, tabs=None, group: int = 0, steps: int = 0):
    """conv3x3 weight (+bias) gradient of 128-output-channel tiles on W % 64 == 0 grids: one workgroup per
    (range of 64-pixel K-steps, 128 output channels x 64 input channels x 9 taps); split-K slabs reduced by
    dpa_wgrad_reduce (same slab layout as :func:`_wgrad_gemm`)."""
    NA, HA, WA, CA, lda = _nhwc(A, "wgrad_band128.A")
    NB, HB, WB, CB, ldb = _nhwc(B, "wgrad_band128.B")
    N, Hg, Wg = grid
    assert (HA, WA) == (Hg, Wg) == (HB, WB) and CA >= M and CB >= Nc
    assert (NA == NB == N) or (tabs is not None and tabs[0].numel() == tabs[1].numel() == N and group > 0
                               and N % group == 0)
    assert gw.dtype == torch.float32 and gw.is_contiguous() and gw.numel() == M * Nreal * 9
    HW = Hg * Wg
    sps = steps or wgrad_band128_steps(N, Hg, Wg, M, Nc, group if tabs is not None else 0)
    # 32-bit offsets over a split's span from its first image
    while sps > 1 and (sps * 64 + 2 * HW) * max(lda, ldb) * 2 >= 2 ** 31:
        sps = sps - HW // 64 if sps > HW // 64 else sps // 2
    pps = sps * 64
    splits = -(-N * HW // pps)
    slab = torch.empty(splits * 9 * M * Nc + splits * M, dtype=torch.float32, device=A.device)
    bslab = slab[splits * 9 * M * Nc:] if gb is not None else None
    a = WgradArgs(A.data_ptr(), B.data_ptr(), slab.data_ptr(), None if bslab is None else bslab.data_ptr(), lda, ldb,
                  N, Hg, Wg, HA, WA, HB, WB, M, Nc, 1, 1, 3, pps, splits, pps * lda * 2, pps * ldb * 2)
    if tabs is not None:
        assert pps % HW == 0 and group % (pps // HW) == 0
        a.atab, a.btab = tabs[0].data_ptr(), tabs[1].data_ptr()
    L = _lib.lib()
    st = _stream(A)
    _check(L.dpa_wgrad_band128(ctypes.byref(a), st), "wgrad_band128")
    _check(L.dpa_wgrad_reduce(_p(slab), _p(bslab), _p(gw), _p(gb), c_int(splits), c_int(9), c_int(M), c_int(Nc),
                              c_int(Nreal), c_int(0), st), "wgrad_reduce(band128)")


def _wgrad_band(A, B, *, grid, M, Nc, gw, gb, Nreal, tabs=None, group: int = 0, ips: int = 0):
    """conv3x3 weight (+bias) gradient of the deep layers (64^2 / 32^2 grids, Cout % 256 == 0): one
    workgroup per (group of images, 256 output channels x 32 input channels x 9 taps); split-K slabs over
    the image groups, reduced by dpa_wgrad_reduce (same slab layout as :func:`_wgrad_gemm`)."""
    NA, HA, WA, CA, lda = _nhwc(A, "wgrad_band.A")
    NB, HB, WB, CB, ldb = _nhwc(B, "wgrad_band.B")
    N, Hg, Wg = grid
    assert (HA, WA) == (Hg, Wg) == (HB, WB) and CA >= M and CB >= Nc
    assert (NA == NB == N) or (tabs is not None and tabs[0].numel() == tabs[1].numel() == N and group > 0
                               and N % group == 0)
    assert gw.dtype == torch.float32 and gw.is_contiguous() and gw.numel() == M * Nreal * 9
    ips = ips or wgrad_band_ips(N, Hg, Wg, M, Nc, group if tabs is not None else 0)
    ips = max(1, min(ips, (_MAX_BYTES - 1) // (Hg * Wg * max(lda, ldb) * 2)))
    if tabs is not None:
        while group % ips:        # a split never straddles two tensors
            ips -= 1
    splits = -(-N // ips)
    slab = torch.empty(splits * 9 * M * Nc + splits * M, dtype=torch.float32, device=A.device)
    bslab = slab[splits * 9 * M * Nc:] if gb is not None else None
    a = WgradArgs(A.data_ptr(), B.data_ptr(), slab.data_ptr(), None if bslab is None else bslab.data_ptr(), lda, ldb,
                  N, Hg, Wg, HA, WA, HB, WB, M, Nc, 1, 1, 3, ips, splits, ips * Hg * Wg * lda * 2,
                  ips * Hg * Wg * ldb * 2)
    if tabs is not None:
        a.atab, a.btab = tabs[0].data_ptr(), tabs[1].data_ptr()
    L = _lib.lib()
    st = _stream(A)
    _check(L.dpa_wgrad_band(ctypes.byref(a), st), "wgrad_band")
    _check(L.dpa_wgrad_reduce(_p(slab), _p(bslab), _p(gw), _p(gb), c_int(splits), c_int(9), c_int(M), c_int(Nc),
                              c_int(Nreal), c_int(0), st), "wgrad_reduce(band)")


def _image_table(ts, C_min: int, name: str):
    """Device array of per-image base pointers over the images of tensors ``ts`` (same H, W, ld)."""
    ptrs, geo = [], None
    for t in ts:
        n, h, w, c, ld = _nhwc(t, name)
        assert c >= C_min and (geo is None or geo == (h, w, ld)), f"{name}: images of different layouts"
        geo = (h, w, ld)
        ptrs.extend(t.data_ptr() + i * h * w * ld * 2 for i in range(n))
    return torch.tensor(ptrs, dtype=torch.int64, device=ts[0].device), len(ptrs)


def wgrad_multi(As, Bs, *, M: int, Nc: int, gw: torch.Tensor, gb: Optional[torch.Tensor], Nreal: int):
    """conv3x3 weight (+bias) gradient over the images of several (gradient, input) tensor pairs in
    ONE launch -- the microbatches of a pipeline stage: one split-K slab set and one reduction for
    the whole batch instead of one per microbatch.  Accumulates into gw / gb."""
    assert len(As) == len(Bs) and As
    N = sum(a.shape[0] for a in As)
    _, H, W, _, _ = _nhwc(As[0], "wgrad_multi.A")
    atab, na = _image_table(As, M, "wgrad_multi.A")
    btab, nb = _image_table(Bs, Nc, "wgrad_multi.B")
    assert na == nb == N
    tabs = (atab, btab)
    sizes = {a.shape[0] for a in As} | {b.shape[0] for b in Bs}
    # splits cannot straddle two microbatch tensors: with few-image microbatches at the deepest levels
    # (UNet-XL, 2 images of 32x32) that means short splits and a slab set several times the batch's
    # dW -- keep the gemm path for >= 64 K-steps per split (profiles/pipeline_rehearsal_r03.txt)
    if wgrad_band_eligible(M, Nc, (N, H, W)) and len(sizes) == 1:
        return _wgrad_band(As[0], Bs[0], grid=(N, H, W), M=M, Nc=Nc, gw=gw, gb=gb, Nreal=Nreal, tabs=tabs,
                           group=sizes.pop())
    if wgrad_band128_eligible(M, Nc, (N, H, W)) and len(sizes) == 1:
        return _wgrad_band128(As[0], Bs[0], grid=(N, H, W), M=M, Nc=Nc, gw=gw, gb=gb, Nreal=Nreal, tabs=tabs,
                              group=sizes.pop())
    if wgrad_gemm_eligible(M, Nc, (N, H, W)) and len(sizes) == 1 and min(sizes) * (H * W // 64) >= 64:
        return _wgrad_gemm(As[0], Bs[0], grid=(N, H, W), M=M, Nc=Nc, gw=gw, gb=gb, Nreal=Nreal, tabs=tabs,
                           group=sizes.pop())
    return _wgrad_stream(As[0], Bs[0], grid=(N, H, W), M=M, Nc=Nc, gw=gw, gb=gb, Nreal=Nreal, tabs=tabs)


def _wgrad_stream_geom(N: int, Hg: int, Wg: int, M: int, Nc: int):
    """(tile cfg, strip width, rows per split, images per split, slab rows) of a row-streaming weight gradient."""
    if Nc == 8:            # first layer (RGB padded to 8 channels): 32x16 tile, half the columns zero
        hcfg = 4
    elif WGRAD_STREAM_CFG in (1, 2, 3) and not (WGRAD_STREAM_CFG == 2 and M % 64) and not (WGRAD_STREAM_CFG == 3 and Nc % 64):
        hcfg = WGRAD_STREAM_CFG
    else:
        hcfg = 2 if M % 64 == 0 else (3 if Nc % 64 == 0 else 1)
    bm, bn = {1: (32, 32), 2: (64, 32), 3: (32, 64), 4: (32, 16)}[hcfg]
    tiles = (M // bm) * (-(-Nc // bn))
    nb = N
    # one launch for the whole batch: the kernel binds one image at a time (per-image extents below).
    # Strip width: 64 pixels unless 32-pixel strips waste less of a ragged row (the first layer's
    # 8-channel tile exists only with 64-pixel strips)
    waste = lambda b: -(-Wg // b) * b - Wg     # noqa: E731
    bp = 64 if (Nc == 8 or waste(64) <= waste(32)) else 32
    strips = -(-Wg // bp)
    rh = 64 if nb * -(-Hg // 64) * strips * tiles >= 1024 else 32
    per_img = -(-Hg // rh) * strips
    # images per split: keep >= ~2048 blocks (8 per CU) but no more slabs than that -- the fp32
    # slab reduction otherwise grows linearly with the batch
    ipb = max(1, (nb * per_img * tiles) // WGRAD_STREAM_BLOCKS)
    splits = -(-nb // ipb) * per_img
    return hcfg, bp, rh, ipb, splits


def _wgrad_stream(A, B, *, grid, M, Nc, gw, gb, Nreal, tabs=None, abn=None, sink=None):
    NA, HA, WA, CA, lda = _nhwc(A, "wgrad.A")
    NB, HB, WB, CB, ldb = _nhwc(B, "wgrad.B")
    N, Hg, Wg = grid
    assert (HA, WA) == (Hg, Wg) == (HB, WB) and CA >= M and CB >= Nc
    assert (NA == NB == N) or (tabs is not None and tabs[0].numel() == tabs[1].numel() == N)
    assert gw.dtype == torch.float32 and gw.is_contiguous() and gw.numel() == M * Nreal * 9
    hcfg, bp, rh, ipb, splits = _wgrad_stream_geom(N, Hg, Wg, M, Nc)
    L = _lib.lib()
    st = _stream(A)
    nb = N
    if sink is not None:
        slab, bslab = sink.take(splits, M, Nc, gb is not None)
    else:
        slab = torch.empty(splits * 9 * M * Nc + splits * M, dtype=torch.float32, device=A.device)
        bslab = slab[splits * 9 * M * Nc:] if gb is not None else None
    a = WgradArgs(A.data_ptr(), B.data_ptr(), slab.data_ptr(), None if bslab is None else bslab.data_ptr(), lda, ldb,
                  nb, Hg, Wg, HA, WA, HB, WB, M, Nc, 1, 1, 3, 0, splits, _extent_bytes(1, HA, WA, CA, lda),
                  _extent_bytes(1, HB, WB, CB, ldb))
    if tabs is not None:
        a.atab, a.btab = tabs[0].data_ptr(), tabs[1].data_ptr()
    if abn is not None:
        z, coef3 = abn
        assert tabs is None and z.dtype == torch.bfloat16 and z.shape == A.shape and z.stride() == A.stride()
        assert coef3.dtype == torch.float32 and coef3.is_contiguous() and coef3.numel() == 3 * M and CA == M
        a.az, a.abn = z.data_ptr(), coef3.data_ptr()
    _check(L.dpa_wgrad_stream(ctypes.byref(a), c_int(hcfg), c_int(bp), c_int(rh), c_int(ipb), st), "wgrad_stream")
    if sink is None:
        _check(L.dpa_wgrad_reduce(_p(slab), _p(bslab), _p(gw), _p(gb), c_int(splits), c_int(9), c_int(M), c_int(Nc),
                                  c_int(Nreal), c_int(0), st), "wgrad_reduce")


def wgrad_stream_rows(N: int, H: int, W: int, M: int, Nc: int) -> int:
    """Slab rows one :func:`wgrad` launch on the row-streaming kernel writes (:class:`SlabSink` sizing)."""
    return _wgrad_stream_geom(N, H, W, M, Nc)[4]


class SlabSink:
    """The split-K weight-gradient slab rows of SEVERAL launches for one layer in one buffer, summed by a
    single dpa_wgrad_reduce (fixed row order) instead of one per launch.  The first encoder level's backward
    runs in image chunks (models/hip_unet.py ``_EncFn``) so each chunk's side-stream weight gradient overlaps
    the next chunk's fused backward; per chunk both streams then paid a presum + reduce, the side one waiting
    ~0.45 ms for dispatch behind the fused backward (profiles/hip_b256_512_summary_r06.txt).  The buffer is
    allocated at the first :meth:`take`, in the stream context of that launch (so it lives in that stream's
    pool), and :meth:`reduce` runs on the same stream."""

    def __init__(self, rows: int, M: int, Nc: int, gw: torch.Tensor, gb: Optional[torch.Tensor], Nreal: int):
        assert gw.dtype == torch.float32 and gw.is_contiguous() and gw.numel() == M * Nreal * 9
        self.rows, self.M, self.Nc, self.Nreal, self.gw, self.gb = rows, M, Nc, Nreal, gw, gb
        self.buf = None
        self.used = 0

    def take(self, n: int, M: int, Nc: int, bias: bool):
        assert (M, Nc, bias) == (self.M, self.Nc, self.gb is not None), "slab sink: another layer's shape"
        assert self.used + n <= self.rows, "slab sink: more rows than sized for"
        if self.buf is None:
            self.buf = torch.empty(self.rows * 9 * M * Nc + (self.rows * M if bias else 0), dtype=torch.float32,
                                   device=self.gw.device)
        slab = self.buf[self.used * 9 * M * Nc:]
        bslab = self.buf[self.rows * 9 * M * Nc + self.used * M:] if bias else None
        self.used += n
        return slab, bslab

    def reduce(self):
        """Sum every row taken into gw / gb (on the current stream) and release the buffer."""
        if self.buf is None:
            return
        M, Nc = self.M, self.Nc
        bslab = self.buf[self.rows * 9 * M * Nc:] if self.gb is not None else None
        _check(_lib.lib().dpa_wgrad_reduce(_p(self.buf), _p(bslab), _p(self.gw), _p(self.gb), c_int(self.used), c_int(9),
                                           c_int(M), c_int(Nc), c_int(self.Nreal), c_int(0),
                                           _stream(self.gw)), "wgrad_reduce(sink)")
        self.buf = None


# ------------------------------------------------------------------------------- fused conv backward
# minimum workgroups of a fused backward launch (image column strips are split into row segments
# below it); more segments = more fp32 weight-gradient slab rows to reduce
BWD_BLOCKS = CFG.bwd_blocks
# launches over fewer than BWD_SMALL_PIXELS output pixels (pipeline microbatches, small batches) aim at
# BWD_BLOCKS_SMALL: each launch's slab rows are reduced separately, and at 1024 blocks per microbatch the
# reductions read 8x the single-batch bytes (2 stages x 8 microbatches: 2690 -> 2760 img/s at 512,
# 256 worse; profiles/knobs_r03_end.txt).  DPA_BWD_BLOCKS set explicitly applies to every launch.
BWD_BLOCKS_SMALL = CFG.bwd_blocks_small
BWD_SMALL_PIXELS = 1 << 25
_BWD_BLOCKS_SET = CFG.bwd_blocks_set
def _strips_ok(W: int, bp: int) -> bool:
    """Whole strips, or a ragged last one that keeps >= 85 % of the strip pixels useful."""
    t = -(-W // bp)
    return W >= 16 and (W % bp == 0 or W * 100 >= 85 * t * bp)


def bwd_fused_eligible(ci: int, co: int, W: int, whole: bool = False) -> bool:
    """csrc/bwd_stream.hip serves conv3x3 s1 p1 with (Cin, Cout) in {32, 64}^2; ``whole``: the fused
    pool / head modes, which need W % strip == 0 (the plain modes mask a ragged last strip)."""
    bp = ctypes.c_int(0)
    pg = _lib.lib().dpa_bwd_stream_geom(c_int(ci), c_int(co), ctypes.byref(bp))
    return pg > 0 and (W % bp.value == 0 if whole else _strips_ok(W, bp.value))


def bwd_pool_foldable(ci: int, co: int) -> bool:
    return bool(_lib.lib().dpa_bwd_stream_pool_ok(c_int(ci), c_int(co)))


def _bwd_rows(N: int, H: int, W: int, bp: int, target_blocks: int = 0):
    """(rows per block, blocks) of a fused-backward launch: whole image columns per block; the rows are split
    only when the batch gives too few blocks."""
    strips = -(-W // bp)
    if not target_blocks:
        target_blocks = BWD_BLOCKS if (_BWD_BLOCKS_SET or N * H * W >= BWD_SMALL_PIXELS) else BWD_BLOCKS_SMALL
    segs = max(1, min(H, -(-target_blocks // max(1, N * strips))))
    rh = -(-H // segs)
    return rh, N * strips * (-(-H // rh))


def bwd_fused_rows(N: int, H: int, W: int, CI: int, CO: int) -> int:
    """Slab rows one :func:`conv_bwd_fused` launch writes (:class:`SlabSink` sizing)."""
    bp = ctypes.c_int(0)
    pg = _lib.lib().dpa_bwd_stream_geom(c_int(CI), c_int(CO), ctypes.byref(bp))
    assert pg > 0
    return _bwd_rows(N, H, W, bp.value)[1] * pg


def conv_bwd_fused(g: Optional[torch.Tensor], x: torch.Tensor, wd: torch.Tensor, Kd: int, gw: torch.Tensor,
                   gb: Optional[torch.Tensor], *, mask: bool, dx: Optional[torch.Tensor] = None,
                   dx2: Optional[torch.Tensor] = None, split: int = 0, target_blocks: int = 0, head=None,
                   pool=None, w1=None, bn=None, bn_stats: bool = False, x2: Optional[torch.Tensor] = None,
                   xbn: Optional[torch.Tensor] = None, ybn: Optional[torch.Tensor] = None,
                   sink: Optional["SlabSink"] = None):
    """Backward of ``y = conv3x3(x) (+bias)`` in one pass (csrc/bwd_stream.hip): returns
    ``dx = conv3x3^T(g)`` (times ``x > 0`` when ``mask``; with ``dx2``/``split`` the channels
    ``>= split`` go to ``dx2``) and ACCUMULATES the weight gradient into ``gw`` (PyTorch OIHW
    layout, fp32) and the bias gradient into ``gb``.  ``g`` is the gradient w.r.t. the conv output
    (ReLU mask already applied), ``wd`` the dgrad-packed weights ``[Cin][Kd]``.

    ``head`` = (target fp32 [N*H*W], segmap weight [C], segmap bias [1], dS [4], segmap weight grad,
    segmap bias grad, the forward's probabilities fp32 [N*H*W]): ``g`` is then the conv's OUTPUT y (the
    last decoder conv, whose epilogue computed the fused head + loss partials -- and stored p -- in the
    forward) and the head backward (``head_bwd``) is folded into the loader: the gradient is formed
    from (y, p) on the fly and never stored; the segmap gradients accumulate into the weight / bias grads.

    ``pool`` = (window codes uint8 [N, H/2, W/2, Cout], pooled gradient [N, H/2, W/2, Cout]): the conv
    is an encoder conv2 whose output was max-pooled in its forward epilogue; ``g`` is then the skip
    gradient (or None) and the max-pool backward (``pool_bwd_code``) is folded into the loader.

    ``w1`` = (x1 [N, H, W, 8] bf16, weight grad [32*Creal*9], bias grad [32]) with ``pool``: ``x`` is
    the output of a first conv ``x = relu(conv3x3(x1))`` (32 channels, 8-channel padded input of
    which ``Creal`` are real) whose input needs no gradient.  dx -- that conv's output gradient -- is
    then never stored: the kernel accumulates the first conv's weight and bias gradients from it row
    by row, and the function returns None.

    ``bn`` = (z, coef3 fp32 [3*Cout]) (:func:`bn_bwd_coef`): the conv is followed by BatchNorm + ReLU,
    ``g`` is the ReLU-masked gradient of the BN output and the conv-output gradient
    ``dz = coef3[c] g + coef3[C+c] z + coef3[2C+c]`` is formed on load (no dz pass over HBM).
    ``bn_stats``: ``x`` is the ReLU output of a BatchNorm (the dx mask); the kernel also writes that
    BN's backward partial sums (sum dx, sum dx*x per block, as :func:`igemm` ``bn_stats``) and the
    function returns ``(dx, (slab, rows))``.

    ``x2``: dual input -- the conv input is [x | x2] (two [N,H,W,32] tensors of identical layout), as
    :func:`igemm` ``x2``; the kernel's x loader reads both.  ``xbn`` (with ``bn`` and ``bn_stats``):
    ``x`` is the pre-BatchNorm output z of the layer below and the kernel uses relu(z * xbn[c] +
    xbn[CI + c]) as the conv input, dx mask and BN-statistics operand (:func:`igemm` ``xbn``).
    ``sink`` (:class:`SlabSink`): the weight / bias gradient slab rows go there and the sink reduces them
    later (not with ``w1`` or ``head``)."""
    Nx, Hx, Wx, CI, ldx = _nhwc(x, "bwd.x")
    if x2 is not None:
        assert _nhwc(x2, "bwd.x2") == (Nx, Hx, Wx, CI, ldx) and CI == 32, "dual input: two [N,H,W,32]"
        assert head is None and pool is None and w1 is None, "dual input: plain / split / BN modes"
        CI = 64
    if "bwd" in _ABLATE:
        N_, H_, W_ = Nx, Hx, Wx
        if w1 is not None:
            return None
        d1 = dx if dx is not None else torch.empty(N_, H_, W_, split if dx2 is not None else CI, dtype=torch.bfloat16,
                                                   device=x.device)
        return (d1, dx2) if dx2 is not None else d1
    if g is None:                       # pool mode without a skip gradient
        assert pool is not None
        N, H, W, CO, ldg = Nx, Hx, Wx, pool[0].shape[3], 0
    else:
        N, H, W, CO, ldg = _nhwc(g, "bwd.g")
    assert (Nx, Hx, Wx) == (N, H, W), ((N, H, W), tuple(x.shape))
    assert wd.dtype == torch.bfloat16 and wd.numel() >= CI * Kd and Kd >= 9 * CO and Kd % 32 == 0
    assert gw.dtype == torch.float32 and gw.is_contiguous() and gw.numel() == CO * CI * 9
    assert gb is None or (gb.dtype == torch.float32 and gb.numel() == CO)
    bp = ctypes.c_int(0)
    L = _lib.lib()
    pg = L.dpa_bwd_stream_geom(c_int(CI), c_int(CO), ctypes.byref(bp))
    assert pg > 0 and (W % bp.value == 0 or (head is None and pool is None and w1 is None and _strips_ok(W, bp.value))), \
        f"fused backward not available for {CI}->{CO} at W={W}"
    if dx2 is not None:
        assert 0 < split < CI and split % 16 == 0 and not mask
        if dx is None:
            dx = torch.empty(N, H, W, split, dtype=torch.bfloat16, device=x.device)
        _, _, _, C1, ldy = _nhwc(dx, "bwd.dx")
        _, _, _, C2, ldy2 = _nhwc(dx2, "bwd.dx2")
        assert C1 >= split and C2 >= CI - split and tuple(dx2.shape[:3]) == (N, H, W)
        epi = 1
    elif w1 is not None:
        assert pool is not None and mask and dx is None and CI == CO == 32
        ldy, ldy2, epi = 0, 0, 0
    else:
        if dx is None:
            dx = torch.empty(N, H, W, CI, dtype=torch.bfloat16, device=x.device)
        _, _, _, C1, ldy = _nhwc(dx, "bwd.dx")
        assert C1 >= CI
        ldy2, epi = 0, (0 if mask else 2)
    assert dx is None or tuple(dx.shape[:3]) == (N, H, W)
    rh, nblk = _bwd_rows(N, H, W, bp.value, target_blocks)
    if sink is not None:
        assert w1 is None and head is None, "slab sink: plain / split / pool / BN modes"
        slab, bslab = sink.take(nblk * pg, CO, CI, gb is not None)
    else:
        slab = torch.empty(nblk * pg * 9 * CO * CI + (nblk * pg * CO if gb is not None else 0), dtype=torch.float32,
                           device=x.device)
        bslab = slab[nblk * pg * 9 * CO * CI:] if gb is not None else None
    a = BwdArgs(None if g is None else g.data_ptr(), x.data_ptr(), wd.data_ptr(), None if dx is None else dx.data_ptr(),
                None if dx2 is None else dx2.data_ptr(),
                slab.data_ptr(), None if bslab is None else bslab.data_ptr(), ldg, ldx, ldy, ldy2, split, Kd,
                N, H, W, rh, 1, _extent_bytes(1, H, W, CO, ldg) if g is not None else 0,
                _extent_bytes(1, H, W, 32 if x2 is not None else CI, ldx))
    if x2 is not None:
        a.x2 = x2.data_ptr()
    st = _stream(x)
    if pool is not None:
        code, dpool = pool
        assert L.dpa_bwd_stream_pool_ok(c_int(CI), c_int(CO)) and epi == 0 and H % 2 == 0 and head is None
        assert code.dtype == torch.uint8 and code.is_contiguous() and tuple(code.shape) == (N, H // 2, W // 2, CO)
        Np, Hp, Wp, Cp, ldp = _nhwc(dpool, "bwd.dpool")
        assert (Np, Hp, Wp) == (N, H // 2, W // 2) and Cp >= CO
        a.pcode, a.dpool, a.ldp = code.data_ptr(), dpool.data_ptr(), ldp
    slab1 = None
    if w1 is not None:
        x1, gw1, gb1 = w1
        assert x1.dtype == torch.bfloat16 and x1.is_contiguous() and tuple(x1.shape) == (N, H, W, 8)
        creal = gw1.numel() // (CI * 9)
        assert gw1.dtype == torch.float32 and gw1.is_contiguous() and gw1.numel() == CI * creal * 9 and 0 < creal <= 8
        assert gb1.dtype == torch.float32 and gb1.numel() == CI
        slab1 = torch.empty(nblk * (9 * CI * 8 + CI), dtype=torch.float32, device=x.device)   # one row per block
        a.x1, a.slab1, a.bslab1 = x1.data_ptr(), slab1.data_ptr(), slab1[nblk * 9 * CI * 8:].data_ptr()
        a.x1bytes = _extent_bytes(1, H, W, 8, 8)
    hslab = None
    if head is not None:
        tgt, hw, hb, dS, hgw, hgb, hprob = head
        assert epi == 0 and CI == CO == 32, "head mode: the 32->32 last decoder conv"
        assert tgt.dtype == torch.float32 and tgt.is_contiguous() and tgt.numel() == N * H * W
        assert hprob.dtype == torch.float32 and hprob.is_contiguous() and hprob.numel() == N * H * W
        assert hw.dtype == torch.float32 and hw.numel() == CO and hb.numel() == 1
        dS = dS.float().contiguous()
        hw = hw.reshape(-1).contiguous()
        a.tgt, a.hw, a.hb, a.dS = tgt.data_ptr(), hw.data_ptr(), hb.data_ptr(), dS.data_ptr()
        a.hprob = hprob.data_ptr()
        if ybn is not None:
            # head + BN: g is the BN input z; the segmap gradients came from the head statistics pass
            assert bn is not None and bn_stats and bn[0].data_ptr() == g.data_ptr(), "head + BN: g is z, with BN sums"
            assert ybn.dtype == torch.float32 and ybn.is_contiguous() and ybn.numel() == 2 * CO
            a.ybn = ybn.data_ptr()
        else:
            assert hgw.is_contiguous() and hgw.numel() == CO and hgb.numel() == 1
            hslab = torch.empty(nblk * (CO + 1) + CO + 1, dtype=torch.float32, device=x.device)
            a.hslab = hslab.data_ptr()
    bnslab = None
    if bn is not None:
        z, coef3 = bn
        assert (head is None or ybn is not None) and pool is None and w1 is None, "BN mode: plain or head gradient source"
        Nz, Hz, Wz, Cz, ldz = _nhwc(z, "bwd.z")
        assert (Nz, Hz, Wz, Cz) == (N, H, W, CO) and ldz == ldg, "BN mode: z laid out like g"
        assert coef3.dtype == torch.float32 and coef3.is_contiguous() and coef3.numel() == 3 * CO
        a.z, a.bncoef = z.data_ptr(), coef3.data_ptr()
    if bn_stats:
        assert bn is not None and epi == 0, "BN statistics of the layer below: BN mode with the masked dx"
        bnslab = torch.empty(nblk * 2 * CI, dtype=torch.float32, device=x.device)
        a.bnslab = bnslab.data_ptr()
    if xbn is not None:
        assert (bn_stats or (bn is not None and x2 is not None)) and xbn.dtype == torch.float32
        assert xbn.is_contiguous() and xbn.numel() == (64 if x2 is not None else 2 * CI)   # dual: x's only
        a.xbn = xbn.data_ptr()
    _check(L.dpa_bwd_stream(ctypes.byref(a), c_int(CI), c_int(CO), c_int(epi), st), "bwd_stream")
    if hslab is not None:
        _check(L.dpa_head_grad_from_slab(_p(hslab), c_int(nblk), c_int(CO), _p(hslab[nblk * (CO + 1):]), _p(hgw),
                                         _p(hgb), st), "head_grad_from_slab")
    if sink is None:
        _check(L.dpa_wgrad_reduce(_p(slab), _p(bslab), _p(gw), _p(gb), c_int(nblk * pg), c_int(9), c_int(CO), c_int(CI),
                                  c_int(CI), c_int(0), st), "wgrad_reduce(bwd_stream)")
    if slab1 is not None:
        _check(L.dpa_wgrad_reduce(_p(slab1), _p(slab1[nblk * 9 * CI * 8:]), _p(gw1), _p(gb1), c_int(nblk),
                                  c_int(9), c_int(CI), c_int(8), c_int(creal), c_int(0), st), "wgrad_reduce(bwd_stream.w1)")
    out = (dx, dx2) if dx2 is not None else dx
    return (out, (bnslab, nblk)) if bnslab is not None else out


# ------------------------------------------------------------------------------------------ aux
def input_nhwc8(x: torch.Tensor) -> torch.Tensor:
    assert x.dtype == torch.float32 and x.dim() == 4 and x.shape[1] <= 8
    x = x.contiguous()
    B, C, H, W = x.shape
    y = torch.empty(B, H, W, 8, dtype=torch.bfloat16, device=x.device)
    _check(_lib.lib().dpa_input_nhwc8(_p(x), _p(y), c_int(B), c_int(C), c_int(H), c_int(W), _stream(x)), "input_nhwc8")
    return y


def maxpool2(x: torch.Tensor, y: torch.Tensor, code: Optional[torch.Tensor] = None):
    N, H, W, C, ldx = _nhwc(x, "maxpool.x")
    _, Ho, Wo, Cy, ldy = _nhwc(y, "maxpool.y")
    assert (Ho, Wo) == (H // 2, W // 2) and Cy == C and C % 8 == 0
    if code is not None:
        assert code.dtype == torch.uint8 and code.is_contiguous() and tuple(code.shape) == (N, Ho, Wo, C)
    _check(_lib.lib().dpa_maxpool2(_p(x), c_int(ldx), _p(y), c_int(ldy), c_int(N), c_int(H), c_int(W), c_int(C),
                                   _p(code), _stream(x)), "maxpool2")


def pool_bwd_code(code: torch.Tensor, dskip: Optional[torch.Tensor], dpool: torch.Tensor, g: torch.Tensor,
                  y: Optional[torch.Tensor] = None, bn_stats: Optional[list] = None, coef: Optional[torch.Tensor] = None):
    """Max-pool backward + skip-gradient add + ReLU mask from the forward's window codes.  ``y`` + ``bn_stats``
    (an empty list): y (the pooled tensor) is a BatchNorm+ReLU output and the list receives (slab [blocks][2][C],
    blocks) of sum g, sum g*y -- the BN backward's partial sums (:func:`bn_bwd` ``stats``).  ``coef`` (fp32
    [scale C | shift C]): ``y`` is that BN's input z and relu(bn(z)) is formed on load (z is dense where the
    skip y may be a concat half)."""
    N, H, W, C, ldg = _nhwc(g, "pool_bwd_code.g")
    assert code.dtype == torch.uint8 and tuple(code.shape) == (N, H // 2, W // 2, C) and code.is_contiguous()
    ldd = 8
    if dskip is not None:
        Nd, Hd, Wd, Cd, ldd = _nhwc(dskip, "pool_bwd_code.dskip")
        assert (Nd, Hd, Wd, Cd) == (N, H, W, C)
    Np, Hp, Wp, Cp, ldp = _nhwc(dpool, "pool_bwd_code.dpool")
    assert (Np, Hp, Wp, Cp) == (N, H // 2, W // 2, C)
    L = _lib.lib()
    ldy, bnslab = 0, None
    if bn_stats is not None and y is not None:
        Ny, Hy, Wy, Cy, ldy = _nhwc(y, "pool_bwd_code.y")
        assert (Ny, Hy, Wy, Cy) == (N, H, W, C)
        rows = L.dpa_pool_bwd_code_blocks(c_int(N), c_int(H), c_int(W), c_int(C))
        bnslab = torch.empty(rows * 2 * C, dtype=torch.float32, device=g.device)
        if coef is not None:
            assert coef.dtype == torch.float32 and coef.is_contiguous() and coef.numel() == 2 * C
    else:
        coef = None
    _check(L.dpa_pool_bwd_code(_p(code), _p(dskip), c_int(ldd), _p(dpool), c_int(ldp), _p(g), c_int(ldg),
                               c_int(N), c_int(H), c_int(W), c_int(C), _p(y if bnslab is not None else None), c_int(ldy),
                               _p(bnslab), _p(coef), _stream(g)), "pool_bwd_code")
    if bnslab is not None:
        bn_stats.extend([bnslab, rows])


def pool_bwd(skip: torch.Tensor, dskip: Optional[torch.Tensor], dpool: torch.Tensor, g: torch.Tensor):
    N, H, W, C, lds = _nhwc(skip, "pool_bwd.skip")
    ldd = 8
    if dskip is not None:
        Nd, Hd, Wd, Cd, ldd = _nhwc(dskip, "pool_bwd.dskip")
        assert (Nd, Hd, Wd, Cd) == (N, H, W, C)
    Np, Hp, Wp, Cp, ldp = _nhwc(dpool, "pool_bwd.dpool")
    assert (Np, Hp, Wp, Cp) == (N, H // 2, W // 2, C)
    _, Hg, Wg, Cg, ldg = _nhwc(g, "pool_bwd.g")
    assert (Hg, Wg, Cg) == (H, W, C)
    _check(_lib.lib().dpa_pool_bwd(_p(skip), c_int(lds), _p(dskip), c_int(ldd), _p(dpool), c_int(ldp), _p(g), c_int(ldg),
                                   c_int(N), c_int(H), c_int(W), c_int(C), _stream(skip)), "pool_bwd")


def pack_weights(packed: torch.Tensor, descs_dev: torch.Tensor, ndesc: int, max_elems: int):
    """Batched fp32 -> bf16 GEMM-layout packing; each descriptor holds its weight's device address."""
    assert packed.dtype == torch.bfloat16
    _check(_lib.lib().dpa_pack_weights(None, _p(packed), _p(descs_dev), c_int(ndesc), c_ll(max_elems),
                                       _stream(packed)), "pack_weights")


def head_fwd(y: torch.Tensor, w: torch.Tensor, b: torch.Tensor, t: Optional[torch.Tensor], want_probs: bool = False,
             coef: Optional[torch.Tensor] = None):
    """-> (S[4] fp32 or None, probs[N,H,W] fp32 or None).  ``coef`` ([scale C | shift C] fp32, bn_fwd's
    ``coef_out``): ``y`` is the pre-BN output z of a BatchNorm+ReLU layer and relu(bn(z)) is formed on load."""
    N, H, W, C, ldy = _nhwc(y, "head.y")
    if coef is not None:
        assert C in (32, 64) and coef.dtype == torch.float32 and coef.is_contiguous() and coef.numel() == 2 * C
    P = N * H * W
    L = _lib.lib()
    nblk = L.dpa_head_slab_blocks(c_ll(P))
    S = slab = None
    if t is not None:
        assert t.dtype == torch.float32 and t.is_contiguous() and t.numel() == P
        slab = torch.empty(nblk * 4 + 4, dtype=torch.float32, device=y.device)
        S = slab[nblk * 4:]
    probs = torch.empty(N, H, W, dtype=torch.float32, device=y.device) if want_probs else None
    wf = w.reshape(-1).contiguous()
    _check(L.dpa_head_fwd(_p(y), c_int(ldy), c_int(C), _p(wf), _p(b), _p(t), _p(slab), _p(S), _p(probs), c_ll(P),
                          _p(coef), _stream(y)), "head_fwd")
    return S, probs


def head_bwd(y: torch.Tensor, w: torch.Tensor, b: torch.Tensor, t: torch.Tensor, dS: torch.Tensor,
             gw: torch.Tensor, gb: torch.Tensor, bn_stats: Optional[list] = None,
             coef: Optional[torch.Tensor] = None, store: bool = True) -> Optional[torch.Tensor]:
    """Segmentation-head backward: returns gy = dL/dy (ReLU-masked by y).  ``bn_stats`` (an empty list):
    y is a BatchNorm+ReLU output and the list receives (slab [blocks][2][C], blocks) of sum gy, sum gy*y,
    the BN backward's partial sums (:func:`bn_bwd` ``stats``) -- no statistics pass over (gy, z).
    ``coef`` (with ``bn_stats``): ``y`` is that BN's input z, y = relu(bn(z)) formed on load (:func:`head_fwd`).
    ``store`` False (with ``bn_stats``): only the segmap gradients and the BN partial sums, returns None (the
    fused conv backward's head + BN mode forms gy itself, :func:`conv_bwd_fused` ``ybn``)."""
    N, H, W, C, ldy = _nhwc(y, "head_bwd.y")
    if coef is not None:
        assert bn_stats is not None and C in (32, 64) and coef.dtype == torch.float32 and coef.numel() == 2 * C
    P = N * H * W
    L = _lib.lib()
    nblk = L.dpa_head_slab_blocks(c_ll(P))
    assert store or bn_stats is not None
    gy = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=y.device) if store else None
    want = bn_stats is not None and C in (32, 64)
    slab = torch.empty(nblk * (C + 1) + C + 1 + (nblk * 2 * C if want else 0), dtype=torch.float32, device=y.device)
    tmp = slab[nblk * (C + 1):nblk * (C + 1) + C + 1]
    bnslab = slab[nblk * (C + 1) + C + 1:] if want else None
    dS = dS.float().contiguous()
    assert gw.is_contiguous() and gw.numel() == C and gb.numel() == 1
    _check(L.dpa_head_bwd(_p(y), c_int(ldy), c_int(C), _p(w.reshape(-1).contiguous()), _p(b), _p(t), _p(dS), _p(gy),
                          c_int(C), _p(slab), _p(tmp), _p(gw), _p(gb), c_ll(P), _p(bnslab), _p(coef), _stream(y)),
           "head_bwd")
    if want:
        bn_stats.extend([bnslab, nblk])
    return gy


# ------------------------------------------------------------------------------------- fused deconv bwd
USE_FUSED_DECONV = CFG.fused_deconv
DECONV_BWD_SHAPES = ((64, 32), (128, 64))


def deconv_bwd_fused(gup: torch.Tensor, x: torch.Tensor, wd: torch.Tensor, gw: torch.Tensor,
                     gb: Optional[torch.Tensor], bn_stats: Optional[list] = None,
                     xbn: Optional[torch.Tensor] = None) -> torch.Tensor:
    """ConvTranspose2d(k2, s2) dgrad (ReLU-masked by x) AND weight/bias gradient in one pass over
    (gup, x) (csrc/deconv.hip); gw [Cin*Cout*4] / gb [Cout] accumulate.  Returns dx [N,h,w,Cin].
    ``bn_stats`` (an empty list): x is a BatchNorm+ReLU output; the list receives (slab [rows][2][Cin],
    rows) of sum dx, sum dx*x -- that BN's backward partial sums (:func:`bn_bwd` ``stats``).
    ``xbn`` (with ``bn_stats``; fp32 [scale Cin | shift Cin]): ``x`` is that BN's input z, relu(bn(z)) on load."""
    if xbn is not None:
        assert bn_stats is not None and xbn.dtype == torch.float32 and xbn.is_contiguous()
    N, H2, W2, Cout, ldg = _nhwc(gup, "deconv_bwd.g")
    Nx, h, w, Cin, ldx = _nhwc(x, "deconv_bwd.x")
    assert Nx == N and (H2, W2) == (2 * h, 2 * w) and (Cin, Cout) in DECONV_BWD_SHAPES
    assert wd.dtype == torch.bfloat16 and wd.numel() >= Cin * 4 * Cout
    assert gw.dtype == torch.float32 and gw.is_contiguous() and gw.numel() == Cin * Cout * 4
    dx = torch.empty(N, h, w, Cin, dtype=torch.bfloat16, device=x.device)
    if "deconv" in _ABLATE:
        return dx
    L = _lib.lib()
    st = _stream(x)
    bn_parts = []
    for n0, n1 in _image_chunks(N, max(H2 * W2 * ldg, h * w * ldx) * 2):
        nb = n1 - n0
        ntiles = -(-nb * h * w // 64)
        splits = min(ntiles, 512 if Cin == 64 else 256)
        tpb = -(-ntiles // splits)
        splits = -(-ntiles // tpb)
        bnn = splits * 2 * Cin if bn_stats is not None else 0
        slab = torch.empty(splits * 4 * Cout * Cin + splits * Cout + bnn, dtype=torch.float32, device=x.device)
        bslab = slab[splits * 4 * Cout * Cin:splits * 4 * Cout * Cin + splits * Cout] if gb is not None else None
        bnslab = slab[splits * 4 * Cout * Cin + splits * Cout:] if bnn else None
        if bnslab is not None:
            bn_parts.append((bnslab, splits))
        _check(L.dpa_deconv_bwd(_p(gup[n0:n1]), c_int(ldg), _p(x[n0:n1]), c_int(ldx), _p(wd), _p(dx[n0:n1]), c_int(Cin),
                                _p(slab), _p(bslab), c_int(nb), c_int(h), c_int(w), c_int(Cin), c_int(Cout),
                                c_int(splits), ctypes.c_uint(_extent_bytes(nb, H2, W2, Cout, ldg)),
                                ctypes.c_uint(_extent_bytes(nb, h, w, Cin, ldx)), _p(bnslab), _p(xbn), st), "deconv_bwd")
        _check(L.dpa_wgrad_reduce(_p(slab), _p(bslab), _p(gw), _p(gb), c_int(splits), c_int(4), c_int(Cout), c_int(Cin),
                                  c_int(Cin), c_int(1), st), "wgrad_reduce")
    if bn_parts:
        rows = sum(r for _, r in bn_parts)
        bn_stats.extend([bn_parts[0][0] if len(bn_parts) == 1 else torch.cat([t for t, _ in bn_parts]), rows])
    return dx


def deconv_fwd_fused(x: torch.Tensor, wf: torch.Tensor, bias: Optional[torch.Tensor], y: torch.Tensor,
                     xbn: Optional[torch.Tensor] = None):
    """ConvTranspose2d(k2, s2) forward of the full-resolution up-convs (csrc/deconv.hip) into ``y``
    (the decoder concat buffer's second half), whole-chunk stores along each output row.  ``xbn`` (fp32
    [scale Cin | shift Cin]): ``x`` is the pre-BN output z of a BatchNorm+ReLU layer, read as relu(bn(z))."""
    N, h, w, Cin, ldx = _nhwc(x, "deconv_fwd.x")
    if xbn is not None:
        assert xbn.dtype == torch.float32 and xbn.is_contiguous() and xbn.numel() == 2 * Cin
    Ny, H2, W2, Cy, ldy = _nhwc(y, "deconv_fwd.y")
    Cout = Cy
    assert Ny == N and (H2, W2) == (2 * h, 2 * w) and (Cin, Cout) in DECONV_BWD_SHAPES
    assert wf.dtype == torch.bfloat16 and wf.numel() >= 4 * Cout * Cin
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.numel() == Cout
    if "deconv" in _ABLATE:
        return
    L = _lib.lib()
    st = _stream(x)
    for n0, n1 in _image_chunks(N, max(H2 * W2 * ldy, h * w * ldx) * 2):
        nb = n1 - n0
        _check(L.dpa_deconv_fwd(_p(x[n0:n1]), c_int(ldx), _p(wf), _p(bias), _p(y[n0:n1]), c_int(ldy), c_int(nb), c_int(h),
                                c_int(w), c_int(Cin), c_int(Cout), c_int(1024 if Cin == 64 else 512),
                                ctypes.c_uint(_extent_bytes(nb, h, w, Cin, ldx)), _p(xbn), st), "deconv_fwd")


# ------------------------------------------------------------------------------------- BN / bilinear
def _flat_f32(t: torch.Tensor, n: int, name: str):
    assert t.dtype == torch.float32 and t.is_contiguous() and t.numel() == n and t.is_cuda, f"{name}: need fp32[{n}]"
    return t


def _fold_slab(slab: torch.Tensor, rows: int, K: int, max_rows: int = 512):
    """(slab [rows][K], rows) -> at most ``max_rows`` rows (parallel fixed-order partial sums)."""
    assert slab.numel() >= rows * K
    if rows <= max_rows:
        return slab, rows
    out = torch.empty(max_rows * K, dtype=torch.float32, device=slab.device)
    R = -(-rows // max_rows)
    nout = -(-rows // R)
    _check(_lib.lib().dpa_slab_fold(_p(slab), c_int(rows), c_int(K), c_int(max_rows), _p(out), _stream(slab)),
           "slab_fold")
    return out, nout


def bn_fwd(z: torch.Tensor, y: Optional[torch.Tensor], bn: torch.nn.BatchNorm2d, train: bool, relu: bool = True,
           stats: Optional[list] = None, pool: Optional[torch.Tensor] = None, pcode: Optional[torch.Tensor] = None,
           coef_out: Optional[list] = None):
    """y = relu(BatchNorm2d(z)) (NHWC bf16; y may be a concat half).  Training: batch statistics,
    running stats updated (torch momentum semantics); returns ``saved`` = [mean, invstd] (fp32 [2C])
    for :func:`bn_bwd`.  Eval: running statistics, returns None.  ``stats`` = (slab, rows) partial
    sums the producing conv already computed (:func:`igemm` ``bn_stats``): no statistics pass.
    ``pool``/``pcode``: also the 2x2 max-pool of y and its window codes, in the same pass (even H, W;
    otherwise a separate :func:`maxpool2`).  ``y=None`` (with ``coef_out``, an empty list): no
    normalise pass at all -- the statistics and running stats update as usual and ``coef_out``
    receives the fp32 [2C] (scale, shift) with which a consumer forms relu(z * scale + shift) on load
    (:func:`igemm` / :func:`conv_bwd_fused` ``xbn``)."""
    N, H, W, C, ldz = _nhwc(z, "bn.z")
    if y is None:
        # coefficients only, or (pool) only the pooled tensor + codes: the consumers of y read z on load
        assert coef_out is not None and relu and (pool is None or (pcode is not None and H % 2 == 0 and W % 2 == 0)), \
            "no y: the consumer applies BN + ReLU"
        ldy = 0
    else:
        Ny, Hy, Wy, Cy, ldy = _nhwc(y, "bn.y")
        assert (Ny, Hy, Wy, Cy) == (N, H, W, C)
    assert bn.num_features == C and bn.affine
    P = N * H * W
    L = _lib.lib()
    rows = L.dpa_bn_slab_rows(c_ll(P), c_int(C))
    assert rows > 0, f"bn: unsupported shape P={P} C={C}"
    gamma, beta = _flat_f32(bn.weight, C, "bn.weight"), _flat_f32(bn.bias, C, "bn.bias")
    track = bn.track_running_stats and bn.running_mean is not None
    use_batch = train or not track
    scratch = torch.empty(rows * 2 * C + 4 * C, dtype=torch.float32, device=z.device)
    slab, coef, saved = scratch[:rows * 2 * C], scratch[rows * 2 * C:rows * 2 * C + 2 * C], scratch[rows * 2 * C + 2 * C:]
    rm = rv = None
    if track:
        rm, rv = _flat_f32(bn.running_mean, C, "bn.running_mean"), _flat_f32(bn.running_var, C, "bn.running_var")
        if train and bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
    if bn.momentum is not None:
        mom = bn.momentum
    else:   # cumulative moving average (torch: momentum = 1 / num_batches_tracked)
        mom = 1.0 / max(1, int(bn.num_batches_tracked.item())) if track else 0.0
    # running stats: updated when training, read in eval (use_batch False), untouched otherwise
    pre_rows = 0
    if stats and use_batch:
        slab, pre_rows = _fold_slab(*stats, 2 * C)
    fuse_pool = pool is not None and H % 2 == 0 and W % 2 == 0
    ldp = 0
    if fuse_pool:
        Np, Hp, Wp, Cp, ldp = _nhwc(pool, "bn.pool")
        assert (Np, Hp, Wp, Cp) == (N, H // 2, W // 2, C)
        if pcode is not None:
            assert pcode.dtype == torch.uint8 and pcode.is_contiguous() and tuple(pcode.shape) == (N, H // 2, W // 2, C)
    if coef_out is not None:
        coef_out.append(coef)
    _check(L.dpa_bn_fwd(_p(z), c_int(ldz), _p(y), c_int(ldy), c_ll(P), c_int(C), _p(gamma), _p(beta),
                        ctypes.c_float(bn.eps), ctypes.c_float(mom), _p(rm), _p(rv), _p(slab) if use_batch else None,
                        _p(coef), _p(saved), c_int(int(use_batch)), c_int(int(relu)), c_int(pre_rows),
                        _p(pool) if fuse_pool else None, c_int(ldp), _p(pcode) if fuse_pool else None,
                        c_int(N), c_int(H), c_int(W), _stream(z)), "bn_fwd")
    if pool is not None and not fuse_pool:
        maxpool2(y, pool, pcode)
    return saved if use_batch else None


def bn_bwd(g: torch.Tensor, z: torch.Tensor, saved: torch.Tensor, bn: torch.nn.BatchNorm2d,
           dgamma: Optional[torch.Tensor], dbeta: Optional[torch.Tensor], stats: Optional[list] = None) -> torch.Tensor:
    """dz from g = dL/d(BN output) (ReLU mask already applied); dgamma/dbeta += (fp32 [C]).
    ``stats`` = (slab, rows) of (sum g, sum g*y) from the dgrad that produced g (:func:`igemm`
    ``bn_stats`` with the BN output as mask): no reduction pass over (g, z)."""
    N, H, W, C, ldg = _nhwc(g, "bn_bwd.g")
    Nz, Hz, Wz, Cz, ldz = _nhwc(z, "bn_bwd.z")
    assert (Nz, Hz, Wz, Cz) == (N, H, W, C) and saved.numel() == 2 * C
    P = N * H * W
    L = _lib.lib()
    rows = L.dpa_bn_slab_rows(c_ll(P), c_int(C))
    dz = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=g.device)
    scratch = torch.empty(rows * 2 * C + 3 * C, dtype=torch.float32, device=g.device)
    if dgamma is not None:
        _flat_f32(dgamma, C, "bn.dgamma")
    if dbeta is not None:
        _flat_f32(dbeta, C, "bn.dbeta")
    slab, pre_rows = scratch[:rows * 2 * C], 0
    if stats:
        slab, pre_rows = _fold_slab(*stats, 2 * C)
    _check(L.dpa_bn_bwd(_p(g), c_int(ldg), _p(z), c_int(ldz), _p(dz), c_int(C), c_ll(P), c_int(C),
                        _p(_flat_f32(bn.weight, C, "bn.weight")), _p(saved), _p(slab),
                        _p(scratch[rows * 2 * C:]), _p(dgamma), _p(dbeta), _p(_flat_f32(bn.bias, C, "bn.bias")),
                        c_int(pre_rows), _stream(g)), "bn_bwd")
    return dz


def bn_bwd_coef(g: torch.Tensor, z: torch.Tensor, saved: torch.Tensor, bn: torch.nn.BatchNorm2d,
                dgamma: Optional[torch.Tensor], dbeta: Optional[torch.Tensor], stats: Optional[list] = None) -> torch.Tensor:
    """:func:`bn_bwd` without its elementwise pass: returns coef3 (fp32 [3C]) with
    ``dz = coef3[c] g + coef3[C+c] z + coef3[2C+c]`` for a consumer that forms dz on load
    (:func:`conv_bwd_fused` ``bn``); dgamma/dbeta accumulate as in :func:`bn_bwd`."""
    N, H, W, C, ldg = _nhwc(g, "bn_coef.g")
    Nz, Hz, Wz, Cz, ldz = _nhwc(z, "bn_coef.z")
    assert (Nz, Hz, Wz, Cz) == (N, H, W, C) and saved.numel() == 2 * C
    P = N * H * W
    L = _lib.lib()
    rows = L.dpa_bn_slab_rows(c_ll(P), c_int(C))
    scratch = torch.empty(rows * 2 * C + 3 * C, dtype=torch.float32, device=g.device)
    if dgamma is not None:
        _flat_f32(dgamma, C, "bn.dgamma")
    if dbeta is not None:
        _flat_f32(dbeta, C, "bn.dbeta")
    slab, pre_rows = scratch[:rows * 2 * C], 0
    if stats:
        slab, pre_rows = _fold_slab(*stats, 2 * C)
    coef3 = scratch[rows * 2 * C:]
    _check(L.dpa_bn_bwd_coef(_p(g), c_int(ldg), _p(z), c_int(ldz), c_ll(P), c_int(C),
                             _p(_flat_f32(bn.weight, C, "bn.weight")), _p(saved), _p(slab), _p(coef3), _p(dgamma),
                             _p(dbeta), _p(_flat_f32(bn.bias, C, "bn.bias")), c_int(pre_rows), _stream(g)), "bn_bwd_coef")
    return coef3


def up2_fwd(x: torch.Tensor, y: torch.Tensor):
    """Bilinear x2 up-sampling (align_corners=False) of NHWC x into y (may be a concat half)."""
    N, h, w, C, ldx = _nhwc(x, "up2.x")
    Ny, Hy, Wy, Cy, ldy = _nhwc(y, "up2.y")
    assert (Ny, Hy, Wy, Cy) == (N, 2 * h, 2 * w, C)
    _check(_lib.lib().dpa_up2_fwd(_p(x), c_int(ldx), _p(y), c_int(ldy), c_int(N), c_int(h), c_int(w), c_int(C),
                                  _stream(x)), "up2_fwd")


def up2_bwd(g: torch.Tensor) -> torch.Tensor:
    N, H, W, C, ldg = _nhwc(g, "up2_bwd.g")
    assert H % 2 == 0 and W % 2 == 0
    dx = torch.empty(N, H // 2, W // 2, C, dtype=torch.bfloat16, device=g.device)
    _check(_lib.lib().dpa_up2_bwd(_p(g), c_int(ldg), _p(dx), c_int(C), c_int(N), c_int(H // 2), c_int(W // 2), c_int(C),
                                  _stream(g)), "up2_bwd")
    return dx


# ------------------------------------------------------------------------------------- loss tail
class _LossFromPartials(torch.autograd.Function):
    """loss = S0/n - log(2 S1 / (S2 + S3 + eps)) in one launch forward and one backward."""

    @staticmethod
    def forward(ctx, S, n: int, dice: bool):
        assert S.dtype == torch.float32 and S.is_contiguous() and S.numel() == 4
        out = torch.empty(5, dtype=torch.float32, device=S.device)
        L = _lib.lib()
        _check(L.dpa_loss_finish(_p(S), ctypes.c_float(1.0 / n), c_int(int(dice)), _p(out), _stream(S)), "loss_finish")
        ctx.save_for_backward(out)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        (out,) = ctx.saved_tensors
        g = g.float().contiguous()
        dS = torch.empty(4, dtype=torch.float32, device=out.device)
        L = _lib.lib()
        _check(L.dpa_loss_grad(_p(g), _p(out[1:]), ctypes.c_float(1.0), _p(dS), _stream(out)), "loss_grad")
        return dS, None, None


def loss_from_partials(S: torch.Tensor, n: int, dice: bool = True) -> torch.Tensor:
    return _LossFromPartials.apply(S.contiguous(), n, dice)


def zero_(t: torch.Tensor) -> torch.Tensor:
    """In-place zero of a dense device tensor by hipMemsetAsync on the current stream (no compute kernel)."""
    assert t.is_cuda and t.is_contiguous()
    _check(_lib.lib().dpa_zero(_p(t), c_ll(t.numel() * t.element_size()), _stream(t)), "zero")
    return t


_SEEDS = {}


def backward_scaled(loss: torch.Tensor, scale: float) -> None:
    """``(loss * scale).backward()`` without the two elementwise launches: the backward is seeded with a
    cached device scalar (one per device and scale value), which the loss op's HIP backward consumes."""
    key = (loss.device, float(scale))
    seed = _SEEDS.get(key)
    if seed is None:
        seed = _SEEDS[key] = torch.full((), float(scale), dtype=loss.dtype, device=loss.device)
    torch.autograd.backward(loss, seed)


def comm_probe(src: torch.Tensor, dst: torch.Tensor, stamp: torch.Tensor, blocks: int = 32):
    """RCCL-bucket stand-in (csrc/unet_aux.hip ``comm_probe_kernel``): ``blocks`` workgroups copy ``src``
    into ``dst`` (16-B aligned, same byte size) on the CURRENT stream; ``stamp`` (int64, >= 2 * blocks) gets
    each workgroup's start / end on the GPU's constant 100 MHz clock."""
    nb = src.numel() * src.element_size()
    assert nb % 16 == 0 and dst.numel() * dst.element_size() == nb and stamp.numel() >= 2 * blocks
    assert stamp.dtype == torch.int64 and src.is_cuda and dst.is_cuda and stamp.is_cuda
    _check(_lib.lib().dpa_comm_probe(_p(src), _p(dst), c_ll(nb // 16), c_int(blocks), _p(stamp),
                                     c_void_p(torch.cuda.current_stream(src.device).cuda_stream)), "comm_probe")


def cu_masked_stream(device, reserve: int) -> torch.cuda.ExternalStream:
    """A HIP stream of ``device`` whose kernels may use every CU but ``reserve`` (spread over the CU index
    range): compute on it always leaves CUs free for another stream's kernels (an RCCL bucket's).  Returns a
    torch ExternalStream (the stream lives for the process)."""
    dev = torch.device(device)
    L = _lib.lib()
    L.dpa_stream_create_cumask.restype = c_int
    out = c_void_p()
    kept = L.dpa_stream_create_cumask(c_int(dev.index or 0), c_int(int(reserve)), ctypes.byref(out))
    if kept < 0 or out.value is None:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({kept})")
    s = torch.cuda.ExternalStream(out.value, device=dev)
    s.cus = kept
    return s
