"""Python wrappers of the fp32 kernel family (csrc/fp32.hip): the hand-written fp32 training path.

Every wrapper checks the tensor contracts (dtype, NHWC strides, 16-B alignment) before it builds an
argument block, and launches on the current stream of the output's device.  Weights are packed into
their GEMM layouts by ONE batched kernel per parameter update (:func:`pack_weights`, the bf16 engine's
descriptor table with fp32 output); the ``pack_*`` torch forms below are the reference layouts the
tests compare it with.  Weight / bias gradients are reduced straight into the flat fp32 gradient buffer.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from . import _lib
from . import config as _config

c_int, c_ll, c_void_p = ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p
_MAX = 2 ** 31 - 1024          # per-launch element-offset range the host keeps (int pixel math)


class F32ConvArgs(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("w", c_void_p), ("bias", c_void_p), ("y", c_void_p), ("mask", c_void_p)] + \
               [(n, c_int) for n in ("ldx", "ldy", "ldm", "mask_ch", "N", "Ho", "Wo", "Hs", "Ws", "Cs", "KH", "KW",
                                     "stride", "pad", "Ngemm", "Kpad", "mode", "relu", "accumulate", "Cout", "wide", "halo")]


USE_WGRAD_HALO = _config.KernelConfig.from_env().f32_wgrad_halo   # 3x3 weight gradients with the input halo staged
USE_WGRAD_BIG = _config.KernelConfig.from_env().f32_wgrad_big     # 256 x 256 8-wave weight-gradient tiles (deep layers)
IGEMM_WIDE = _config.KernelConfig.from_env().f32_igemm_wide      # 256-pixel 8-wave conv / dgrad tiles for GEMM-N % 128 == 0
WGRAD_PX = _config.KernelConfig.from_env().f32_wgrad_px          # pixel-major LDS weight-gradient operands
WGRAD3_HALVES = _config.KernelConfig.from_env().f32_wgrad3_halves  # 64-input-channel halo weight gradients as 2 x 32
WGRAD_C4 = _config.KernelConfig.from_env().f32_wgrad_c4          # first layer's weight gradient: 4-channel form
CONV_HALO = _config.KernelConfig.from_env().f32_conv_halo         # 3x3 convs with GEMM-N 32 (1) / also 64 (2): halo-staged


def wgrad_f32_tile(M: int, Ncols: int, big: bool):
    """(rows, columns) of the weight-gradient block tile (csrc/fp32.hip wgrad_f32_bm).  The 256 x 256 tile
    pays for 256 output channels over >= 256 input channels (b16, 512^2: enc3.c2 / dec0.c1 / dec0.c2
    +5-9 %); with 512 outputs at 32^2 or 128 inputs its grid is too small (-3..-16 %,
    profiles/f32_kbench_b16_512_r05.txt)."""
    if big and M == 256 and Ncols >= 9 * 256:
        return 256, 256
    return (128 if M % 128 == 0 else 64 if M % 64 == 0 else 32), 128


class F32WgradArgs(ctypes.Structure):
    _fields_ = [("A", c_void_p), ("B", c_void_p), ("slab", c_void_p), ("bslab", c_void_p)] + \
               [(n, c_int) for n in ("lda", "ldb", "N", "Hg", "Wg", "HB", "WB", "M", "Nc", "s", "pad", "KH", "KW")] + \
               [("pix_per_split", ctypes.c_long), ("splits", c_int), ("halo", c_int), ("big", c_int), ("px", c_int)]


def _st(t: torch.Tensor):
    return c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _p(t: Optional[torch.Tensor]):
    return None if t is None else c_void_p(t.data_ptr())


def _check(err, name):
    _lib.check(int(err), name)


def nhwc(t: torch.Tensor, name: str) -> Tuple[int, int, int, int, int]:
    """(N, H, W, C, ld) of an NHWC fp32 tensor (channel slice allowed: ld = W stride)."""
    assert t.dtype == torch.float32 and t.dim() == 4 and t.is_cuda, f"{name}: need cuda fp32 NHWC, got {t.dtype} {tuple(t.shape)}"
    N, H, W, C = t.shape
    sN, sH, sW, sC = t.stride()
    assert sC == 1 and sH == W * sW and (N == 1 or sN == H * sH), f"{name}: unsupported strides {t.stride()}"
    assert sW % 4 == 0 and t.data_ptr() % 16 == 0, f"{name}: ld {sW} / pointer not 16-byte aligned"
    return N, H, W, C, sW


def nhwc_ok(t: torch.Tensor) -> bool:
    """True when :func:`nhwc` accepts ``t`` (dense or channel-sliced NHWC, 16-byte aligned)."""
    try:
        nhwc(t, "")
        return True
    except AssertionError:
        return False


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


# ---------------------------------------------------------------------------------------- packing
def pack_conv_fwd(w: torch.Tensor, cs: int) -> Tuple[torch.Tensor, int]:
    """Conv2d weight [Cout, Cin, 3, 3] -> [Cout][Kpad], k = tap * cs + ci (input channels padded to cs)."""
    co, ci, kh, kw = w.shape
    wp = torch.zeros(co, kh * kw, cs, dtype=torch.float32, device=w.device)
    wp[:, :, :ci] = w.detach().permute(0, 2, 3, 1).reshape(co, kh * kw, ci)
    kpad = round_up(kh * kw * cs, 16)
    out = torch.zeros(co, kpad, dtype=torch.float32, device=w.device)
    out[:, :kh * kw * cs] = wp.reshape(co, -1)
    return out.contiguous(), kpad


def pack_conv_dgrad(w: torch.Tensor) -> Tuple[torch.Tensor, int]:
    """dx = conv3x3(g, flipped W^T): [Cin][Kpad], k = tap * Cout + co, tap of the flipped kernel."""
    co, ci, kh, kw = w.shape
    wd = w.detach().flip(2, 3).permute(1, 2, 3, 0).reshape(ci, kh * kw * co)
    kpad = round_up(kh * kw * co, 16)
    out = torch.zeros(ci, kpad, dtype=torch.float32, device=w.device)
    out[:, :kh * kw * co] = wd
    return out.contiguous(), kpad


def pack_deconv_fwd(w: torch.Tensor) -> torch.Tensor:
    """ConvTranspose2d weight [Cin, Cout, 2, 2] -> [4 Cout][Cin], row (2i + j) Cout + co."""
    ci, co = w.shape[:2]
    return w.detach().permute(2, 3, 1, 0).reshape(4 * co, ci).contiguous()


def pack_deconv_dgrad(w: torch.Tensor) -> torch.Tensor:
    """dx[h][w][ci] = sum_{i,j,co} g[2h+i][2w+j][co] W[ci][co][i][j]: [Cin][4 Cout], k = (2i + j) Cout + co."""
    ci, co = w.shape[:2]
    return w.detach().permute(0, 2, 3, 1).reshape(ci, 4 * co).contiguous()


# ---------------------------------------------------------------------------------------- GEMMs
def igemm(x: torch.Tensor, wp: torch.Tensor, y: torch.Tensor, *, Ngemm: int, Kpad: int, KH: int, KW: int,
          stride: int, pad: int, Cs: int, out_grid, bias: Optional[torch.Tensor] = None, relu: bool = False,
          mask: Optional[torch.Tensor] = None, mask_ch: int = 0, mode: int = 0, Cout: int = 0,
          accumulate: bool = False) -> torch.Tensor:
    """fp32 implicit GEMM (see csrc/fp32.hip igemm_f32_kernel); ``out_grid`` = (N, Ho, Wo) of GEMM-M."""
    N, Hs, Ws, Cx, ldx = nhwc(x, "igemm_f32.x")
    _, _, _, Cy, ldy = nhwc(y, "igemm_f32.y")
    No, Ho, Wo = out_grid
    assert No == N and Cs <= Cx and Cs % 4 == 0 and Kpad % 16 == 0 and Kpad >= KH * KW * Cs and Ngemm % 32 == 0
    assert wp.dtype == torch.float32 and wp.is_contiguous() and wp.numel() >= Ngemm * Kpad
    if mode == 0:
        assert tuple(y.shape[:3]) == (N, Ho, Wo) and Cy >= Ngemm
    else:
        assert tuple(y.shape[:3]) == (N, 2 * Ho, 2 * Wo) and Cy >= Cout and Ngemm == 4 * Cout and Cout % 4 == 0
    assert (Ho - 1) * stride + KH - 1 - pad <= Hs - 1 + pad and (Wo - 1) * stride + KW - 1 - pad <= Ws - 1 + pad
    ldm = 0
    if mask is not None:
        Nm, Hm, Wm, Cm, ldm = nhwc(mask, "igemm_f32.mask")
        assert (Nm, Hm, Wm) == (N, Ho, Wo) and mode == 0
        mask_ch = mask_ch or min(Cm, Ngemm)
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous() and bias.numel() >= (Cout or Ngemm)
    L = _lib.lib()
    st = _st(y)
    per_img = max(Hs * Ws * ldx, (4 if mode else 1) * Ho * Wo * ldy)
    step = max(1, _MAX // max(per_img, 1))
    for n0 in range(0, N, step):
        n1 = min(N, n0 + step)
        a = F32ConvArgs(x[n0:n1].data_ptr(), wp.data_ptr(), None if bias is None else bias.data_ptr(), y[n0:n1].data_ptr(),
                        None if mask is None else mask[n0:n1].data_ptr(), ldx, ldy, ldm, mask_ch, n1 - n0, Ho, Wo, Hs, Ws,
                        Cs, KH, KW, stride, pad, Ngemm, Kpad, mode, int(relu), int(accumulate), Cout, int(IGEMM_WIDE),
                        CONV_HALO)
        _check(L.dpa_igemm_f32(ctypes.byref(a), st), "igemm_f32")
    return y


def pack_weights(packed: torch.Tensor, descs_dev: torch.Tensor, ndesc: int, max_elems: int) -> None:
    """Every layer's GEMM weight layouts in one launch (csrc/unet_aux.hip pack_kernel<float>; descriptors
    as ``ops.kernels.PackDesc``: mode 0 conv fwd, 1 conv dgrad, 2 / 3 transposed conv fwd / dgrad)."""
    assert packed.dtype == torch.float32 and packed.is_contiguous()
    _check(_lib.lib().dpa_pack_weights_f32(_p(packed), _p(descs_dev), c_int(ndesc), c_ll(max_elems), _st(packed)),
           "pack_weights_f32")


def wgrad(A: torch.Tensor, B: torch.Tensor, gw: torch.Tensor, gb: Optional[torch.Tensor], *, KH: int, KW: int, s: int,
          pad: int, target_blocks: int = 1024, nreal: int = 0) -> None:
    """gw[m][n][kh][kw] += sum_p A[p][m] B[p*s + (kh, kw) - pad][n] (OIHW with O = A's channels), gb[m] +=
    sum_p A[p][m]; A is the pixel grid.  Split over pixel ranges into fp32 slabs, summed in a fixed order.
    ``nreal``: channels of B that gw holds (the first layer's zero padding channels are dropped)."""
    N, Hg, Wg, M, lda = nhwc(A, "wgrad_f32.A")
    NB, HB, WB, Nc, ldb = nhwc(B, "wgrad_f32.B")
    nreal = nreal or Nc
    assert NB == N and M % 32 == 0 and Nc % 4 == 0 and nreal <= Nc
    assert gw.dtype == torch.float32 and gw.is_contiguous() and gw.numel() == M * nreal * KH * KW
    assert gb is None or (gb.dtype == torch.float32 and gb.numel() == M)
    T = KH * KW
    P = N * Hg * Wg
    halo = int(USE_WGRAD_HALO and (KH, KW, s, pad) == (3, 3, 1, 1) and (HB, WB) == (Hg, Wg) and Hg % 2 == 0
               and Wg % 32 == 0 and Nc in (32, 64))
    if (WGRAD_C4 and (KH, KW, s, pad) == (3, 3, 1, 1) and (HB, WB) == (Hg, Wg) and Nc == 4 and M == 32
            and Wg % 64 == 0):
        halo = 3   # first layer: 64-pixel row segments, <= 512 blocks (splits)
        units = N * Hg * (Wg // 64)
        upb = -(-units // min(512, units))
        splits = -(-units // upb)
        pps = 64 * upb
    elif halo:     # stages of 2 rows x 32 pixels, all 9 taps of 32 A channels per block
        if Nc == 64 and WGRAD3_HALVES:
            halo = 2   # each block: one 32-column half of B
        nst = N * (Hg // 2) * (Wg // 32)
        splits = max(1, min(nst, -(-target_blocks // ((M // 32) * halo))))
        sps = -(-nst // splits)
        splits = -(-nst // sps)
        pps = 64 * sps
    else:
        bm, bn = wgrad_f32_tile(M, T * Nc, USE_WGRAD_BIG)
        tiles = (M // bm) * -(-(T * Nc) // bn)
        splits = max(1, min(-(-target_blocks // tiles), -(-P // 1024)))
        pps = round_up(-(-P // splits), 32)
        splits = -(-P // pps)
    slab = torch.empty(splits * T * M * Nc + (splits * M if gb is not None else 0), dtype=torch.float32, device=A.device)
    bslab = slab[splits * T * M * Nc:] if gb is not None else None
    a = F32WgradArgs(A.data_ptr(), B.data_ptr(), slab.data_ptr(), None if bslab is None else bslab.data_ptr(),
                     lda, ldb, N, Hg, Wg, HB, WB, M, Nc, s, pad, KH, KW, pps, splits, halo, int(USE_WGRAD_BIG),
                     int(WGRAD_PX))
    L = _lib.lib()
    st = _st(A)
    _check(L.dpa_wgrad_f32(ctypes.byref(a), st), "wgrad_f32")
    _check(L.dpa_wgrad_reduce(_p(slab), _p(bslab), _p(gw), _p(gb), c_int(splits), c_int(T), c_int(M), c_int(Nc),
                              c_int(nreal), c_int(0), st), "wgrad_reduce(f32)")


# ---------------------------------------------------------------------------------------- elementwise
def relu_bwd(g: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
    """g * (r > 0) (same shape, contiguous fp32)."""
    assert g.dtype == r.dtype == torch.float32 and g.shape == r.shape and g.is_contiguous() and r.is_contiguous()
    out = torch.empty_like(g)
    _check(_lib.lib().dpa_relu_bwd_f32(_p(g), _p(r), _p(out), c_ll(g.numel()), _st(g)), "relu_bwd_f32")
    return out


def maxpool2(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """2x2 max-pool + window codes of NHWC fp32 x (a channel slice allowed: the skip half of a concat buffer)."""
    N, H, W, C, ld = nhwc(x, "maxpool2_f32.x")
    y = torch.empty(N, H // 2, W // 2, C, dtype=torch.float32, device=x.device)
    code = torch.empty(N, H // 2, W // 2, C, dtype=torch.uint8, device=x.device)
    _check(_lib.lib().dpa_maxpool2_f32(_p(x), c_int(ld), _p(y), _p(code), c_int(N), c_int(H), c_int(W), c_int(C), _st(x)),
           "maxpool2_f32")
    return y, code


def maxpool2_bwd(g: torch.Tensor, code: torch.Tensor, H: int, W: int) -> torch.Tensor:
    N, Ho, Wo, C = g.shape
    assert g.is_contiguous() and code.shape == g.shape and (Ho, Wo) == (H // 2, W // 2)
    dx = torch.empty(N, H, W, C, dtype=torch.float32, device=g.device)
    _check(_lib.lib().dpa_maxpool2_bwd_f32(_p(g), _p(code), _p(dx), c_int(N), c_int(H), c_int(W), c_int(C), _st(g)),
           "maxpool2_bwd_f32")
    return dx


def enc_out_bwd(gs: Optional[torch.Tensor], gp: Optional[torch.Tensor], code: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """(y > 0) * (gs + maxpool2_bwd(gp, code)) in one pass: the gradient entering an encoder DoubleConv's
    last ReLU from its skip output (``gs``: NHWC, channel slice allowed) and its pooled output (``gp``)."""
    N, H, W, C, ldy = nhwc(y, "enc_out_bwd_f32.y")
    assert C % 4 == 0
    lds = 0
    if gs is not None:
        assert tuple(gs.shape) == (N, H, W, C)
        _, _, _, _, lds = nhwc(gs, "enc_out_bwd_f32.gs")
    if gp is not None:
        assert gp.is_contiguous() and code.shape == gp.shape and tuple(gp.shape) == (N, H // 2, W // 2, C)
    ge = torch.empty(N, H, W, C, dtype=torch.float32, device=y.device)
    _check(_lib.lib().dpa_enc_out_bwd_f32(_p(gs), c_int(lds), _p(gp), _p(code), _p(y), c_int(ldy), _p(ge), c_int(N),
                                         c_int(H), c_int(W), c_int(C), _st(y)), "enc_out_bwd_f32")
    return ge


def head_fwd(y: torch.Tensor, w: torch.Tensor, b: torch.Tensor, t: Optional[torch.Tensor], want_probs: bool = False):
    """Segmentation head on NHWC fp32 y: (S[4] partial sums or None, probabilities [P] or None)."""
    N, H, W, C, ld = nhwc(y, "head_f32.y")
    assert ld == C and y.is_contiguous()
    P = N * H * W
    L = _lib.lib()
    blocks = L.dpa_head_f32_blocks(c_ll(P))
    slab = torch.empty(blocks * 4, dtype=torch.float32, device=y.device)
    probs = torch.empty(P, dtype=torch.float32, device=y.device) if want_probs else None
    tf = None
    if t is not None:
        tf = t.reshape(-1).float().contiguous()
        assert tf.numel() == P
    w = w.detach().reshape(-1).float().contiguous()
    b = b.detach().reshape(-1).float().contiguous()
    st = _st(y)
    _check(L.dpa_head_f32(_p(y), c_int(C), _p(w), _p(b), _p(tf), c_ll(P), _p(slab), _p(probs), st), "head_f32")
    S = None
    if t is not None:
        S = torch.empty(4, dtype=torch.float32, device=y.device)
        _check(L.dpa_slab_sum(_p(slab), c_int(blocks), c_int(4), _p(S), st), "head_f32(slab_sum)")
    return S, probs


def head_bwd(y: torch.Tensor, w: torch.Tensor, b: torch.Tensor, t: torch.Tensor, dS: torch.Tensor,
             gw: Optional[torch.Tensor] = None, gb: Optional[torch.Tensor] = None, relu: bool = False):
    """(dL/dy of the head -- NHWC fp32, ReLU-backward masked by y > 0 with ``relu`` (y is then the last decoder
    block's ReLU output) --, segmap weight gradient [C], bias gradient [1]).
    With ``gw`` / ``gb`` (the flat gradient buffer's views, adjacent: weight then bias) the parameter
    gradients are reduced into them in place and returned as those views."""
    N, H, W, C, ld = nhwc(y, "head_bwd_f32.y")
    P = N * H * W
    L = _lib.lib()
    blocks = L.dpa_head_f32_blocks(c_ll(P))
    gy = torch.empty_like(y)
    slab = torch.empty(blocks * (C + 1), dtype=torch.float32, device=y.device)
    tf = t.reshape(-1).float().contiguous()
    dS = dS.reshape(-1).float().contiguous()
    wv = w.detach().reshape(-1).float().contiguous()
    bv = b.detach().reshape(-1).float().contiguous()
    st = _st(y)
    _check(L.dpa_head_bwd_f32(_p(y), c_int(C), _p(wv), _p(bv), _p(tf), _p(dS), c_ll(P), _p(gy), _p(slab), c_int(int(relu)), st),
           "head_bwd_f32")
    if (gw is not None and gb is not None and gw.is_contiguous() and gw.numel() == C and gb.numel() == 1
            and gb.data_ptr() == gw.data_ptr() + 4 * C):
        _check(L.dpa_wgrad_reduce_cfg(None, _p(slab), None, _p(gw), c_int(blocks), c_int(0), c_int(C + 1), c_int(1),
                                      c_int(1), c_int(0), c_int(0), st), "head_bwd_f32(reduce)")
        return gy, gw, gb
    red = slab.view(blocks, C + 1).sum(0)
    if gw is not None:
        gw.view(-1).add_(red[:C])
        gb.view(-1).add_(red[C:])
        return gy, gw, gb
    return gy, red[:C], red[C:]


def input_nhwc4(x: torch.Tensor) -> torch.Tensor:
    """NCHW fp32 (C <= 4) -> NHWC fp32 with 4 channels (zero padded)."""
    assert x.dtype == torch.float32 and x.dim() == 4 and x.shape[1] <= 4
    x = x.contiguous()
    N, C, H, W = x.shape
    y = torch.empty(N, H, W, 4, dtype=torch.float32, device=x.device)
    _check(_lib.lib().dpa_nchw_to_nhwc4_f32(_p(x), _p(y), c_int(N), c_int(C), c_ll(H * W), _st(x)), "nchw_to_nhwc4_f32")
    return y


def channel_sum(g: torch.Tensor, out: torch.Tensor) -> None:
    """out[c] += sum over pixels of NHWC fp32 g (channel slice allowed): per-block partial sums, then the
    fixed-order slab reduction of the weight gradients (bias rows only) straight into ``out``."""
    N, H, W, C, ld = nhwc(g, "channel_sum_f32.g")
    assert out.dtype == torch.float32 and out.is_contiguous() and out.numel() == C
    P = N * H * W
    L = _lib.lib()
    blocks = L.dpa_head_f32_blocks(c_ll(P))
    slab = torch.empty(blocks * C, dtype=torch.float32, device=g.device)
    st = _st(g)
    _check(L.dpa_channel_sum_f32(_p(g), c_ll(P), c_int(C), c_int(ld), _p(slab), st), "channel_sum_f32")
    _check(L.dpa_wgrad_reduce_cfg(None, _p(slab), None, _p(out), c_int(blocks), c_int(0), c_int(C), c_int(1), c_int(1),
                                  c_int(0), c_int(0), st), "channel_sum_f32(reduce)")


# ---------------------------------------------------------------------------------------- BN / bilinear
def _declare_norm():
    L = _lib.lib()
    for name in ("dpa_bn_fwd_f32", "dpa_bn_bwd_f32", "dpa_up2_fwd_f32", "dpa_up2_bwd_f32"):
        getattr(L, name).restype = ctypes.c_int
    L.dpa_bn_slab_rows_f32.restype = ctypes.c_int
    L.dpa_bn_slab_rows_f32.argtypes = [ctypes.c_longlong, ctypes.c_int]
    return L


def bn_fwd(z: torch.Tensor, bn: torch.nn.BatchNorm2d, train: bool, relu: bool = True,
           y: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """y = relu(BatchNorm2d(z)), NHWC fp32 (csrc/norm_up.hip fp32 forms; torch.nn.BatchNorm2d semantics:
    biased batch variance to normalise, unbiased for running_var, ``momentum`` update).  Returns (y, saved):
    saved = [mean, invstd] for :func:`bn_bwd` in training, None in eval (running statistics)."""
    L = _declare_norm()
    N, H, W, C, ldz = nhwc(z, "bn_fwd_f32.z")
    if y is None:
        y = torch.empty(N, H, W, C, dtype=torch.float32, device=z.device)
    _, _, _, _, ldy = nhwc(y, "bn_fwd_f32.y")
    P = N * H * W
    rows = L.dpa_bn_slab_rows_f32(P, C)
    slab = torch.empty(max(rows, 1) * 2 * C, dtype=torch.float32, device=z.device)
    coef = torch.empty(2 * C, dtype=torch.float32, device=z.device)
    saved = torch.empty(2 * C, dtype=torch.float32, device=z.device) if train else None
    track = train and bn.track_running_stats and bn.running_mean is not None
    if train and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    mom = bn.momentum if bn.momentum is not None else 0.1
    _check(L.dpa_bn_fwd_f32(_p(z), c_int(ldz), _p(y), c_int(ldy), c_ll(P), c_int(C), _p(bn.weight.detach()),
                            _p(bn.bias.detach()), ctypes.c_float(bn.eps), ctypes.c_float(mom),
                            _p(bn.running_mean) if (track or not train) else None,
                            _p(bn.running_var) if (track or not train) else None, _p(slab), _p(coef), _p(saved),
                            c_int(1 if train else 0), c_int(1 if relu else 0), _st(z)), "bn_fwd_f32")
    return y, saved


def bn_bwd(g: torch.Tensor, z: torch.Tensor, saved: torch.Tensor, bn: torch.nn.BatchNorm2d,
           dgamma: Optional[torch.Tensor], dbeta: Optional[torch.Tensor]) -> torch.Tensor:
    """dz from g = dL/d(BN output) with the ReLU mask applied; dgamma / dbeta += (the flat fp32 gradients)."""
    L = _declare_norm()
    N, H, W, C, ldg = nhwc(g, "bn_bwd_f32.g")
    _, _, _, _, ldz = nhwc(z, "bn_bwd_f32.z")
    P = N * H * W
    rows = L.dpa_bn_slab_rows_f32(P, C)
    slab = torch.empty(max(rows, 1) * 2 * C, dtype=torch.float32, device=g.device)
    coef3 = torch.empty(3 * C, dtype=torch.float32, device=g.device)
    dz = torch.empty(N, H, W, C, dtype=torch.float32, device=g.device)
    _check(L.dpa_bn_bwd_f32(_p(g), c_int(ldg), _p(z), c_int(ldz), _p(dz), c_int(C), c_ll(P), c_int(C),
                            _p(bn.weight.detach()), _p(saved), _p(slab), _p(coef3), _p(dgamma), _p(dbeta), _st(g)),
           "bn_bwd_f32")
    return dz


def up2_fwd(x: torch.Tensor, y: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Bilinear x2 up-sampling (align_corners=False) of NHWC fp32 x (into ``y``: a concat half allowed)."""
    L = _declare_norm()
    N, h, w, C, ldx = nhwc(x, "up2_f32.x")
    if y is None:
        y = torch.empty(N, 2 * h, 2 * w, C, dtype=torch.float32, device=x.device)
    Ny, Hy, Wy, Cy, ldy = nhwc(y, "up2_f32.y")
    assert (Ny, Hy, Wy, Cy) == (N, 2 * h, 2 * w, C)
    _check(L.dpa_up2_fwd_f32(_p(x), c_int(ldx), _p(y), c_int(ldy), c_int(N), c_int(h), c_int(w), c_int(C), _st(x)),
           "up2_fwd_f32")
    return y


def up2_bwd(g: torch.Tensor) -> torch.Tensor:
    L = _declare_norm()
    N, H, W, C, ldg = nhwc(g, "up2_bwd_f32.g")
    assert H % 2 == 0 and W % 2 == 0
    dx = torch.empty(N, H // 2, W // 2, C, dtype=torch.float32, device=g.device)
    _check(L.dpa_up2_bwd_f32(_p(g), c_int(ldg), _p(dx), c_int(C), c_int(N), c_int(H // 2), c_int(W // 2), c_int(C),
                             _st(g)), "up2_bwd_f32")
    return dx
