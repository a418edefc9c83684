"""The LDS-DMA GEMMs that carry the deep and 128-channel UNet levels (csrc/igemm_glds.hip):
``igemm_pp2h_kernel`` (cfg 14 / 15: row-block staging, four quadrant phases per K-tile) and
``igemm_sl_kernel`` (cfg 18: slice-staged 128 x 512 tiles, the default for 128-output-channel layers on
rows of <= 128 pixels), anchored DIRECTLY to a plain PyTorch fp32 convolution at real 512^2-UNet layer
shapes (64^2 / 32^2 / 128^2 grids, 256-pixel parts of 512- and 768-wide rows) for every specialised
epilogue the model uses: forward bias + ReLU, dgrad with the ReLU-backward mask, the split dgrad of a
concat input, and the BatchNorm partial sums of the forward and backward epilogues.

Inputs are bf16-rounded (the kernels' storage type); the fp32 reference sees the same values, so what
remains is the fp32 accumulation order and the bf16 rounding of the output (< 1e-2 of the output's
max magnitude).  The generic (pointer-math) epilogue must equal the specialised ones bitwise.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

PP2H = {256: 14, 128: 15}
SL = 262144                          # slice-staged kernel variant code (cfg 18: 128 x 512 tiles)


def _sl_ok(H, W, Ng):
    return W in (32, 64, 128) and (H * W) % 512 == 0 and Ng % 128 == 0


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def _operands(N, H, W, Cs, Ng, seed):
    """x [N,H,W,Cs] bf16 (cuda), packed GEMM weights w [Ng][9 Cs] (k = tap * Cs + ci, tap = 3 kh + kw),
    and the same weights as an fp32 OIHW conv kernel for F.conv2d."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, H, W, Cs, generator=g).to(torch.bfloat16)
    w = (torch.randn(Ng, 9 * Cs, generator=g) / (9 * Cs) ** 0.5).to(torch.bfloat16)
    wconv = w.float().view(Ng, 9, Cs).permute(0, 2, 1).reshape(Ng, Cs, 3, 3)
    return x.cuda(), w.cuda(), x.float().permute(0, 3, 1, 2), wconv


def _ref_conv(xc, wconv):
    return F.conv2d(xc, wconv, padding=1).permute(0, 2, 3, 1)          # NHWC fp32


SHAPES = [
    # (N, H, W, Cs, Ngemm): 512^2 UNet layers at small batch (enc4 / dec1 at 64^2, mid at 32^2, the
    # 128-channel level at 128^2, enc4.0's 128-channel dgrad at 64^2) and 256-pixel parts of wide rows
    (2, 64, 64, 256, 256), (2, 32, 32, 512, 512), (2, 128, 128, 128, 128), (2, 64, 64, 256, 128),
    (2, 128, 128, 256, 128), (1, 8, 512, 64, 256), (1, 6, 768, 128, 128),
]


def _run(kind, x, w, N, H, W, Cs, Ng, variant, extra):
    from distributedpytorch_amd.ops import kernels as K
    y = torch.empty(N, H, W, Ng if kind != "split" else extra["split"], dtype=torch.bfloat16, device="cuda")
    kw = dict(extra)
    stats = None
    if kind == "split":
        kw["y2"] = torch.empty(N, H, W, Ng - extra["split"], dtype=torch.bfloat16, device="cuda")
    if kind.startswith("bn"):
        stats = []
        kw["bn_stats"] = stats
    K.igemm(x, w, y, Ngemm=Ng, Kpad=9 * Cs, KH=3, KW=3, stride=1, pad=1, Cs=Cs, out_grid=(N, H, W),
            path="auto" if kind.startswith("bn") else "glds", variant=variant, **kw)
    torch.cuda.synchronize()
    return y, kw.get("y2"), stats


def _extra(kind, N, H, W, Ng, seed):
    g = torch.Generator().manual_seed(seed + 1)
    if kind == "fwd":
        return dict(bias=(torch.randn(Ng, generator=g) * 0.1).cuda(), relu=True)
    if kind == "bn_fwd":    # conv followed by BatchNorm: bias, no ReLU, batch sums of the stored output
        return dict(bias=(torch.randn(Ng, generator=g) * 0.1).cuda(), relu=False)
    if kind in ("dgrad", "bn_dgrad"):   # mask = the (ReLU / BN+ReLU) output of the layer below
        return dict(mask=torch.relu(torch.randn(N, H, W, Ng, generator=g)).to(torch.bfloat16).cuda())
    if kind == "split":
        return dict(split=Ng // 2)
    raise ValueError(kind)


def _expected(kind, ref, extra):
    if kind == "fwd":
        return torch.relu(ref + extra["bias"].cpu())
    if kind == "bn_fwd":
        return ref + extra["bias"].cpu()
    if kind in ("dgrad", "bn_dgrad"):
        return ref * (extra["mask"].float().cpu() > 0)
    return ref


@pytest.mark.parametrize("kind", ["fwd", "dgrad", "split", "bn_fwd", "bn_dgrad"])
@pytest.mark.parametrize("shape", SHAPES)
def test_rowblock_fp32_anchor(hip_lib, shape, kind):
    N, H, W, Cs, Ng = shape
    x, w, xc, wconv = _operands(N, H, W, Cs, Ng, seed=31 + Cs + Ng)
    ref = _ref_conv(xc, wconv)
    extra = _extra(kind, N, H, W, Ng, seed=Cs)
    exp = _expected(kind, ref, extra)
    bc = 256 if Ng % 256 == 0 else 128
    v = PP2H[bc]
    y, y2, stats = _run(kind, x, w, N, H, W, Cs, Ng, v, extra)
    got = torch.cat([y, y2], dim=3) if kind == "split" else y
    assert _rel(got.float().cpu(), exp) < 1e-2, (v, kind)
    if kind.startswith("bn"):
        assert stats, "the row-block epilogue did not take the BatchNorm sums"
        slab, rows = stats
        sums = slab.view(rows, 2, Ng).double().sum(0).cpu()
        yd = y.double().cpu().reshape(-1, Ng)
        s2 = (yd * yd) if kind == "bn_fwd" else (yd * extra["mask"].double().cpu().reshape(-1, Ng))
        assert _rel(sums[0], yd.sum(0)) < 1e-4 and _rel(sums[1], s2.sum(0)) < 1e-4, (v, kind)
    elif _sl_ok(H, W, Ng):            # slice-staged kernel: 32-channel K order, fp32 anchor
        y, y2, _ = _run(kind, x, w, N, H, W, Cs, Ng, SL, extra)
        got = torch.cat([y, y2], dim=3) if kind == "split" else y
        assert _rel(got.float().cpu(), exp) < 1e-2, ("sl", kind)


@pytest.mark.parametrize("N,H,W,Cs,Ng,kind", [(3, 30, 128, 64, 256, "dgrad"), (2, 70, 256, 64, 256, "fwd"),
                                               (16, 32, 32, 128, 256, "fwd"), (2, 9, 512, 64, 256, "dgrad"),
                                               (4, 128, 128, 128, 128, "fwd"), (3, 30, 256, 64, 128, "dgrad"),
                                               (2, 64, 64, 256, 384, "fwd"), (8, 32, 32, 64, 128, "dgrad")])
def test_rowblock_generic_epilogue_bitwise(hip_lib, N, H, W, Cs, Ng, kind):
    """Partial last row groups, 8 / 2 / 1 rows per tile: the specialised epilogue == the generic
    (pointer-math) epilogue (variant + 2048) bitwise, for the row-block and the slice-staged kernels."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(37)
    x = torch.randn(N, H, W, Cs, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Ng, 9 * Cs, device="cuda") / (9 * Cs) ** 0.5).to(torch.bfloat16)
    extra = (dict(bias=torch.randn(Ng, device="cuda") * 0.1, relu=True) if kind == "fwd" else
             dict(mask=torch.randn(N, H, W, Ng, device="cuda").to(torch.bfloat16)))
    bc = 256 if Ng % 256 == 0 else 128
    variants = [PP2H[bc]] + ([SL] if _sl_ok(H, W, Ng) else [])
    for v in variants:
        outs = []
        for vv in (v, v + 2048):
            y = torch.empty(N, H, W, Ng, device="cuda", dtype=torch.bfloat16)
            K.igemm(x, w, y, Ngemm=Ng, Kpad=9 * Cs, KH=3, KW=3, stride=1, pad=1, Cs=Cs, out_grid=(N, H, W),
                    path="glds", variant=vv, **extra)
            outs.append(y)
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1]), v


@pytest.mark.parametrize("N,H,W,Cs,Ng,kind", [(2, 128, 128, 128, 128, "fwd"), (2, 128, 128, 256, 128, "dgrad"),
                                               (2, 64, 64, 256, 128, "dgrad"), (3, 32, 32, 64, 128, "fwd"),
                                               (2, 128, 128, 64, 256, "fwd"), (1, 16, 128, 64, 128, "dgrad")])
def test_slice_staged_pingpong_bitwise(hip_lib, N, H, W, Cs, Ng, kind):
    """igemm_slp_kernel (the ping-pong schedule of the slice-staged 128 x 512 tile, one phase per tap) runs
    the same MFMA sequence on every accumulator as igemm_sl_kernel (three taps per barrier step): bitwise
    equal outputs, one slice to eight, 4 / 8 / 16 image rows per tile, two channel tiles."""
    import ctypes
    from distributedpytorch_amd.ops import _lib
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(41)
    x = torch.randn(N, H, W, Cs, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Ng, 9 * Cs, device="cuda") / (9 * Cs) ** 0.5).to(torch.bfloat16)
    extra = (dict(bias=torch.randn(Ng, device="cuda") * 0.1, relu=True) if kind == "fwd" else
             dict(mask=torch.randn(N, H, W, Ng, device="cuda").to(torch.bfloat16)))
    L = _lib.lib()
    outs = []
    try:
        for on in (1, 0):
            L.dpa_igemm_set_slpp(ctypes.c_int(on))
            y = torch.empty(N, H, W, Ng, device="cuda", dtype=torch.bfloat16)
            K.igemm(x, w, y, Ngemm=Ng, Kpad=9 * Cs, KH=3, KW=3, stride=1, pad=1, Cs=Cs, out_grid=(N, H, W),
                    path="glds", variant=SL, **extra)
            torch.cuda.synchronize()
            outs.append(y)
    finally:
        L.dpa_igemm_set_slpp(ctypes.c_int(int(K.CFG.slpp)))
    assert torch.equal(outs[0], outs[1])
    ref = _ref_conv(x.float().cpu().permute(0, 3, 1, 2),
                    w.float().cpu().view(Ng, 9, Cs).permute(0, 2, 1).reshape(Ng, Cs, 3, 3))
    assert _rel(outs[0].float().cpu(), _expected(kind, ref, extra)) < 1e-2


@pytest.mark.parametrize("kind", ["fwd", "dgrad", "split"])
@pytest.mark.parametrize("shape", [(2, 64, 64, 256, 256), (2, 32, 32, 512, 512), (2, 64, 64, 512, 256),
                                   (3, 32, 32, 256, 512)])
def test_slp256_fp32_anchor(hip_lib, shape, kind):
    """igemm_slp_kernel<EP, 256> (DPA_SLP256: the 256-channel convs of the 64^2 / 32^2 levels as slice-staged
    ping-pong instead of the row-block kernel) at real layer shapes for the forward, the masked dgrad and the
    split dgrad epilogues: within bf16 output rounding of the fp32 convolution, like the row-block kernel."""
    import ctypes
    from distributedpytorch_amd.ops import _lib
    from distributedpytorch_amd.ops import kernels as K
    N, H, W, Cs, Ng = shape
    x, w, xc, wconv = _operands(N, H, W, Cs, Ng, seed=43 + Cs)
    exp = _expected(kind, _ref_conv(xc, wconv), _extra(kind, N, H, W, Ng, seed=Cs))
    L = _lib.lib()
    try:
        for on in (1, 0):
            L.dpa_igemm_set_slp256(ctypes.c_int(on))
            y, y2, _ = _run(kind, x, w, N, H, W, Cs, Ng, PP2H[256], _extra(kind, N, H, W, Ng, seed=Cs))
            got = torch.cat([y, y2], dim=3) if kind == "split" else y
            assert _rel(got.float().cpu(), exp) < 1e-2, (on, kind)
    finally:
        L.dpa_igemm_set_slp256(ctypes.c_int(int(K.CFG.slp256)))


@pytest.mark.parametrize("N,H,W,Cs,kind", [(2, 256, 256, 128, "fwd"), (2, 128, 128, 128, "dgrad"),
                                           (2, 64, 64, 256, "fwd"), (3, 32, 32, 64, "dgrad")])
def test_slp64_bitwise_vs_halo(hip_lib, N, H, W, Cs, kind):
    """igemm_slp_kernel<EP, 64> (cfg 19, DPA_SLP64: the 64-output-channel convs as slice-staged ping-pong,
    waves 4-7 issuing dummy weight DMAs, the next image 3 slots per phase) runs each accumulator's MFMAs in the
    row-halo kernel's order (slice, then tap): bitwise equal to row-halo cfg 4 where that takes the shape, and
    within bf16 rounding of the fp32 convolution; 2-8 image rows per 512-pixel tile."""
    from distributedpytorch_amd.ops import kernels as K
    Ng = 64
    torch.manual_seed(47 + Cs + W)
    x = torch.randn(N, H, W, Cs, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Ng, 9 * Cs, device="cuda") / (9 * Cs) ** 0.5).to(torch.bfloat16)
    extra = (dict(bias=torch.randn(Ng, device="cuda") * 0.1, relu=True) if kind == "fwd" else
             dict(mask=torch.randn(N, H, W, Ng, device="cuda").to(torch.bfloat16)))
    y = torch.empty(N, H, W, Ng, device="cuda", dtype=torch.bfloat16)
    K.igemm(x, w, y, Ngemm=Ng, Kpad=9 * Cs, KH=3, KW=3, stride=1, pad=1, Cs=Cs, out_grid=(N, H, W),
            path="glds", variant=524288, **extra)
    torch.cuda.synchronize()
    if W % 128 == 0:
        yh = torch.empty_like(y)
        K.igemm(x, w, yh, Ngemm=Ng, Kpad=9 * Cs, KH=3, KW=3, stride=1, pad=1, Cs=Cs, out_grid=(N, H, W),
                path="halo", variant=4, **extra)
        torch.cuda.synchronize()
        assert torch.equal(y, yh)
    ref = _ref_conv(x.float().cpu().permute(0, 3, 1, 2),
                    w.float().cpu().view(Ng, 9, Cs).permute(0, 2, 1).reshape(Ng, Cs, 3, 3))
    assert _rel(y.float().cpu(), _expected(kind, ref, extra)) < 1e-2
