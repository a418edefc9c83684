"""Numerics of every gfx950 kernel against a plain PyTorch fp32 CPU reference of the same op.

Inputs are rounded to bf16 first (the kernels' storage type), so the only differences left are the
fp32-accumulation order and the final bf16 rounding of the outputs -> tolerances ~1e-2 relative to
the output's max magnitude.  Shapes cover the first layer (3 -> padded 8 channels), odd spatial
sizes (partial tiles, zero padding), concat-buffer strides and every tile family.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def _bf(t):
    return t.to(torch.bfloat16).float()


def _nhwc(x):   # NCHW fp32 -> NHWC bf16 cuda
    return x.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)


def _nchw(y):   # NHWC cuda -> NCHW fp32 cpu
    return y.float().permute(0, 3, 1, 2).cpu()


def _pack_one(mode, w, cin_pad=None):
    """Pack a single fp32 weight with the production pack kernel."""
    from distributedpytorch_amd.ops import kernels as K
    flat = w.reshape(-1).float().cuda().contiguous()
    if mode in (0, 1):
        Cout, Cin = w.shape[:2]
        Cs = cin_pad or Cin
        if mode == 0:
            ngemm, kpad, cs = Cout, K.round_up(9 * Cs, 32), Cs
        else:
            ngemm, kpad, cs = Cin, K.round_up(9 * Cout, 32), Cout
    else:
        Cin, Cout = w.shape[:2]
        if mode == 2:
            ngemm, kpad, cs = 4 * Cout, K.round_up(Cin, 32), Cin
        else:
            ngemm, kpad, cs = Cin, K.round_up(4 * Cout, 32), Cout
    d = K.PackDesc(flat.data_ptr(), 0, mode, Cout, Cin, cs, ngemm, kpad)
    descs = torch.frombuffer(bytearray(bytes(d)), dtype=torch.uint8).cuda()
    packed = torch.empty(ngemm * kpad, dtype=torch.bfloat16, device="cuda")
    K.pack_weights(packed, descs, 1, ngemm * kpad)
    return packed, ngemm, kpad


@pytest.mark.parametrize("Cout,Cin,cs", [(32, 3, 8), (64, 32, 32), (96, 160, 160), (256, 512, 512)])
def test_pack_weights_conv_layouts(hip_lib, Cout, Cin, cs):
    """The weight pack kernel's conv3x3 forward (mode 0) and dgrad (mode 1) layouts, bit for bit against a torch
    construction: dst[co][tap*Cs + ci] = W[co][ci][tap] (ci >= Cin zero) and dst[ci][tap*Cout + co] =
    W[co][ci][8 - tap]; K padding columns zero."""
    torch.manual_seed(5)
    w = torch.randn(Cout, Cin, 3, 3)
    p0, ng0, kp0 = _pack_one(0, w, cs)
    r0 = torch.zeros(Cout, kp0)
    r0[:, :9 * cs].view(Cout, 9, cs)[:, :, :Cin] = w.reshape(Cout, Cin, 9).permute(0, 2, 1)
    assert torch.equal(p0.view(ng0, kp0).cpu(), r0.to(torch.bfloat16))
    p1, ng1, kp1 = _pack_one(1, w)
    r1 = torch.zeros(Cin, kp1)
    r1[:, :9 * Cout].view(Cin, 9, Cout)[:] = w.reshape(Cout, Cin, 9).flip(2).permute(1, 2, 0)
    assert torch.equal(p1.view(ng1, kp1).cpu(), r1.to(torch.bfloat16))


@pytest.mark.parametrize("N,H,W,Cin,Cout,cfg", [
    (2, 17, 23, 3, 32, 0),      # first layer: 3 -> padded 8 input channels, partial tiles
    (2, 16, 16, 32, 64, 0),
    (1, 12, 20, 64, 128, 0),
    (1, 8, 8, 128, 256, 0),
    (1, 8, 8, 256, 256, 7),
    (2, 16, 16, 64, 32, 5),
    (2, 16, 16, 64, 32, 6),
    (1, 16, 16, 64, 128, 1),
    (1, 16, 16, 64, 128, 2),
    (1, 16, 16, 64, 64, 3),
    (1, 16, 16, 64, 64, 4),
    # row-streaming / row-halo kernels (W a multiple of the 128/256-pixel tile)
    (2, 3, 256, 32, 32, "stream"), (2, 3, 256, 32, 32, "halo"),
    (1, 37, 128, 64, 32, "stream"), (1, 4, 256, 64, 32, "halo"),
    (1, 3, 128, 32, 64, "stream"), (1, 3, 128, 32, 64, "halo"),
    (2, 20, 128, 64, 64, "stream"),
    # rows narrower than the 128-pixel strip: the 64-pixel variant of the same channel pair
    (2, 5, 64, 32, 32, "stream"), (1, 3, 64, 32, 64, "stream"), (1, 6, 192, 64, 64, "stream"),
    (2, 2, 128, 64, 128, "auto"),
    (2, 5, 128, 3, 32, "stream"),          # first layer (8 padded channels) streaming kernel
    (1, 34, 256, 3, 32, "auto"),
    (2, 5, 128, 3, 64, "stream"), (1, 35, 256, 3, 64, "auto"), (1, 5, 200, 3, 64, "stream"),   # UNet-XL first conv
    # ragged rows (640x960 widths 480 / 240 / 120 and others): a partial last strip / tile
    (2, 5, 96, 32, 32, "stream"), (1, 6, 240, 64, 64, "stream"), (1, 4, 480, 32, 64, "auto"),
    (1, 4, 240, 64, 128, "halo"), (2, 3, 120, 128, 128, "halo"), (1, 3, 480, 64, 32, "halo"),
    (1, 5, 200, 3, 32, "stream"), (2, 4, 240, 128, 128, "auto"),
])
def test_conv3x3_fwd(hip_lib, N, H, W, Cin, Cout, cfg):
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(0)
    x = _bf(torch.randn(N, Cin, H, W))
    w = _bf(torch.randn(Cout, Cin, 3, 3) * (2.0 / (9 * Cin)) ** 0.5)
    b = torch.randn(Cout) * 0.1
    ref = F.relu(F.conv2d(x, w, b, padding=1))
    Cs = K.round_up(Cin, 8)
    xin = torch.zeros(N, Cs, H, W)
    xin[:, :Cin] = x
    packed, ng, kp = _pack_one(0, w, Cs)
    y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device="cuda")
    path = cfg if isinstance(cfg, str) else "auto"
    cfg = cfg if isinstance(cfg, int) else 0
    K.igemm(_nhwc(xin), packed, y, Ngemm=ng, Kpad=kp, KH=3, KW=3, stride=1, pad=1, Cs=Cs, out_grid=(N, H, W),
            bias=b.cuda(), relu=True, cfg=cfg, path=path)
    torch.cuda.synchronize()
    assert _rel(_nchw(y), ref) < 2e-2


@pytest.mark.parametrize("N,H,W,Cin,Cout,path", [
    (2, 13, 18, 32, 64, "auto"), (1, 8, 8, 256, 128, "auto"), (2, 16, 16, 64, 32, "auto"),
    (2, 3, 256, 32, 32, "stream"), (1, 3, 256, 64, 32, "halo"), (1, 2, 128, 32, 64, "stream"),
    (1, 35, 128, 64, 64, "stream"), (2, 3, 256, 32, 32, "generic"), (2, 5, 64, 32, 32, "stream"),
    (1, 4, 192, 64, 64, "stream"),
    # ragged rows
    (1, 4, 240, 128, 64, "halo"), (2, 3, 96, 64, 32, "stream"), (1, 3, 120, 128, 128, "auto")])
def test_conv3x3_dgrad_masked(hip_lib, N, H, W, Cin, Cout, path):
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(1)
    x = _bf(F.relu(torch.randn(N, Cin, H, W)))          # a ReLU output -> mask source
    w = _bf(torch.randn(Cout, Cin, 3, 3) * 0.05)
    g = _bf(torch.randn(N, Cout, H, W))
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, w, padding=1).backward(g)
    ref = xr.grad * (x > 0)
    packed, ng, kp = _pack_one(1, w)
    out = torch.empty(N, H, W, Cin, dtype=torch.bfloat16, device="cuda")
    K.igemm(_nhwc(g), packed, out, Ngemm=ng, Kpad=kp, KH=3, KW=3, stride=1, pad=1, Cs=Cout, out_grid=(N, H, W),
            mask=_nhwc(x), path=path)
    torch.cuda.synchronize()
    assert _rel(_nchw(out), ref) < 2e-2


@pytest.mark.parametrize("N,H,W,Cin,Cout,var", [
    (2, 9, 13, 128, 256, 1), (1, 16, 16, 256, 256, 1), (2, 9, 13, 64, 128, 2), (2, 7, 11, 128, 128, 4),
    (1, 32, 32, 64, 256, 0), (3, 11, 7, 512, 256, 0),
    # persistent kernel (one workgroup per CU, several tiles each when tiles > CUs)
    (2, 9, 13, 128, 256, 8), (1, 16, 16, 256, 512, 8), (2, 128, 160, 128, 512, 8),
    # ping-pong kernel with per-K-tile staging (shapes the row-block form does not take)
    (2, 9, 13, 128, 256, 14), (1, 16, 16, 256, 256, 14), (3, 11, 7, 512, 256, 14), (2, 5, 6, 256, 512, 14),
    # >= 4 channel tiles: grouped tile order, full and partial groups of 8 pixel tiles
    (2, 40, 40, 64, 1024, 8), (2, 40, 40, 256, 1024, 14)])
def test_conv3x3_glds(hip_lib, N, H, W, Cin, Cout, var):
    """LDS-DMA implicit GEMM (csrc/igemm_glds.hip): fwd with bias+ReLU and masked dgrad, every tile
    config, pixel counts that are not tile multiples (zero-filled DMA rows)."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(7)
    x = _bf(F.relu(torch.randn(N, Cin, H, W)))
    w = _bf(torch.randn(Cout, Cin, 3, 3) * (2.0 / (9 * Cin)) ** 0.5)
    b = torch.randn(Cout) * 0.1
    ref = F.relu(F.conv2d(x, w, b, padding=1))
    packed, ng, kp = _pack_one(0, w, Cin)
    y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device="cuda")
    K.igemm(_nhwc(x), packed, y, Ngemm=ng, Kpad=kp, KH=3, KW=3, stride=1, pad=1, Cs=Cin, out_grid=(N, H, W),
            bias=b.cuda(), relu=True, path="glds", variant=var)
    torch.cuda.synchronize()
    assert _rel(_nchw(y), ref) < 2e-2
    if Cin % 128:          # dgrad has Ngemm = Cin: needs a 128-multiple
        return
    g = _bf(torch.randn(N, Cout, H, W))
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, w, padding=1).backward(g)
    dref = xr.grad * (x > 0)
    packed, ng, kp = _pack_one(1, w)
    dx = torch.empty(N, H, W, Cin, dtype=torch.bfloat16, device="cuda")
    v = var if (var not in (1, 8, 14) or Cin % 256 == 0) else 2      # 256-channel tiles need Ngemm % 256
    K.igemm(_nhwc(g), packed, dx, Ngemm=ng, Kpad=kp, KH=3, KW=3, stride=1, pad=1, Cs=Cout, out_grid=(N, H, W),
            mask=_nhwc(x), path="glds", variant=v)
    torch.cuda.synchronize()
    assert _rel(_nchw(dx), dref) < 2e-2


@pytest.mark.parametrize("N,h,w,Cin,Cout", [(2, 5, 7, 64, 32), (1, 4, 4, 512, 256), (2, 8, 8, 128, 64),
                                          (2, 7, 9, 256, 128), (1, 33, 17, 512, 256)])
def test_deconv_fwd_into_concat(hip_lib, N, h, w, Cin, Cout):
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(2)
    x = _bf(torch.randn(N, Cin, h, w))
    wt = _bf(torch.randn(Cin, Cout, 2, 2) * 0.05)
    b = torch.randn(Cout) * 0.1
    ref = F.conv_transpose2d(x, wt, b, stride=2)
    packed, ng, kp = _pack_one(2, wt)
    cat = torch.full((N, 2 * h, 2 * w, 2 * Cout), 7.0, dtype=torch.bfloat16, device="cuda")
    K.igemm(_nhwc(x), packed, cat[..., Cout:], Ngemm=ng, Kpad=kp, KH=1, KW=1, stride=1, pad=0, Cs=Cin,
            out_grid=(N, h, w), bias=b.cuda(), mode=1, Cout=Cout)
    torch.cuda.synchronize()
    assert _rel(_nchw(cat[..., Cout:]), ref) < 2e-2
    assert (cat[..., :Cout] == 7.0).all()              # skip half untouched


@pytest.mark.parametrize("N,h,w,Cin,Cout", [(2, 5, 7, 64, 32), (1, 4, 4, 512, 256)])
def test_deconv_dgrad_from_concat(hip_lib, N, h, w, Cin, Cout):
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(3)
    x = _bf(F.relu(torch.randn(N, Cin, h, w)))
    wt = _bf(torch.randn(Cin, Cout, 2, 2) * 0.05)
    gup = _bf(torch.randn(N, Cout, 2 * h, 2 * w))
    xr = x.clone().requires_grad_(True)
    F.conv_transpose2d(xr, wt, stride=2).backward(gup)
    ref = xr.grad * (x > 0)
    packed, ng, kp = _pack_one(3, wt)
    dcat = torch.zeros(N, 2 * h, 2 * w, 2 * Cout, dtype=torch.bfloat16, device="cuda")
    dcat[..., Cout:] = _nhwc(gup)
    out = torch.empty(N, h, w, Cin, dtype=torch.bfloat16, device="cuda")
    K.igemm(dcat[..., Cout:], packed, out, Ngemm=ng, Kpad=kp, KH=2, KW=2, stride=2, pad=0, Cs=Cout,
            out_grid=(N, h, w), mask=_nhwc(x))
    torch.cuda.synchronize()
    assert _rel(_nchw(out), ref) < 2e-2


@pytest.mark.parametrize("N,H,W,Cin,Cout,cin_pad,path", [
    (2, 19, 21, 3, 32, 8, "auto"), (2, 16, 16, 32, 32, None, "auto"), (1, 12, 16, 64, 128, None, "auto"),
    (2, 8, 8, 128, 64, None, "auto"),
    # row-halo wgrad (W % 32 == 0)
    (2, 5, 32, 32, 32, None, "halo"), (1, 4, 64, 64, 32, None, "halo"), (2, 3, 32, 32, 64, None, "halo"),
    (1, 4, 32, 128, 64, None, "halo"), (2, 4, 32, 3, 32, 8, "auto"),
    # row-streaming wgrad (W % 64 == 0), odd row counts -> partial row segments
    (2, 5, 64, 32, 32, None, "stream"), (1, 37, 64, 64, 32, None, "stream"), (2, 3, 128, 32, 64, None, "stream"),
    (1, 70, 64, 128, 64, None, "stream"), (1, 4, 64, 64, 128, None, "generic"),
    # 32-pixel strips (the 32x32 bottleneck): W % 64 != 0
    (2, 5, 32, 32, 32, None, "stream"), (1, 33, 32, 64, 128, None, "stream"), (2, 3, 96, 128, 64, None, "stream"),
    # first layer through the streaming wgrad (8 padded input channels in a 16-wide tile)
    (2, 5, 128, 3, 32, 8, "stream"), (1, 66, 64, 3, 32, 8, "stream"),
    # ragged rows (partial last strip: out-of-row gradient pixels read as zeros)
    (1, 5, 240, 128, 64, None, "stream"), (2, 3, 120, 64, 128, None, "stream"), (1, 4, 60, 128, 128, None, "stream"),
    (2, 5, 200, 3, 32, 8, "stream"), (1, 3, 480, 64, 64, None, "stream"),
    # deep-layer shapes through the automatic choice (band128 on W % 64 grids, the row-streaming kernel on ragged
    # widths: odd row counts, W = 120 / 48 / 100, 192 input channels)
    (2, 5, 64, 128, 128, None, "auto"), (1, 7, 120, 64, 128, None, "auto"), (2, 4, 128, 256, 256, None, "auto"),
    (1, 3, 48, 64, 256, None, "auto"), (1, 66, 64, 128, 128, None, "auto"), (2, 9, 100, 192, 128, None, "auto"),
    # deep layers as a dense 256x256 LDS-DMA GEMM (csrc/wgrad_gemm.hip): partial last column tile
    # (9 x 128 = 1152, 9 x 64 = 576 columns), 32-wide rows (two rows per K-step), several channel tiles
    (2, 4, 64, 128, 256, None, "gemm"), (3, 6, 32, 256, 256, None, "gemm"), (1, 2, 128, 64, 512, None, "gemm"),
    (2, 5, 64, 512, 256, None, "gemm"),
    # deep layers with the input band staged once for all 9 taps (csrc/wgrad_band.hip): 64-wide rows (one row
    # per K-step), 32-wide rows (two), several channel and output-channel tiles, one-image batches
    (2, 4, 64, 128, 256, None, "band"), (3, 6, 32, 256, 256, None, "band"), (2, 5, 64, 512, 256, None, "band"),
    (1, 2, 32, 64, 512, None, "band"), (3, 2, 64, 32, 256, None, "band"), (1, 1, 64, 32, 256, None, "band"),
    # its 128-output-channel form (W % 64 == 0: K-steps are 64-pixel strips of one row, real halo columns)
    (2, 4, 128, 64, 128, None, "band128"), (1, 3, 192, 128, 128, None, "band128"), (2, 2, 64, 256, 128, None, "band128"),
    (1, 5, 128, 64, 256, None, "band128"), (2, 1, 64, 64, 128, None, "band128")])
def test_conv3x3_wgrad(hip_lib, N, H, W, Cin, Cout, cin_pad, path):
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(4)
    x = _bf(torch.randn(N, Cin, H, W))
    g = _bf(torch.randn(N, Cout, H, W))
    wr = torch.zeros(Cout, Cin, 3, 3, requires_grad=True)
    br = torch.zeros(Cout, requires_grad=True)
    F.conv2d(x, wr, br, padding=1).backward(g)
    Cs = cin_pad or Cin
    xin = torch.zeros(N, Cs, H, W)
    xin[:, :Cin] = x
    gw = torch.full((Cout, Cin, 3, 3), 0.5, device="cuda")    # accumulates on top
    gb = torch.full((Cout,), 0.5, device="cuda")
    K.wgrad(_nhwc(g), _nhwc(xin), kind=0, grid=(N, H, W), M=Cout, Nc=Cs, s=1, pad=1, KW=3, gw=gw.view(-1), gb=gb,
            Nreal=Cin, path=path)
    torch.cuda.synchronize()
    assert _rel(gw.cpu() - 0.5, wr.grad) < 1e-2
    assert _rel(gb.cpu() - 0.5, br.grad) < 1e-2


@pytest.mark.parametrize("N,h,w,Cin,Cout", [(2, 5, 7, 64, 32), (1, 4, 4, 512, 256), (2, 8, 8, 128, 64),
                                          (2, 7, 9, 256, 128), (1, 33, 17, 512, 256)])
def test_deconv_wgrad(hip_lib, N, h, w, Cin, Cout):
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(5)
    x = _bf(torch.randn(N, Cin, h, w))
    gup = _bf(torch.randn(N, Cout, 2 * h, 2 * w))
    wr = torch.zeros(Cin, Cout, 2, 2, requires_grad=True)
    br = torch.zeros(Cout, requires_grad=True)
    F.conv_transpose2d(x, wr, br, stride=2).backward(gup)
    dcat = torch.zeros(N, 2 * h, 2 * w, 2 * Cout, dtype=torch.bfloat16, device="cuda")
    dcat[..., Cout:] = _nhwc(gup)
    gw = torch.zeros(Cin, Cout, 2, 2, device="cuda")
    gb = torch.zeros(Cout, device="cuda")
    K.wgrad(dcat[..., Cout:], _nhwc(x), kind=1, grid=(N, h, w), M=Cout, Nc=Cin, s=2, pad=0, KW=2, gw=gw.view(-1),
            gb=gb, Nreal=Cin)
    torch.cuda.synchronize()
    assert _rel(gw.cpu(), wr.grad) < 1e-2
    assert _rel(gb.cpu(), br.grad) < 1e-2


@pytest.mark.parametrize("N,h,w,Cin,Cout", [(2, 5, 7, 64, 32), (1, 8, 8, 128, 64), (2, 33, 31, 128, 64)])
def test_deconv_fwd_fused(hip_lib, N, h, w, Cin, Cout):
    """Full-resolution transposed-conv forward (csrc/deconv.hip) into the concat buffer's second half."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(7)
    x = _bf(torch.randn(N, Cin, h, w))
    wt = torch.randn(Cin, Cout, 2, 2) / Cin ** 0.5
    b = torch.randn(Cout)
    ref = F.conv_transpose2d(x, _bf(wt), b, stride=2)
    wf, _, _ = _pack_one(2, wt)
    cat = torch.zeros(N, 2 * h, 2 * w, 2 * Cout, dtype=torch.bfloat16, device="cuda")
    K.deconv_fwd_fused(_nhwc(x), wf, b.cuda(), cat[..., Cout:])
    torch.cuda.synchronize()
    assert _rel(_nchw(cat[..., Cout:]), ref) < 1e-2
    assert cat[..., :Cout].abs().max().item() == 0


@pytest.mark.parametrize("N,h,w,Cin,Cout,strided", [(2, 5, 7, 64, 32, False), (1, 8, 8, 128, 64, False),
                                                     (3, 16, 20, 64, 32, True), (2, 33, 31, 128, 64, False)])
def test_deconv_bwd_fused(hip_lib, N, h, w, Cin, Cout, strided):
    """One-pass transposed-conv backward (csrc/deconv.hip): ReLU-masked dgrad + weight/bias grads."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(6)
    x = _bf(torch.randn(N, Cin, h, w)).relu()
    gup = _bf(torch.randn(N, Cout, 2 * h, 2 * w))
    wt = torch.randn(Cin, Cout, 2, 2) / Cin ** 0.5
    xr = x.clone().requires_grad_(True)
    wr = _bf(wt).clone().requires_grad_(True)
    br = torch.zeros(Cout, requires_grad=True)
    F.conv_transpose2d(xr, wr, br, stride=2).backward(gup)
    wd, _, _ = _pack_one(3, wt)
    if strided:   # gradient read from a concat half
        buf = torch.zeros(N, 2 * h, 2 * w, 2 * Cout, dtype=torch.bfloat16, device="cuda")
        buf[..., Cout:] = _nhwc(gup)
        g_in = buf[..., Cout:]
    else:
        g_in = _nhwc(gup)
    gw = torch.full((Cin, Cout, 2, 2), 0.5, device="cuda")
    gb = torch.full((Cout,), 0.5, device="cuda")
    dx = K.deconv_bwd_fused(g_in, _nhwc(x), wd, gw.view(-1), gb)
    torch.cuda.synchronize()
    assert _rel(_nchw(dx), xr.grad * (x > 0)) < 1e-2
    assert _rel(gw.cpu() - 0.5, wr.grad) < 1e-2
    assert _rel(gb.cpu() - 0.5, br.grad) < 1e-2
    # x a BatchNorm+ReLU output: the same dx, plus sum dx and sum dx*x per input channel from the epilogue
    stats = []
    dx2 = K.deconv_bwd_fused(g_in, _nhwc(x), wd, torch.zeros_like(gw).view(-1), torch.zeros_like(gb), bn_stats=stats)
    torch.cuda.synchronize()
    assert torch.equal(dx2, dx) and stats
    slab, rows = stats
    sums = slab.view(rows, 2, Cin).double().sum(0).cpu()
    dd, xd = dx.double().cpu().reshape(-1, Cin), _nhwc(x).double().cpu().reshape(-1, Cin)
    assert _rel(sums[0], dd.sum(0)) < 1e-4 and _rel(sums[1], (dd * xd).sum(0)) < 1e-4


@pytest.mark.parametrize("N,h,w,Cin,Cout", [(2, 5, 7, 64, 32), (2, 33, 31, 128, 64)])
def test_deconv_bn_on_load(hip_lib, N, h, w, Cin, Cout):
    """Transposed conv forward / fused backward reading a BatchNorm input z with relu(bn(z)) formed on load
    == the same kernels over the BN output materialised by bn_fwd, bit for bit (incl. the BN sums)."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(8)
    z = (torch.randn(N, h, w, Cin, device="cuda") * 1.4 - 0.2).to(torch.bfloat16)
    bn = torch.nn.BatchNorm2d(Cin).cuda()
    with torch.no_grad():
        bn.weight.uniform_(-1.0, 1.5)          # negative scales too
        bn.bias.uniform_(-0.5, 0.5)
    y = torch.empty_like(z)
    coef = []
    K.bn_fwd(z, y, bn, train=True, coef_out=coef)
    coef = coef[0]
    wt = torch.randn(Cin, Cout, 2, 2) / Cin ** 0.5
    wf, _, _ = _pack_one(2, wt)
    wd, _, _ = _pack_one(3, wt)
    b = torch.randn(Cout).cuda()
    outs = []
    for src, xbn in ((y, None), (z, coef)):
        cat = torch.zeros(N, 2 * h, 2 * w, 2 * Cout, dtype=torch.bfloat16, device="cuda")
        K.deconv_fwd_fused(src, wf, b, cat[..., Cout:], xbn=xbn)
        gup = torch.randn(N, 2 * h, 2 * w, Cout, generator=torch.Generator().manual_seed(3)).cuda().to(torch.bfloat16)
        gw = torch.zeros(Cin * Cout * 4, device="cuda")
        gb = torch.zeros(Cout, device="cuda")
        stats = []
        dx = K.deconv_bwd_fused(gup, src, wd, gw, gb, bn_stats=stats, xbn=xbn)
        torch.cuda.synchronize()
        outs.append((cat, dx, gw, gb, stats[0][:stats[1] * 2 * Cin]))
    for a, c in zip(*outs):
        assert torch.equal(a, c)


@pytest.mark.parametrize("N,H,W,C", [(2, 16, 16, 32), (1, 9, 11, 64)])
def test_maxpool_and_backward(hip_lib, N, H, W, C):
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(6)
    s = _bf(F.relu(torch.randn(N, C, H, W)))
    cat = torch.zeros(N, H, W, 2 * C, dtype=torch.bfloat16, device="cuda")
    cat[..., :C] = _nhwc(s)
    pooled = torch.empty(N, H // 2, W // 2, C, dtype=torch.bfloat16, device="cuda")
    K.maxpool2(cat[..., :C], pooled)
    sr = s.clone().requires_grad_(True)
    pr = F.max_pool2d(sr, 2, 2)
    assert _rel(_nchw(pooled), pr.detach()) == 0.0
    dpool = _bf(torch.randn_like(pr))
    dskip = _bf(torch.randn(N, C, H, W))
    pr.backward(dpool)
    ref = (sr.grad + dskip) * (s > 0)
    dcat = torch.zeros(N, H, W, 2 * C, dtype=torch.bfloat16, device="cuda")
    dcat[..., :C] = _nhwc(dskip)
    g = torch.empty(N, H, W, C, dtype=torch.bfloat16, device="cuda")
    K.pool_bwd(cat[..., :C], dcat[..., :C], _nhwc(dpool), g)
    torch.cuda.synchronize()
    assert _rel(_nchw(g), ref) < 1e-2


def test_head_loss_fwd_bwd(hip_lib):
    from distributedpytorch_amd.ops import kernels as K
    from distributedpytorch_amd.loss import bce_dice_from_probs
    torch.manual_seed(7)
    N, H, W, C = 2, 33, 40, 32
    y = _bf(F.relu(torch.randn(N, C, H, W)))
    w = torch.randn(1, C, 1, 1) * 0.2
    b = torch.randn(1) * 0.1
    t = (torch.rand(N, 1, H, W) > 0.6).float()
    yr, wr, br = y.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    loss = bce_dice_from_probs(torch.sigmoid(F.conv2d(yr, wr, br)), t)
    (3.0 * loss).backward()
    wc, bc, tc = w.cuda(), b.cuda(), t.cuda().contiguous()
    S, probs = K.head_fwd(_nhwc(y), wc, bc, tc, want_probs=True)
    n = t.numel()
    Sc = S.detach().clone().requires_grad_(True)
    loss_k = Sc[0] / n - torch.log(2 * Sc[1] / (Sc[2] + Sc[3] + 1e-15))
    (3.0 * loss_k).backward()
    assert abs(loss_k.item() - loss.item()) < 1e-4 * max(1.0, abs(loss.item()))
    gw = torch.zeros(C, device="cuda")
    gb = torch.zeros(1, device="cuda")
    gy = K.head_bwd(_nhwc(y), wc, bc, tc, Sc.grad, gw, gb)
    torch.cuda.synchronize()
    assert _rel(gw.cpu(), wr.grad.view(-1)) < 1e-3
    assert _rel(gb.cpu(), br.grad) < 1e-3
    assert _rel(_nchw(gy), yr.grad * (y > 0)) < 1e-2
    assert _rel(probs.cpu(), torch.sigmoid(F.conv2d(y, w, b))[:, 0]) < 1e-5
    # with a BatchNorm before the head: the same gy, plus the BN backward's partial sums of the stored gy
    stats = []
    gy2 = K.head_bwd(_nhwc(y), wc, bc, tc, Sc.grad, torch.zeros(C, device="cuda"), torch.zeros(1, device="cuda"),
                     bn_stats=stats)
    torch.cuda.synchronize()
    assert torch.equal(gy2, gy) and stats
    slab, rows = stats
    sums = slab.view(rows, 2, C).double().sum(0).cpu()
    g64, y64 = gy.double().cpu().reshape(-1, C), _nhwc(y).double().cpu().reshape(-1, C)
    assert _rel(sums[0], g64.sum(0)) < 1e-4 and _rel(sums[1], (g64 * y64).sum(0)) < 1e-4
    # the head reading the BN input z with y = relu(bn(z)) formed on load (forward and backward)
    z = _bf(torch.randn(N, C, H, W))
    coef = torch.cat([torch.rand(C) + 0.5, torch.randn(C) * 0.3]).cuda()
    yz = _bf(F.relu(z * coef[:C].cpu().view(1, C, 1, 1) + coef[C:].cpu().view(1, C, 1, 1)))
    Sy, _ = K.head_fwd(_nhwc(yz), wc, bc, tc)
    Sz, _ = K.head_fwd(_nhwc(z), wc, bc, tc, coef=coef)
    torch.cuda.synchronize()
    assert _rel(Sz.cpu(), Sy.cpu()) < 1e-4
    sy, sz = [], []
    gyy = K.head_bwd(_nhwc(yz), wc, bc, tc, Sc.grad, torch.zeros(C, device="cuda"), torch.zeros(1, device="cuda"),
                     bn_stats=sy)
    gwz, gbz = torch.zeros(C, device="cuda"), torch.zeros(1, device="cuda")
    gyz = K.head_bwd(_nhwc(z), wc, bc, tc, Sc.grad, gwz, gbz, bn_stats=sz, coef=coef)
    torch.cuda.synchronize()
    assert _rel(_nchw(gyz), _nchw(gyy)) < 1e-3
    a0 = sy[0].view(sy[1], 2, C).double().sum(0)
    a1 = sz[0].view(sz[1], 2, C).double().sum(0)
    assert _rel(a1.cpu(), a0.cpu()) < 1e-3


def test_input_conversion(hip_lib):
    from distributedpytorch_amd.ops import kernels as K
    x = torch.rand(2, 3, 7, 9)
    y = K.input_nhwc8(x.cuda())
    torch.cuda.synchronize()
    assert tuple(y.shape) == (2, 7, 9, 8)
    assert (y[..., 3:] == 0).all()
    assert _rel(_nchw(y[..., :3].contiguous()), _bf(x)) == 0.0


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 34, 128, 32, 32), (1, 9, 128, 64, 64), (1, 6, 256, 32, 64),
                                          (1, 6, 96, 32, 32), (2, 5, 240, 64, 64)])     # ragged rows
def test_conv_fused_maxpool(hip_lib, N, H, W, Cin, Cout):
    """Encoder conv2 writes its output into the concat buffer AND its 2x2 max-pool in one pass."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(8)
    x = _bf(torch.randn(N, Cin, H, W))
    w = _bf(torch.randn(Cout, Cin, 3, 3) * (2.0 / (9 * Cin)) ** 0.5)
    b = torch.randn(Cout) * 0.1
    packed, ng, kp = _pack_one(0, w)
    cat = torch.zeros(N, H, W, 2 * Cout, dtype=torch.bfloat16, device="cuda")
    pooled = torch.empty(N, H // 2, W // 2, Cout, dtype=torch.bfloat16, device="cuda")
    K.igemm(_nhwc(x), packed, cat[..., :Cout], Ngemm=ng, Kpad=kp, KH=3, KW=3, stride=1, pad=1, Cs=Cin,
            out_grid=(N, H, W), bias=b.cuda(), relu=True, pool=pooled)
    torch.cuda.synchronize()
    y = _nchw(cat[..., :Cout])
    assert _rel(y, F.relu(F.conv2d(x, w, b, padding=1))) < 2e-2
    assert torch.equal(_nchw(pooled), F.max_pool2d(y, 2, 2))      # pool of the stored values, exactly


@pytest.mark.parametrize("dice", [True, False])
def test_loss_from_partials_kernel(hip_lib, dice):
    """Fused loss tail (csrc/unet_aux.hip loss_finish/loss_grad) == the torch formula, value and grad."""
    from distributedpytorch_amd.ops import kernels as K
    from distributedpytorch_amd.loss import EPS
    S0 = torch.tensor([1234.5, 321.25, 800.0, 600.0], dtype=torch.float32)
    n = 4096
    a = S0.clone().cuda().requires_grad_(True)
    la = K.loss_from_partials(a, n, dice)
    (la * 3.0).backward()
    b = S0.clone().requires_grad_(True)
    lb = b[0] / n
    if dice:
        lb = lb - torch.log(2 * b[1] / (b[2] + b[3] + EPS))
    (lb * 3.0).backward()
    torch.testing.assert_close(la.cpu(), lb, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(a.grad.cpu(), b.grad, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("N,H,W,C,fused", [(2, 6, 128, 32, True), (1, 8, 256, 64, True), (2, 10, 14, 32, False),
                                           (1, 16, 16, 128, False)])
def test_pool_codes_backward(hip_lib, N, H, W, C, fused):
    """Window codes (argmax + ReLU masks) written by the fused streaming-conv pool epilogue or by
    maxpool2 drive pool_bwd_code to the same gradient as the value-based pool_bwd (incl. ties)."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(9)
    x = _bf(F.relu(torch.randn(N, C, H, W)))
    w = _bf(torch.randn(C, C, 3, 3) * (2.0 / (9 * C)) ** 0.5)
    b = torch.randn(C) * 0.1
    packed, ng, kp = _pack_one(0, w, C)
    cat = torch.zeros(N, H, W, 2 * C, dtype=torch.bfloat16, device="cuda")
    pooled = torch.empty(N, H // 2, W // 2, C, dtype=torch.bfloat16, device="cuda")
    code = torch.empty(N, H // 2, W // 2, C, dtype=torch.uint8, device="cuda")
    K.igemm(_nhwc(x), packed, cat[..., :C], Ngemm=ng, Kpad=kp, KH=3, KW=3, stride=1, pad=1, Cs=C,
            out_grid=(N, H, W), bias=b.cuda(), relu=True, pool=pooled, pcode=code, path="stream" if fused else "auto")
    skip = cat[..., :C]
    skip[:, 0, 0, :4] = skip[:, 0, 1, :4]          # force ties inside a window
    skip[:, 1, 0, 4:8] = 0
    K.maxpool2(skip, pooled, code)                 # codes of the edited values
    dpool = torch.randn(N, H // 2, W // 2, C, device="cuda").to(torch.bfloat16)
    dskip = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
    g_ref = torch.empty(N, H, W, C, dtype=torch.bfloat16, device="cuda")
    K.pool_bwd(skip, dskip, dpool, g_ref)
    g = torch.empty_like(g_ref)
    K.pool_bwd_code(code, dskip, dpool, g)
    torch.cuda.synchronize()
    assert torch.equal(g, g_ref)
    # with a BatchNorm behind the pooled tensor: the same g, plus sum g and sum g*skip per channel
    stats = []
    g2 = torch.empty_like(g_ref)
    K.pool_bwd_code(code, dskip, dpool, g2, y=skip, bn_stats=stats)
    torch.cuda.synchronize()
    assert torch.equal(g2, g_ref) and stats
    slab, rows = stats
    sums = slab.view(rows, 2, C).double().sum(0).cpu()
    gd, yd = g2.double().cpu().reshape(-1, C), skip.double().cpu().reshape(-1, C)
    assert _rel(sums[0], gd.sum(0)) < 1e-4 and _rel(sums[1], (gd * yd).sum(0)) < 1e-4
    # the sums against y = relu(bn(z)) re-formed on load from a dense z
    z = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
    coef = torch.cat([torch.rand(C) + 0.5, torch.randn(C) * 0.3]).cuda()
    yz = torch.relu(z.float() * coef[:C] + coef[C:]).to(torch.bfloat16)
    sz = []
    g3 = torch.empty_like(g_ref)
    K.pool_bwd_code(code, dskip, dpool, g3, y=z, bn_stats=sz, coef=coef)
    torch.cuda.synchronize()
    assert torch.equal(g3, g_ref) and sz
    sums = sz[0].view(sz[1], 2, C).double().sum(0).cpu()
    yd = yz.double().cpu().reshape(-1, C)
    assert _rel(sums[0], gd.sum(0)) < 1e-4 and _rel(sums[1], (gd * yd).sum(0)) < 1e-3


def test_stream_pool_codes_match_maxpool(hip_lib):
    """Codes from the fused streaming epilogue == codes from maxpool2 on the stored conv output."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(10)
    N, H, W, C = 2, 6, 128, 32
    x = _bf(F.relu(torch.randn(N, C, H, W)))
    w = _bf(torch.randn(C, C, 3, 3) * (2.0 / (9 * C)) ** 0.5)
    packed, ng, kp = _pack_one(0, w, C)
    y = torch.empty(N, H, W, C, dtype=torch.bfloat16, device="cuda")
    pooled = torch.empty(N, H // 2, W // 2, C, dtype=torch.bfloat16, device="cuda")
    code = torch.empty(N, H // 2, W // 2, C, dtype=torch.uint8, device="cuda")
    K.igemm(_nhwc(x), packed, y, Ngemm=ng, Kpad=kp, KH=3, KW=3, stride=1, pad=1, Cs=C, out_grid=(N, H, W),
            bias=(torch.randn(C) * 0.1).cuda(), relu=True, pool=pooled, pcode=code, path="stream")
    p2, c2 = torch.empty_like(pooled), torch.empty_like(code)
    K.maxpool2(y, p2, c2)
    torch.cuda.synchronize()
    assert torch.equal(pooled, p2) and torch.equal(code, c2)


@pytest.mark.parametrize("N,H,W,Cin,Cout,path", [(2, 3, 256, 64, 32, "stream"), (1, 4, 128, 128, 64, "halo"),
                                                 (2, 9, 13, 256, 128, "glds"), (2, 9, 13, 128, 64, "generic"),
                                                 (2, 3, 96, 64, 32, "stream"), (1, 4, 240, 128, 64, "halo"),
                                                 # >= 512 tiles of 256 x 256: the ping-pong kernel's split epilogue,
                                                 # with a partial last pixel tile
                                                 (10, 115, 117, 256, 128, "glds")])
def test_dgrad_split_output(hip_lib, N, H, W, Cin, Cout, path):
    """Split output (concat gradient as two dense tensors) == the interleaved output's halves."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(11)
    w = _bf(torch.randn(Cout, Cin, 3, 3) * 0.05)
    g = torch.randn(N, H, W, Cout, device="cuda").to(torch.bfloat16)
    packed, ng, kp = _pack_one(1, w)
    full = torch.empty(N, H, W, Cin, dtype=torch.bfloat16, device="cuda")
    kw = dict(Ngemm=ng, Kpad=kp, KH=3, KW=3, stride=1, pad=1, Cs=Cout, out_grid=(N, H, W), path=path)
    K.igemm(g, packed, full, **kw)
    s = Cin // 2
    lo = torch.empty(N, H, W, s, dtype=torch.bfloat16, device="cuda")
    hi = torch.empty(N, H, W, Cin - s, dtype=torch.bfloat16, device="cuda")
    K.igemm(g, packed, lo, y2=hi, split=s, **kw)
    torch.cuda.synchronize()
    assert torch.equal(lo, full[..., :s]) and torch.equal(hi, full[..., s:])


@pytest.mark.parametrize("N,H,W", [(2, 7, 128), (1, 33, 256), (2, 5, 96), (1, 3, 960)])
def test_stream_conv_fused_head(hip_lib, N, H, W):
    """Last decoder conv with the segmentation head + loss partial sums in its epilogue == conv, then
    the separate head kernel on the stored output (same bf16 values)."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(8)
    x = _nhwc(_bf(torch.randn(N, 32, H, W)).relu())
    w = torch.randn(32, 32, 3, 3) / 17
    wf, _, _ = _pack_one(0, w)
    b = (torch.randn(32) * 0.1).cuda()
    hw = (torch.randn(32) * 0.3).cuda()
    hb = torch.tensor([0.1], device="cuda")
    t = (torch.rand(N * H * W, device="cuda") > 0.5).float()
    y = torch.empty(N, H, W, 32, dtype=torch.bfloat16, device="cuda")
    hprob = torch.full((N * H * W,), -1.0, device="cuda")
    S = K.igemm(x, wf, y, Ngemm=32, Kpad=K.round_up(9 * 32, 32), KH=3, KW=3, stride=1, pad=1, Cs=32,
                out_grid=(N, H, W), bias=b, relu=True, head=(hw, hb, t, hprob))
    y2 = torch.empty_like(y)
    K.igemm(x, wf, y2, Ngemm=32, Kpad=K.round_up(9 * 32, 32), KH=3, KW=3, stride=1, pad=1, Cs=32,
            out_grid=(N, H, W), bias=b, relu=True, path="stream")
    S_ref, _ = K.head_fwd(y2, hw, hb, t)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
    assert torch.allclose(S, S_ref, rtol=1e-4, atol=1e-2), (S, S_ref)
    # the stored probabilities (read by the fused head backward) = sigmoid of the head logit of y
    p_ref = torch.sigmoid(y.float().reshape(-1, 32) @ hw + hb)
    assert (hprob - p_ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("N,H,W,Cin,Cout,hcfg", [
    (2, 5, 128, 64, 128, 4), (1, 4, 128, 128, 64, 4), (2, 3, 128, 32, 64, 5), (1, 7, 256, 256, 128, 4),
    (2, 5, 128, 64, 128, 2), (2, 5, 128, 64, 128, 6), (1, 3, 128, 128, 128, 7), (2, 4, 256, 128, 256, 6),
    (2, 5, 128, 64, 128, 8), (1, 4, 128, 128, 64, 8), (2, 3, 128, 32, 64, 9), (1, 7, 256, 256, 128, 8),
    (1, 3, 128, 128, 128, 10), (2, 5, 256, 32, 32, 9), (2, 5, 128, 128, 64, 11), (1, 5, 128, 64, 64, 12),
    (1, 7, 256, 128, 64, 13), (2, 6, 128, 64, 128, 13), (1, 3, 256, 128, 64, 14)])
def test_conv3x3_halo_two_rows(hip_lib, N, H, W, Cin, Cout, hcfg):
    """Row-halo conv with two (three, four) output rows per block (one weight staging per slice for all;
    heights not a multiple -> the last block's extra rows are masked): forward with bias+ReLU and masked dgrad."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(9)
    x = _bf(F.relu(torch.randn(N, Cin, H, W)))
    w = _bf(torch.randn(Cout, Cin, 3, 3) * (2.0 / (9 * Cin)) ** 0.5)
    b = torch.randn(Cout) * 0.1
    ref = F.relu(F.conv2d(x, w, b, padding=1))
    packed, ng, kp = _pack_one(0, w)
    y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device="cuda")
    K.igemm(_nhwc(x), packed, y, Ngemm=ng, Kpad=kp, KH=3, KW=3, stride=1, pad=1, Cs=Cin, out_grid=(N, H, W),
            bias=b.cuda(), relu=True, path="halo", variant=hcfg)
    g = _bf(torch.randn(N, Cout, H, W))
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, w, padding=1).backward(g)
    packed_d, ngd, kpd = _pack_one(1, w)
    dx = torch.empty(N, H, W, Cin, dtype=torch.bfloat16, device="cuda")
    bc = {2: 64, 4: 64, 5: 32, 6: 128, 7: 128, 8: 64, 9: 32, 10: 128, 11: 64, 12: 64, 13: 64, 14: 64}[hcfg]   # output-channel tile
    if Cin % bc == 0:
        K.igemm(_nhwc(g), packed_d, dx, Ngemm=ngd, Kpad=kpd, KH=3, KW=3, stride=1, pad=1, Cs=Cout,
                out_grid=(N, H, W), mask=_nhwc(x), path="halo", variant=hcfg)
    torch.cuda.synchronize()
    assert _rel(_nchw(y), ref) < 2e-2
    if Cin % bc == 0:
        assert _rel(_nchw(dx), xr.grad * (x > 0)) < 2e-2


@pytest.mark.parametrize("path", ["stream", "halo", "wgrad"])
def test_per_image_launch_beyond_2gib(hip_lib, path):
    """The row-streaming / row-halo kernels bind one image per block (64-bit image base, 32-bit
    offsets inside it), so a batch whose activations exceed the 2 GiB buffer range runs as ONE
    launch: the images past 2 GiB must equal the same images run as a small batch."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(12)
    if path == "halo":
        N, H, W, Cin, Cout = 132, 128, 512, 128, 64       # x: 2.2 GB
    else:
        N, H, W, Cin, Cout = 132, 256, 512, 64, 32        # x: 2.2 GB (concat-sized input)
    x = torch.randn(N, H, W, Cin, device="cuda").to(torch.bfloat16)
    assert x.numel() * 2 > 2 ** 31
    w = torch.randn(Cout, Cin, 3, 3) * (2.0 / (9 * Cin)) ** 0.5
    if path == "wgrad":
        g = torch.randn(N, H, W, Cout, device="cuda").to(torch.bfloat16)
        gw = torch.zeros(Cout * Cin * 9, device="cuda")
        K.wgrad(g, x, kind=0, grid=(N, H, W), M=Cout, Nc=Cin, s=1, pad=1, KW=3, gw=gw, gb=None, Nreal=Cin, path="stream")
        tail = slice(N - 3, N)
        gw2 = torch.zeros_like(gw)
        K.wgrad(g[tail].contiguous(), x[tail].contiguous(), kind=0, grid=(3, H, W), M=Cout, Nc=Cin, s=1, pad=1, KW=3,
                gw=gw2, gb=None, Nreal=Cin, path="stream")
        gw3 = torch.zeros_like(gw)
        K.wgrad(g[:N - 3].contiguous(), x[:N - 3].contiguous(), kind=0, grid=(N - 3, H, W), M=Cout, Nc=Cin, s=1,
                pad=1, KW=3, gw=gw3, gb=None, Nreal=Cin, path="stream")
        torch.cuda.synchronize()
        assert _rel(gw, gw2 + gw3) < 1e-3
        return
    packed, ng, kp = _pack_one(0, w)
    y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device="cuda")
    kw = dict(Ngemm=ng, Kpad=kp, KH=3, KW=3, stride=1, pad=1, Cs=Cin, relu=True, path=path)
    K.igemm(x, packed, y, out_grid=(N, H, W), **kw)
    tail = x[N - 2:].contiguous()
    y2 = torch.empty(2, H, W, Cout, dtype=torch.bfloat16, device="cuda")
    K.igemm(tail, packed, y2, out_grid=(2, H, W), **kw)
    torch.cuda.synchronize()
    assert torch.equal(y[N - 2:], y2)


@pytest.mark.parametrize("blocks", [1, 7, 100000])
def test_wgrad_gemm_image_groups(hip_lib, blocks):
    """csrc/wgrad_gemm.hip with 1 .. N images per split (the split-K slabs over image groups, K-steps
    crossing image boundaries, a short last group) against the fp32 reference."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(17)
    N, H, W, Cin, Cout = 5, 4, 64, 256, 256
    x = _bf(torch.randn(N, Cin, H, W))
    g = _bf(torch.randn(N, Cout, H, W))
    wr = torch.zeros(Cout, Cin, 3, 3, requires_grad=True)
    br = torch.zeros(Cout, requires_grad=True)
    F.conv2d(x, wr, br, padding=1).backward(g)
    gw = torch.zeros(Cout * Cin * 9, device="cuda")
    gb = torch.zeros(Cout, device="cuda")
    K._wgrad_gemm(_nhwc(g), _nhwc(x), grid=(N, H, W), M=Cout, Nc=Cin, gw=gw, gb=gb, Nreal=Cin, blocks=blocks)
    torch.cuda.synchronize()
    assert _rel(gw.cpu().view(Cout, Cin, 3, 3), wr.grad) < 1e-2, blocks
    assert _rel(gb.cpu(), br.grad) < 1e-2, blocks


@pytest.mark.parametrize("N,H,W,Cin,Cout,ips", [
    (8, 64, 64, 256, 256, 0), (8, 64, 64, 512, 256, 3), (8, 64, 64, 128, 256, 8), (16, 32, 32, 512, 512, 0),
    (16, 32, 32, 256, 512, 5), (5, 32, 32, 64, 256, 1)])
def test_wgrad_band_real_shapes(hip_lib, N, H, W, Cin, Cout, ips):
    """csrc/wgrad_band.hip at the UNet's deep-layer shapes (64^2 x 128/256/512 -> 256, 32^2 -> 512) and image
    groups of 1 .. N (ragged last split): fp32-anchored -- torch fp32 conv2d backward on the same bf16
    operands; and equal (fp32 summation-order level) to the dense-GEMM path it replaces."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(23)
    x = torch.randn(N, Cin, H, W, device="cuda").to(torch.bfloat16)
    g = torch.randn(N, Cout, H, W, device="cuda").to(torch.bfloat16)
    # fp32 reference as 9 shifted fp32 GEMMs (no MIOpen algorithm search at these sizes)
    xh, gh = x.permute(0, 2, 3, 1).contiguous(), g.permute(0, 2, 3, 1).contiguous()
    xp = F.pad(xh.float(), (0, 0, 1, 1, 1, 1))
    g2 = gh.float().reshape(-1, Cout).t()
    ref = torch.stack([g2 @ xp[:, kh:kh + H, kw:kw + W].reshape(-1, Cin) for kh in range(3) for kw in range(3)], -1)
    ref = ref.view(Cout, Cin, 3, 3)
    bref = g2.sum(1)
    gw = torch.zeros(Cout * Cin * 9, device="cuda")
    gb = torch.zeros(Cout, device="cuda")
    K._wgrad_band(gh, xh, grid=(N, H, W), M=Cout, Nc=Cin, gw=gw, gb=gb, Nreal=Cin, ips=ips)
    gw2 = torch.zeros(Cout * Cin * 9, device="cuda")
    gb2 = torch.zeros(Cout, device="cuda")
    K._wgrad_gemm(gh, xh, grid=(N, H, W), M=Cout, Nc=Cin, gw=gw2, gb=gb2, Nreal=Cin)
    torch.cuda.synchronize()
    assert _rel(gw.view(Cout, Cin, 3, 3), ref) < 1e-4
    assert _rel(gb, bref) < 1e-4
    assert _rel(gw, gw2) < 1e-5 and _rel(gb, gb2) < 1e-5


@pytest.mark.parametrize("N,H,W,Cin,Cout,steps", [
    (8, 128, 128, 64, 128, 0), (8, 128, 128, 128, 128, 16), (8, 128, 128, 256, 128, 256), (3, 128, 128, 128, 128, 96),
    (4, 64, 64, 128, 128, 0), (2, 256, 256, 64, 128, 0)])
def test_wgrad_band128_real_shapes(hip_lib, N, H, W, Cin, Cout, steps):
    """csrc/wgrad_band.hip's 128-channel kernel at the UNet's 128^2 layer shapes (64/128/256 -> 128) with
    splits of whole images, of part of an image (16 K-steps = 8 rows) and straddling images (96 K-steps of
    256): fp32-anchored (nine shifted fp32 GEMMs on the same bf16 operands)."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(29)
    x = torch.randn(N, Cin, H, W, device="cuda").to(torch.bfloat16)
    g = torch.randn(N, Cout, H, W, device="cuda").to(torch.bfloat16)
    xh, gh = x.permute(0, 2, 3, 1).contiguous(), g.permute(0, 2, 3, 1).contiguous()
    xp = F.pad(xh.float(), (0, 0, 1, 1, 1, 1))
    g2 = gh.float().reshape(-1, Cout).t()
    ref = torch.stack([g2 @ xp[:, kh:kh + H, kw:kw + W].reshape(-1, Cin) for kh in range(3) for kw in range(3)], -1)
    gw = torch.zeros(Cout * Cin * 9, device="cuda")
    gb = torch.zeros(Cout, device="cuda")
    K._wgrad_band128(gh, xh, grid=(N, H, W), M=Cout, Nc=Cin, gw=gw, gb=gb, Nreal=Cin, steps=steps)
    torch.cuda.synchronize()
    assert _rel(gw.view(Cout, Cin, 9), ref) < 1e-4
    assert _rel(gb, g2.sum(1)) < 1e-4


@pytest.mark.parametrize("M,Nc,H,W,mb,nmb", [(256, 256, 4, 64, 3, 3), (256, 128, 3, 32, 2, 4), (512, 64, 2, 64, 4, 2),
                                             (128, 64, 3, 64, 2, 3)])
def test_wgrad_multi_microbatches(hip_lib, M, Nc, H, W, mb, nmb):
    """One weight-gradient launch over the images of several microbatch tensors (per-image pointer
    tables; a pipeline stage's deferred weight gradients): dense-GEMM path for M % 256 == 0, row kernels
    otherwise -- equal to the fp32 reference over the concatenated batch."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(19)
    xs = [_bf(torch.randn(mb, Nc, H, W)) for _ in range(nmb)]
    gs = [_bf(torch.randn(mb, M, H, W)) for _ in range(nmb)]
    wr = torch.zeros(M, Nc, 3, 3, requires_grad=True)
    br = torch.zeros(M, requires_grad=True)
    F.conv2d(torch.cat(xs), wr, br, padding=1).backward(torch.cat(gs))
    gw = torch.zeros(M * Nc * 9, device="cuda")
    gb = torch.zeros(M, device="cuda")
    # separate allocations (not views of one tensor): the tables must carry each tensor's own base
    K.wgrad_multi([_nhwc(g).clone() for g in gs], [_nhwc(x).clone() for x in xs], M=M, Nc=Nc, gw=gw, gb=gb, Nreal=Nc)
    torch.cuda.synchronize()
    assert _rel(gw.cpu().view(M, Nc, 3, 3), wr.grad) < 1e-2
    assert _rel(gb.cpu(), br.grad) < 1e-2


@pytest.mark.parametrize("N,H,W,Cs,Ng,kind", [(9, 64, 64, 256, 256, "fwd"), (5, 61, 67, 128, 512, "fwd"),
                                               (9, 64, 64, 256, 256, "dgrad"), (5, 61, 67, 512, 256, "dgrad"),
                                               # row-block tiles of 8 / 2 / 1 image rows (W = 32 / 128 / 256)
                                               (16, 32, 32, 128, 256, "fwd"), (3, 30, 128, 64, 256, "dgrad"),
                                               (2, 70, 256, 64, 256, "fwd"),
                                               # tiles = half / third of a row (W = 512 / 768)
                                               (2, 9, 512, 64, 256, "dgrad"), (1, 5, 768, 128, 256, "fwd")])
def test_glds_pingpong_epilogues(hip_lib, N, H, W, Cs, Ng, kind):
    """The ping-pong deep GEMM (cfg 14; on whole-row tiles its row-block pixel staging form, 8206 = cfg 14
    without row blocks) with its specialised epilogues (forward bias + ReLU, dgrad ReLU mask; partial
    last pixel tile): both forms accumulate K in the same order -> bitwise equal (fp32 anchors of the
    same kernels: tests/test_rowblock.py)."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(23)
    x = torch.randn(N, H, W, Cs, device="cuda").to(torch.bfloat16)
    Kp = 9 * Cs
    w = (torch.randn(Ng, Kp, device="cuda") / Kp ** 0.5).to(torch.bfloat16)
    extra = (dict(bias=torch.randn(Ng, device="cuda") * 0.1, relu=True) if kind == "fwd" else
             dict(mask=torch.randn(N, H, W, Ng, device="cuda").to(torch.bfloat16)))
    outs = []
    for v in (14, 8206):
        y = torch.empty(N, H, W, Ng, device="cuda", dtype=torch.bfloat16)
        K.igemm(x, w, y, Ngemm=Ng, Kpad=Kp, KH=3, KW=3, stride=1, pad=1, Cs=Cs, out_grid=(N, H, W), path="glds",
                variant=v, **extra)
        outs.append(y)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("N,H,W,Cs,Ng,kind", [(4, 128, 128, 128, 128, "fwd"), (3, 30, 256, 64, 128, "dgrad"),
                                               (2, 64, 64, 256, 384, "fwd"), (8, 32, 32, 64, 128, "dgrad"),
                                               (2, 9, 512, 128, 128, "fwd"), (1, 5, 768, 64, 128, "dgrad")])
def test_glds_rowblock_128(hip_lib, N, H, W, Cs, Ng, kind):
    """The 128-channel row-block kernel (cfg 15) with its specialised and generic (cfg 15 + 2048)
    epilogues: bitwise equal to each other; it and the 128x256 3-stage kernel (cfg 2) each match the fp32
    convolution of the same bf16 operands (their K orders may differ, so no cross-kernel escape)."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(29)
    x = torch.randn(N, H, W, Cs, device="cuda").to(torch.bfloat16)
    Kp = 9 * Cs
    w = (torch.randn(Ng, Kp, device="cuda") / Kp ** 0.5).to(torch.bfloat16)
    extra = (dict(bias=torch.randn(Ng, device="cuda") * 0.1, relu=True) if kind == "fwd" else
             dict(mask=torch.randn(N, H, W, Ng, device="cuda").to(torch.bfloat16)))
    outs = []
    for v in (2, 15, 2048 + 15):
        y = torch.empty(N, H, W, Ng, device="cuda", dtype=torch.bfloat16)
        K.igemm(x, w, y, Ngemm=Ng, Kpad=Kp, KH=3, KW=3, stride=1, pad=1, Cs=Cs, out_grid=(N, H, W), path="glds",
                variant=v, **extra)
        outs.append(y)
    torch.cuda.synchronize()
    assert torch.equal(outs[1], outs[2])
    # cfg 2 and cfg 15 may sum K in different orders: each is anchored to the fp32 convolution of the same
    # bf16 operands (packed k = tap * Cs + ci) instead of to the other kernel
    import torch.nn.functional as F
    wconv = w.float().cpu().view(Ng, 9, Cs).permute(0, 2, 1).reshape(Ng, Cs, 3, 3)
    ref = F.conv2d(x.float().cpu().permute(0, 3, 1, 2), wconv, padding=1).permute(0, 2, 3, 1)
    ref = (torch.relu(ref + extra["bias"].cpu()) if kind == "fwd" else ref * (extra["mask"].float().cpu() > 0))
    for v, y in zip((2, 15), outs[:2]):
        assert _rel(y.float().cpu(), ref) < 1e-2, (v, kind)


@pytest.mark.parametrize("splits,T,M,Nc,Nreal", [(3000, 9, 32, 8, 3), (1500, 9, 32, 32, 32), (40, 9, 32, 8, 8)])
def test_wgrad_reduce_many_splits(hip_lib, splits, T, M, Nc, Nreal):
    """Split-K slab reduction into the OIHW gradient (accumulating), including the in-place presum stage
    taken for thousands of splits over a small weight: == the fp64 sum of the slab rows."""
    from ctypes import c_int
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(3)
    slab = torch.randn(splits, T, M, Nc, device="cuda")
    bslab = torch.randn(splits, M, device="cuda")
    ref_w = slab.double().sum(0)[..., :Nreal].permute(1, 2, 0).cpu()          # [M][Nreal][T]
    ref_b = bslab.double().sum(0).cpu()
    gw = torch.ones(M * Nreal * T, device="cuda")
    gb = torch.ones(M, device="cuda")
    K._check(K._lib.lib().dpa_wgrad_reduce(K._p(slab), K._p(bslab), K._p(gw), K._p(gb), c_int(splits), c_int(T), c_int(M),
                                           c_int(Nc), c_int(Nreal), c_int(0), K._stream(gw)), "wgrad_reduce")
    torch.cuda.synchronize()
    assert _rel(gw.cpu().double().view(M, Nreal, T) - 1.0, ref_w) < 1e-5
    assert _rel(gb.cpu().double() - 1.0, ref_b) < 1e-5


@pytest.mark.parametrize("N,h,w,Cin,Cout,half", [(64, 32, 32, 256, 128, True), (16, 16, 64, 512, 256, False),
                                                  (128, 16, 16, 256, 64, True), (8, 8, 32, 1024, 512, False)])
def test_wgrad_up_matches_split_k(hip_lib, N, h, w, Cin, Cout, half):
    """Transposed-conv weight + bias gradient on the dense GEMM (wgrad_gemm.hip up mode: x as the A operand,
    the gradient as a 4-tap B operand at (2h + i, 2w + j), no padding; bias from dpa_chan_sum_bf16) equals the
    split-K kernel's (cfg 14) up to fp32 summation order, with the gradient a concat half (ld = 2 Cout) or dense."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(11)
    x = torch.randn(N, h, w, Cin, device="cuda").to(torch.bfloat16)
    full = torch.randn(N, 2 * h, 2 * w, 2 * Cout if half else Cout, device="cuda").to(torch.bfloat16)
    g = full[..., Cout:] if half else full
    assert K.wgrad_up_eligible(Cout, Cin, (N, h, w))
    outs = []
    for cfg in (0, 14):
        gw = torch.randn(Cin * Cout * 4, device="cuda")          # accumulates: start from the same values
        gb = torch.randn(Cout, device="cuda")
        gw0, gb0 = gw.clone(), gb.clone()
        K.wgrad(g, x, kind=1, grid=(N, h, w), M=Cout, Nc=Cin, s=2, pad=0, KW=2, gw=gw, gb=gb, Nreal=Cin, cfg=cfg)
        torch.cuda.synchronize()
        outs.append((gw - gw0, gb - gb0))
    (dw, db), (rw, rb) = outs
    ref = torch.einsum("nhwc,nhiwjo->coij", x.float(), g.float().view(N, h, 2, w, 2, Cout)).reshape(-1)
    assert ((dw - ref).abs().max() / ref.abs().max()).item() < 1e-4
    assert ((dw - rw).abs().max() / rw.abs().max()).item() < 1e-4
    assert ((db - rb).abs().max() / rb.abs().max()).item() < 1e-4
