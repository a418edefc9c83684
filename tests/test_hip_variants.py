"""HIP kernels and engine parity for the north-star UNet variants: DoubleConv = Conv2d + BatchNorm +
ReLU and the bilinear Up path (csrc/norm_up.hip, 1x1 projection through igemm / wgrad kind 2),
each against a plain PyTorch fp32 reference of the same op."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def _bf(t):
    return t.to(torch.bfloat16).float()


def _cos(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-30)).item()


@pytest.mark.parametrize("N,H,W,C", [(2, 9, 13, 32), (3, 16, 16, 64), (1, 8, 8, 256), (2, 5, 7, 8), (1, 4, 4, 1024)])
def test_bn_forward_train_and_eval(hip_lib, N, H, W, C):
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(0)
    z = _bf(torch.randn(N, H, W, C) * 2 + 0.5)
    bn_ref = torch.nn.BatchNorm2d(C)
    with torch.no_grad():
        bn_ref.weight.uniform_(0.5, 1.5)
        bn_ref.bias.uniform_(-0.5, 0.5)
    bn = torch.nn.BatchNorm2d(C).cuda()
    bn.load_state_dict(bn_ref.state_dict())
    # wider output tensor: y written into a channel slice (concat half)
    ybuf = torch.zeros(N, H, W, 2 * C, dtype=torch.bfloat16, device="cuda")
    y = ybuf[..., C:]
    saved = K.bn_fwd(z.cuda().to(torch.bfloat16), y, bn, train=True)
    y_ref = F.relu(bn_ref(z.permute(0, 3, 1, 2))).permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    assert _rel(y.float(), y_ref) < 1e-2
    assert ybuf[..., :C].abs().max().item() == 0
    assert torch.allclose(bn.running_mean.cpu(), bn_ref.running_mean, atol=1e-4, rtol=1e-4)
    assert torch.allclose(bn.running_var.cpu(), bn_ref.running_var, atol=1e-4, rtol=1e-3)
    assert int(bn.num_batches_tracked) == int(bn_ref.num_batches_tracked) == 1
    mean = z.reshape(-1, C).mean(0)
    assert torch.allclose(saved[:C].cpu(), mean, atol=1e-4)
    # eval: running statistics
    bn_ref.eval()
    y2 = torch.empty(N, H, W, C, dtype=torch.bfloat16, device="cuda")
    assert K.bn_fwd(z.cuda().to(torch.bfloat16), y2, bn, train=False) is None
    y2_ref = F.relu(bn_ref(z.permute(0, 3, 1, 2))).permute(0, 2, 3, 1)
    assert _rel(y2.float(), y2_ref) < 1e-2


@pytest.mark.parametrize("N,H,W,C", [(2, 9, 13, 32), (3, 16, 16, 64), (1, 8, 8, 512)])
def test_bn_backward(hip_lib, N, H, W, C):
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(1)
    z = _bf(torch.randn(N, H, W, C) * 1.5 - 0.3)
    g = _bf(torch.randn(N, H, W, C))
    bn_ref = torch.nn.BatchNorm2d(C)
    with torch.no_grad():
        bn_ref.weight.uniform_(0.5, 1.5)
        bn_ref.bias.uniform_(-0.5, 0.5)
    bn = torch.nn.BatchNorm2d(C).cuda()
    bn.load_state_dict(bn_ref.state_dict())
    zr = z.permute(0, 3, 1, 2).clone().requires_grad_(True)
    out = bn_ref(zr)                       # gradient w.r.t. the BN output (pre-ReLU) = g
    out.backward(g.permute(0, 3, 1, 2))
    zc = z.cuda().to(torch.bfloat16)
    y = torch.empty_like(zc)
    saved = K.bn_fwd(zc, y, bn, train=True, relu=False)
    dgamma = torch.zeros(C, device="cuda")
    dbeta = torch.full((C,), 0.25, device="cuda")   # accumulates
    dz = K.bn_bwd(g.cuda().to(torch.bfloat16), zc, saved, bn, dgamma, dbeta)
    torch.cuda.synchronize()
    assert _rel(dz.float().permute(0, 3, 1, 2), zr.grad) < 2e-2
    assert _rel(dgamma, bn_ref.weight.grad) < 1e-3
    assert _rel(dbeta - 0.25, bn_ref.bias.grad) < 1e-3


@pytest.mark.parametrize("N,h,w,C", [(2, 4, 6, 32), (1, 7, 5, 64), (3, 16, 16, 8), (1, 1, 3, 16)])
def test_upsample2x_bilinear(hip_lib, N, h, w, C):
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(2)
    x = _bf(torch.randn(N, C, h, w))
    ref = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)
    buf = torch.zeros(N, 2 * h, 2 * w, 2 * C, dtype=torch.bfloat16, device="cuda")
    K.up2_fwd(x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16), buf[..., C:])
    torch.cuda.synchronize()
    assert _rel(buf[..., C:].float().permute(0, 3, 1, 2), ref) < 1e-2
    # backward (adjoint): gather formulation vs autograd of the interpolation
    g = _bf(torch.randn(N, C, 2 * h, 2 * w))
    xr = x.clone().requires_grad_(True)
    F.interpolate(xr, scale_factor=2, mode="bilinear", align_corners=False).backward(g)
    dx = K.up2_bwd(g.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16))
    torch.cuda.synchronize()
    assert _rel(dx.float().permute(0, 3, 1, 2), xr.grad) < 1e-2


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 8, 12, 64, 32), (1, 16, 16, 128, 64), (2, 4, 4, 512, 256)])
def test_conv1x1_fwd_dgrad_wgrad(hip_lib, N, H, W, Cin, Cout):
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(3)
    x = _bf(torch.randn(N, Cin, H, W)).relu()
    w = torch.randn(Cout, Cin, 1, 1) / Cin ** 0.5
    b = torch.randn(Cout) * 0.1
    flat = w.reshape(-1).cuda().contiguous()

    def pack(mode, ngemm, kpad):
        d = K.PackDesc(flat.data_ptr(), 0, mode, Cout, Cin, Cin if mode == 4 else Cout, ngemm, kpad)
        descs = torch.frombuffer(bytearray(bytes(d)), dtype=torch.uint8).cuda()
        packed = torch.empty(ngemm * kpad, dtype=torch.bfloat16, device="cuda")
        K.pack_weights(packed, descs, 1, ngemm * kpad)
        return packed

    kf, kd = K.round_up(Cin, 32), K.round_up(Cout, 32)
    xh = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device="cuda")
    K.igemm(xh, pack(4, Cout, kf), y, Ngemm=Cout, Kpad=kf, KH=1, KW=1, stride=1, pad=0, Cs=Cin, out_grid=(N, H, W),
            bias=b.cuda())
    y_ref = F.conv2d(x, _bf(w), b)
    torch.cuda.synchronize()
    assert _rel(y.float().permute(0, 3, 1, 2), y_ref) < 1e-2
    # dgrad with the ReLU mask of x, wgrad (kind 2) + bias grad
    g = _bf(torch.randn(N, Cout, H, W))
    gh = g.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    dx = torch.empty(N, H, W, Cin, dtype=torch.bfloat16, device="cuda")
    K.igemm(gh, pack(5, Cin, kd), dx, Ngemm=Cin, Kpad=kd, KH=1, KW=1, stride=1, pad=0, Cs=Cout, out_grid=(N, H, W),
            mask=xh)
    xr = x.clone().requires_grad_(True)
    wr = _bf(w).clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    F.conv2d(xr, wr, br).backward(g)
    gw = torch.zeros(Cout * Cin, device="cuda")
    gb = torch.zeros(Cout, device="cuda")
    K.wgrad(gh, xh, kind=2, grid=(N, H, W), M=Cout, Nc=Cin, s=1, pad=0, KW=1, gw=gw, gb=gb, Nreal=Cin)
    torch.cuda.synchronize()
    assert _rel(dx.float().permute(0, 3, 1, 2), xr.grad * (x > 0)) < 1e-2
    assert _rel(gw.view(Cout, Cin, 1, 1), wr.grad) < 1e-2
    assert _rel(gb, br.grad) < 1e-2


@pytest.mark.parametrize("variant", ["bn", "bilinear", "bn+bilinear"])
def test_hip_unet_variants_match_torch_fp32(hip_lib, variant):
    """Whole engine (BN / bilinear variants) vs the reference-semantics UNet on fp32 CPU, training
    mode (batch statistics), then the eval-mode probability map (running statistics).

    BatchNorm's backward (g - mean(g) - xhat*mean(g*xhat)) amplifies bf16 rounding of the deep,
    small-batch layers, so the bar is set per parameter by stock PyTorch bf16 autocast on the same
    GPU (MIOpen convs): per parameter within 0.03 cosine of it, and on average as close."""
    from distributedpytorch_amd.compute import loss_from_partials, make_compute
    from distributedpytorch_amd.loss import bce_dice_from_probs
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.optim import FlatParameterSpace
    from distributedpytorch_amd.data.synthetic import synthetic_batch

    kw = {"batchnorm": "bn" in variant, "bilinear": "bilinear" in variant}
    torch.manual_seed(0)
    ref = build_model("unet", **kw)
    hip = build_model("unet", **kw)
    stock = build_model("unet", **kw)
    hip.load_state_dict(ref.state_dict())
    stock.load_state_dict(ref.state_dict())
    img, mask = synthetic_batch(4, 64, 64, 3, seed=5)
    t = mask.float().unsqueeze(1)
    loss_ref = bce_dice_from_probs(ref(img), t)
    (4 * loss_ref).backward()

    stock = stock.cuda()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        p_stock = stock(img.cuda())
    (4 * bce_dice_from_probs(p_stock.float(), t.cuda())).backward()

    hip = hip.cuda()
    FlatParameterSpace(hip)
    comp = make_compute(hip, backend="hip", dtype="bf16")
    S = comp.forward_partials(img.cuda(), t.cuda())
    loss = loss_from_partials(S, t.numel())
    (4 * loss).backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - loss_ref.item()) < 1e-2 * abs(loss_ref.item()), (loss.item(), loss_ref.item())
    cs, cs_st = [], []
    for (n, p_ref), (_, p), (_, p_st) in zip(ref.named_parameters(), hip.named_parameters(), stock.named_parameters()):
        g_ref, g = p_ref.grad, p.grad.cpu()
        if kw["batchnorm"] and n.endswith("bias") and (".conv_block.0." in n or ".conv_block.3." in n):
            continue   # conv bias right before BatchNorm: its exact gradient is 0 (rounding noise only)
        c, c_st = _cos(g, g_ref), _cos(p_st.grad.cpu(), g_ref)
        cs.append(c)
        cs_st.append(c_st)
        assert c > min(0.97, c_st - 0.03), f"{n}: cosine {c:.4f} (stock bf16 {c_st:.4f})"
        r = (g.norm() / g_ref.norm()).item()
        assert 0.9 < r < 1.1, f"{n}: norm ratio {r:.4f}"
    # on average at least as close to fp32 as stock bf16
    assert sum(cs) / len(cs) >= sum(cs_st) / len(cs_st) - 0.005, (sum(cs) / len(cs), sum(cs_st) / len(cs_st))
    for (n, b_ref), (_, b) in zip(ref.named_buffers(), hip.named_buffers()):
        if b_ref.is_floating_point():
            assert torch.allclose(b.cpu(), b_ref, rtol=2e-2, atol=2e-3), n
    ref.eval()
    hip.eval()
    with torch.no_grad():
        p_ref = ref(img)
        p = comp.probs(img.cuda()).cpu()
    assert (p - p_ref).abs().max().item() < 5e-2


@pytest.mark.parametrize("N,H,W", [(2, 40, 256), (1, 33, 200)])
def test_first_conv_bn_stats_in_stream8_epilogue(hip_lib, N, H, W):
    """The first conv (RGB padded to 8 channels, igemm_stream8_kernel) followed by BatchNorm: its epilogue
    writes the batch sums (sum z, sum z^2 of the stored bf16 output, ragged last strip masked) -- they
    equal the fp64 sums over the z it wrote, and the output equals the plain launch bitwise."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(5)
    x8 = torch.zeros(N, H, W, 8)
    x8[..., :3] = torch.rand(N, H, W, 3)
    xh = x8.to(torch.bfloat16).cuda()
    packed = (torch.randn(32, 96) * 0.2)
    packed[:, 72:] = 0
    packed = packed.to(torch.bfloat16).cuda().reshape(-1)
    b = (torch.randn(32) * 0.1).cuda()
    z0 = torch.empty(N, H, W, 32, dtype=torch.bfloat16, device="cuda")
    K.igemm(xh, packed, z0, Ngemm=32, Kpad=96, KH=3, KW=3, stride=1, pad=1, Cs=8, out_grid=(N, H, W), bias=b, relu=False)
    z1 = torch.empty_like(z0)
    stats = []
    K.igemm(xh, packed, z1, Ngemm=32, Kpad=96, KH=3, KW=3, stride=1, pad=1, Cs=8, out_grid=(N, H, W), bias=b, relu=False,
            bn_stats=stats)
    torch.cuda.synchronize()
    assert torch.equal(z0, z1) and len(stats) == 2
    slab, rows = stats
    sums = slab[:rows * 64].view(rows, 2, 32).double().sum(0).cpu()
    zd = z1.double().reshape(-1, 32).cpu()
    assert _rel(sums[0], zd.sum(0)) < 1e-5 and _rel(sums[1], (zd * zd).sum(0)) < 1e-5


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 5, 128, 32, 32), (1, 7, 64, 64, 32), (2, 6, 128, 32, 64),
                                            (1, 33, 64, 64, 64),
                                            # deep layers: the row-block GEMM's epilogue (256 / 128 channels)
                                            (2, 16, 64, 128, 256), (1, 8, 128, 64, 128), (1, 2, 512, 128, 128)])
def test_conv_bn_stats_fused_in_stream_epilogue(hip_lib, N, H, W, Cin, Cout):
    """Conv followed by BatchNorm on the streaming kernel: the batch statistics come from the conv's
    epilogue (per-block channel sums of the stored bf16 output) instead of a separate pass.  Output,
    saved mean/invstd and running statistics equal the unfused path and match torch fp32."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(3)
    x = _bf(torch.randn(N, Cin, H, W))
    w = _bf(torch.randn(Cout, Cin, 3, 3) * (2.0 / (9 * Cin)) ** 0.5)
    b = torch.randn(Cout) * 0.1
    bn_ref = torch.nn.BatchNorm2d(Cout)
    with torch.no_grad():
        bn_ref.weight.uniform_(0.5, 1.5)
        bn_ref.bias.uniform_(-0.5, 0.5)
    kf = K.round_up(9 * Cin, 32)
    packed = torch.zeros(Cout, kf)
    packed[:, :9 * Cin] = w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin)
    packed = packed.to(torch.bfloat16).cuda().reshape(-1)
    xh = x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).cuda()
    outs = []
    for fused in (True, False):
        bn = torch.nn.BatchNorm2d(Cout).cuda()
        bn.load_state_dict(bn_ref.state_dict())
        z = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device="cuda")
        stats = [] if fused else None
        K.igemm(xh, packed, z, Ngemm=Cout, Kpad=kf, KH=3, KW=3, stride=1, pad=1, Cs=Cin, out_grid=(N, H, W),
                bias=b.cuda(), relu=False, bn_stats=stats)
        if fused:
            assert len(stats) == 2 and stats[1] > 0, "streaming epilogue did not produce the statistics"
        y = torch.empty_like(z)
        saved = K.bn_fwd(z, y, bn, train=True, stats=stats)
        torch.cuda.synchronize()
        # each path's statistics are exact for the z it produced (fp64 reference over that z)
        zd = z.double().reshape(-1, Cout).cpu()
        mean, var = zd.mean(0), zd.var(0, unbiased=False)
        assert torch.allclose(saved.cpu()[:Cout].double(), mean, rtol=1e-5, atol=1e-6)
        assert torch.allclose(saved.cpu()[Cout:].double(), (var + bn.eps).rsqrt(), rtol=1e-3, atol=1e-6)
        outs.append((y.float().cpu(), saved.cpu(), bn.running_mean.cpu(), bn.running_var.cpu(), float(zd.abs().max())))
    (y1, s1, m1, v1, _), (y0, s0, m0, v0, zmax) = outs
    # the fused and unfused paths may run different conv kernels (accumulation order): their z are at most
    # bf16 rounding flips apart, which move a mean over few pixels by ~ulp(|z|) / P
    tol = 2.0 ** -7 * zmax / (N * H * W) * 4
    assert _rel(y1, y0) < 1e-2
    assert torch.allclose(s1, s0, rtol=1e-3, atol=tol) and torch.allclose(m1, m0, rtol=1e-3, atol=tol)
    assert torch.allclose(v1, v0, rtol=1e-3, atol=tol)
    y_ref = F.relu(bn_ref(F.conv2d(x, w, b, padding=1))).permute(0, 2, 3, 1)
    assert _rel(y1, y_ref) < 3e-2


@pytest.mark.parametrize("N,H,W,C", [(2, 6, 10, 32), (1, 16, 16, 64), (2, 5, 8, 32)])
def test_bn_apply_fused_maxpool(hip_lib, N, H, W, C):
    """BN+ReLU and the encoder's 2x2 max-pool (+ window codes) in one pass == BN pass then max-pool
    pass, bitwise (odd H falls back to the separate pool)."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(4)
    z = (torch.randn(N, H, W, C) * 2).to(torch.bfloat16).cuda()
    res = []
    for fused in (True, False):
        bn = torch.nn.BatchNorm2d(C).cuda()
        with torch.no_grad():
            bn.weight.copy_(torch.linspace(0.5, 1.5, C))
            bn.bias.copy_(torch.linspace(-0.5, 0.5, C))
        y = torch.empty_like(z)
        pool = torch.empty(N, H // 2, W // 2, C, dtype=torch.bfloat16, device="cuda")
        code = torch.empty(N, H // 2, W // 2, C, dtype=torch.uint8, device="cuda")
        if fused:
            K.bn_fwd(z, y, bn, train=True, pool=pool, pcode=code)
        else:
            K.bn_fwd(z, y, bn, train=True)
            K.maxpool2(y, pool, code)
        torch.cuda.synchronize()
        res.append((y.cpu(), pool.cpu(), code.cpu()))
    for a, b in zip(*res):
        assert torch.equal(a, b)
    ref = F.max_pool2d(res[0][0].float().permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
    assert torch.equal(res[0][1].float(), ref)


@pytest.mark.parametrize("N,H,W,C1,C2", [(2, 5, 128, 32, 32), (1, 6, 64, 64, 64), (2, 3, 128, 32, 64),
                                         (1, 4, 128, 64, 32),
                                         # deep layers: the row-block GEMM's epilogue (256 / 128 channels)
                                         (1, 8, 64, 256, 128), (2, 4, 64, 128, 256)])
def test_bn_backward_partials_fused_in_stream_dgrad(hip_lib, N, H, W, C1, C2):
    """The dgrad into a BN layer's output y = relu(bn(z)) (ReLU mask y) also writes sum g, sum g*y per
    channel from its epilogue; bn_bwd then skips its reduction pass (sum g*xhat = (sum g*y - beta
    sum g) / gamma on the mask's support).  dz, dgamma, dbeta match the unfused path."""
    from distributedpytorch_amd.ops import kernels as K
    from test_hip_kernels import _pack_one
    torch.manual_seed(6)
    z = (torch.randn(N, H, W, C1) * 1.5 + 0.2).to(torch.bfloat16).cuda()
    w2 = torch.randn(C2, C1, 3, 3) * (2.0 / (9 * C1)) ** 0.5
    g2 = torch.randn(N, H, W, C2).to(torch.bfloat16).cuda()
    packed, ng, kp = _pack_one(1, w2)
    res = []
    for fused in (True, False):
        bn = torch.nn.BatchNorm2d(C1).cuda()
        with torch.no_grad():
            bn.weight.copy_(torch.linspace(0.6, 1.4, C1))
            bn.bias.copy_(torch.linspace(-0.3, 0.3, C1))
        y = torch.empty_like(z)
        saved = K.bn_fwd(z, y, bn, train=True)
        g1 = torch.empty(N, H, W, C1, dtype=torch.bfloat16, device="cuda")
        stats = [] if fused else None
        K.igemm(g2, packed, g1, Ngemm=ng, Kpad=kp, KH=3, KW=3, stride=1, pad=1, Cs=C2, out_grid=(N, H, W),
                mask=y, bn_stats=stats)
        if fused:
            assert len(stats) == 2 and stats[1] > 0, "dgrad epilogue did not produce the BN partials"
        dgam, dbet = torch.zeros(C1, device="cuda"), torch.zeros(C1, device="cuda")
        dz = K.bn_bwd(g1, z, saved, bn, dgam, dbet, stats=stats)
        torch.cuda.synchronize()
        res.append((g1.float().cpu(), dz.float().cpu(), dgam.cpu(), dbet.cpu()))
    (g1a, dza, dga, dba), (g1b, dzb, dgb, dbb) = res
    assert torch.equal(g1a, g1b)
    assert torch.allclose(dba, dbb, rtol=1e-5, atol=1e-4)
    assert torch.allclose(dga, dgb, rtol=2e-2, atol=2e-2 * dgb.abs().max().item())
    assert _rel(dza, dzb) < 2e-2


def test_eval_bn_folded_into_conv(hip_lib, monkeypatch):
    """Inference of the BN DoubleConv model: with running statistics, BatchNorm folds into the conv
    (one fused conv+bias+ReLU(+pool) kernel per layer).  Probabilities match the unfolded HIP path and
    the torch fp32 model in eval mode."""
    from distributedpytorch_amd.compute import make_compute
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(2)
    ref = build_model("unet-bn")
    with torch.no_grad():
        for m in ref.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 2.0)
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.3, 0.3)
    ref.eval()
    hip = build_model("unet-bn")
    hip.load_state_dict(ref.state_dict())
    hip = hip.cuda().eval()
    comp = make_compute(hip, backend="hip", dtype="bf16")
    x = torch.rand(2, 3, 64, 128)
    with torch.no_grad():
        p_ref = ref(x)
        p_fold = comp.probs(x.cuda()).cpu()
        monkeypatch.setattr(K, "FOLD_BN_EVAL", False)
        p_unfold = comp.probs(x.cuda()).cpu()
    assert (p_fold - p_ref).abs().max().item() < 3e-2
    assert (p_fold - p_unfold).abs().max().item() < 2e-2


def test_eval_bn_fold_cache_follows_running_stats(hip_lib, monkeypatch):
    """The folded eval weights are cached; a training-mode forward (running statistics move) and a
    load_state_dict (in-place writes) must both invalidate them."""
    from distributedpytorch_amd.compute import make_compute
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(3)
    model = build_model("unet-bn").cuda()
    comp = make_compute(model, backend="hip", dtype="bf16")
    x = torch.rand(2, 3, 64, 128, device="cuda")
    t = (torch.rand(2, 1, 64, 128, device="cuda") > 0.5).float()

    def both():
        with torch.no_grad():
            monkeypatch.setattr(K, "FOLD_BN_EVAL", True)
            a = comp.probs(x).cpu()
            monkeypatch.setattr(K, "FOLD_BN_EVAL", False)
            b = comp.probs(x).cpu()
        return (a - b).abs().max().item()

    model.eval()
    assert both() < 2e-2                       # fills the cache
    model.train()
    with torch.no_grad():
        comp.forward_partials(x * 3.0 + 1.0, t)   # shifts every BN layer's running statistics
    model.eval()
    assert both() < 2e-2
    sd = {k: (v * 1.5 if k.endswith("running_var") else v) for k, v in model.state_dict().items()}
    model.load_state_dict(sd)
    assert both() < 2e-2
