"""Fused conv3x3 backward (csrc/bwd_stream.hip): input gradient + weight gradient + bias gradient of
one conv in a single row-streaming pass, against the fp32 PyTorch reference of the same op
(autograd of ``F.conv2d``), for every (Cin, Cout) pair it serves and each epilogue: dx masked by the
input's ReLU support, dx split into the two halves of a concat gradient, dx plain.  The weight /
bias gradients accumulate into the flat fp32 buffer (existing content is kept)."""
import pytest
import torch
import torch.nn.functional as F

from test_hip_kernels import _bf, _nchw, _nhwc, _pack_one, _rel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,H,W,Cin,Cout,epi", [
    (2, 5, 64, 32, 32, "mask"), (1, 37, 128, 32, 32, "mask"), (2, 3, 64, 32, 32, "plain"),
    (2, 6, 64, 64, 32, "split"), (1, 9, 128, 64, 32, "mask"),
    (2, 4, 64, 32, 64, "plain"), (1, 7, 192, 32, 64, "mask"),
    (2, 5, 64, 64, 64, "mask"), (1, 3, 128, 64, 64, "split"),
    # ragged last strip (640x960 level widths 480 / 240): out-of-row pixels masked
    (1, 5, 480, 64, 64, "mask"), (2, 4, 120, 32, 64, "plain"), (1, 3, 240, 64, 32, "split"), (2, 3, 60, 32, 32, "mask"),
])
def test_conv_bwd_fused_matches_torch(hip_lib, N, H, W, Cin, Cout, epi):
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(7)
    x = _bf(F.relu(torch.randn(N, Cin, H, W)))          # a ReLU output (mask source)
    w = _bf(torch.randn(Cout, Cin, 3, 3) * 0.05)
    g = _bf(torch.randn(N, Cout, H, W))
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = torch.zeros(Cout, requires_grad=True)
    F.conv2d(xr, wr, br, padding=1).backward(g)
    dx_ref = xr.grad * (x > 0) if epi == "mask" else xr.grad
    packed, ng, kd = _pack_one(1, w)
    gw0 = torch.randn(Cout * Cin * 9, device="cuda")   # accumulate semantics
    gb0 = torch.randn(Cout, device="cuda")
    gw, gb = gw0.clone(), gb0.clone()
    if epi == "split":
        s = Cin // 2
        dx, dx2 = K.conv_bwd_fused(_nhwc(g), _nhwc(x), packed, kd, gw, gb, mask=False,
                                   dx2=torch.empty(N, H, W, Cin - s, dtype=torch.bfloat16, device="cuda"), split=s)
        full = torch.cat([_nchw(dx), _nchw(dx2)], dim=1)
    else:
        full = _nchw(K.conv_bwd_fused(_nhwc(g), _nhwc(x), packed, kd, gw, gb, mask=epi == "mask"))
    torch.cuda.synchronize()
    assert _rel(full, dx_ref) < 2e-2
    # weight / bias gradients: bf16 inputs, fp32 accumulation -> only summation order differs
    assert _rel((gw - gw0).cpu(), wr.grad.reshape(-1)) < 1e-4
    assert _rel((gb - gb0).cpu(), br.grad) < 1e-4


def test_conv_bwd_fused_deterministic_and_matches_unfused(hip_lib):
    """Bitwise run-to-run reproducible (fixed-order slab reduction); agrees with the separate
    dgrad + weight-gradient kernels it replaces."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(8)
    N, H, W, C = 3, 16, 128, 32
    x = _nhwc(_bf(F.relu(torch.randn(N, C, H, W))))
    g = _nhwc(_bf(torch.randn(N, C, H, W)))
    w = _bf(torch.randn(C, C, 3, 3) * 0.05)
    packed, ng, kd = _pack_one(1, w)
    outs = []
    for _ in range(2):
        gw = torch.zeros(C * C * 9, device="cuda")
        gb = torch.zeros(C, device="cuda")
        dx = K.conv_bwd_fused(g, x, packed, kd, gw, gb, mask=True)
        outs.append((dx.clone(), gw, gb))
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
    dx_u = torch.empty_like(outs[0][0])
    K.igemm(g, packed, dx_u, Ngemm=ng, Kpad=kd, KH=3, KW=3, stride=1, pad=1, Cs=C, out_grid=(N, H, W), mask=x)
    gw_u = torch.zeros(C * C * 9, device="cuda")
    gb_u = torch.zeros(C, device="cuda")
    K.wgrad(g, x, kind=0, grid=(N, H, W), M=C, Nc=C, s=1, pad=1, KW=3, gw=gw_u, gb=gb_u, Nreal=C)
    torch.cuda.synchronize()
    assert torch.equal(dx_u, outs[0][0])           # same MFMA sequence per output element
    assert _rel(outs[0][1].cpu(), gw_u.cpu()) < 1e-5 and _rel(outs[0][2].cpu(), gb_u.cpu()) < 1e-5


@pytest.mark.parametrize("N,H,W", [(2, 5, 64), (1, 33, 128)])
def test_conv_bwd_fused_head_mode_matches_separate_head_bwd(hip_lib, N, H, W):
    """Head mode: the segmentation-head backward folded into the last decoder conv's fused backward
    (gradient formed from the conv output y and the forward's stored probabilities on load) equals
    head_bwd followed by the plain fused backward: dx, conv weight/bias gradients and segmap weight/bias
    gradients."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(9)
    C = 32
    a = _nhwc(_bf(F.relu(torch.randn(N, C, H, W))))              # conv input (ReLU output)
    y = _nhwc(_bf(F.relu(torch.randn(N, C, H, W))))              # conv output (ReLU output)
    t = (torch.rand(N * H * W, device="cuda") > 0.5).float()
    hw = (torch.randn(C) * 0.2).cuda()
    hb = torch.randn(1).cuda()
    dS = torch.tensor([1.0 / (N * H * W), -0.01, 0.002, 0.002], device="cuda")
    w = _bf(torch.randn(C, C, 3, 3) * 0.05)
    packed, ng, kd = _pack_one(1, w)
    # reference: separate head backward, then the fused conv backward on the stored gradient
    hgw_r, hgb_r = torch.zeros(C, device="cuda"), torch.zeros(1, device="cuda")
    gy = K.head_bwd(y, hw, hb, t, dS, hgw_r, hgb_r)
    gw_r, gb_r = torch.zeros(C * C * 9, device="cuda"), torch.zeros(C, device="cuda")
    dx_r = K.conv_bwd_fused(gy, a, packed, kd, gw_r, gb_r, mask=True)
    hgw, hgb = torch.zeros(C, device="cuda"), torch.zeros(1, device="cuda")
    gw, gb = torch.zeros(C * C * 9, device="cuda"), torch.zeros(C, device="cuda")
    # the probabilities the forward's fused head epilogue stores (sigmoid of the head logit of y)
    hprob = torch.sigmoid(y.float().reshape(-1, C) @ hw + hb).contiguous()
    dx = K.conv_bwd_fused(y, a, packed, kd, gw, gb, mask=True, head=(t, hw, hb, dS, hgw, hgb, hprob))
    torch.cuda.synchronize()
    assert _rel(dx.float().cpu(), dx_r.float().cpu()) < 1e-2
    assert _rel(gw.cpu(), gw_r.cpu()) < 1e-2 and _rel(gb.cpu(), gb_r.cpu()) < 1e-2
    assert _rel(hgw.cpu(), hgw_r.cpu()) < 1e-4 and _rel(hgb.cpu(), hgb_r.cpu()) < 1e-4


@pytest.mark.parametrize("N,H,W,with_skip", [(2, 6, 64, True), (1, 34, 128, True), (2, 4, 64, False)])
def test_conv_bwd_fused_pool_mode_matches_pool_bwd(hip_lib, N, H, W, with_skip):
    """Pool mode: the max-pool backward (window codes from the forward epilogue) folded into the
    encoder conv2's fused backward equals pool_bwd_code followed by the plain fused backward."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(10)
    C = 32
    a = _nhwc(_bf(F.relu(torch.randn(N, C, H, W))))              # conv input (ReLU output)
    w = _bf(torch.randn(C, C, 3, 3) * 0.05)
    packed_f, _, kf = _pack_one(0, w)
    packed, ng, kd = _pack_one(1, w)
    # forward with the fused pool: the skip (conv output), pooled output and window codes
    y = torch.empty(N, H, W, C, dtype=torch.bfloat16, device="cuda")
    pooled = torch.empty(N, H // 2, W // 2, C, dtype=torch.bfloat16, device="cuda")
    code = torch.empty(N, H // 2, W // 2, C, dtype=torch.uint8, device="cuda")
    K.igemm(a, packed_f, y, Ngemm=C, Kpad=kf, KH=3, KW=3, stride=1, pad=1, Cs=C, out_grid=(N, H, W),
            bias=torch.randn(C).cuda() * 0.1, relu=True, pool=pooled, pcode=code)
    dskip = _nhwc(_bf(torch.randn(N, C, H, W))) if with_skip else None
    dpool = _nhwc(_bf(torch.randn(N, C, H // 2, W // 2)))
    g2 = torch.empty(N, H, W, C, dtype=torch.bfloat16, device="cuda")
    K.pool_bwd_code(code, dskip, dpool, g2)
    gw_r, gb_r = torch.zeros(C * C * 9, device="cuda"), torch.zeros(C, device="cuda")
    dx_r = K.conv_bwd_fused(g2, a, packed, kd, gw_r, gb_r, mask=True)
    gw, gb = torch.zeros(C * C * 9, device="cuda"), torch.zeros(C, device="cuda")
    dx = K.conv_bwd_fused(dskip, a, packed, kd, gw, gb, mask=True, pool=(code, dpool))
    torch.cuda.synchronize()
    assert torch.equal(dx, dx_r)                 # identical gradient bits -> identical MFMA inputs
    assert torch.equal(gw, gw_r) and torch.equal(gb, gb_r)


@pytest.mark.parametrize("N,H,W", [(2, 6, 64), (1, 34, 128), (2, 4, 192)])
def test_conv_bwd_fused_first_level_matches_separate(hip_lib, N, H, W):
    """W1 mode (first encoder level): the pool-mode fused backward of conv2 also accumulates conv1's
    weight and bias gradients from its never-stored input gradient; equals the pool-mode backward
    returning that gradient followed by conv1's separate weight-gradient kernel."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(11)
    C, CR = 32, 3
    x1 = torch.zeros(N, H, W, 8, dtype=torch.bfloat16, device="cuda")
    x1[..., :CR] = torch.rand(N, H, W, CR, device="cuda").to(torch.bfloat16)   # padded 3-channel image
    a = _nhwc(_bf(F.relu(torch.randn(N, C, H, W))))              # conv1 output = conv2 input
    w = _bf(torch.randn(C, C, 3, 3) * 0.05)
    packed_f, _, kf = _pack_one(0, w)
    packed, ng, kd = _pack_one(1, w)
    y = torch.empty(N, H, W, C, dtype=torch.bfloat16, device="cuda")
    pooled = torch.empty(N, H // 2, W // 2, C, dtype=torch.bfloat16, device="cuda")
    code = torch.empty(N, H // 2, W // 2, C, dtype=torch.uint8, device="cuda")
    K.igemm(a, packed_f, y, Ngemm=C, Kpad=kf, KH=3, KW=3, stride=1, pad=1, Cs=C, out_grid=(N, H, W),
            bias=torch.randn(C).cuda() * 0.1, relu=True, pool=pooled, pcode=code)
    dskip = _nhwc(_bf(torch.randn(N, C, H, W)))
    dpool = _nhwc(_bf(torch.randn(N, C, H // 2, W // 2)))
    # reference: pool-mode fused backward returning g1, then conv1's weight gradient
    gw_r, gb_r = torch.zeros(C * C * 9, device="cuda"), torch.zeros(C, device="cuda")
    g1 = K.conv_bwd_fused(dskip, a, packed, kd, gw_r, gb_r, mask=True, pool=(code, dpool))
    gw1_r, gb1_r = torch.zeros(C * CR * 9, device="cuda"), torch.zeros(C, device="cuda")
    K.wgrad(g1, x1, kind=0, grid=(N, H, W), M=C, Nc=8, s=1, pad=1, KW=3, gw=gw1_r, gb=gb1_r, Nreal=CR)
    gw, gb = torch.zeros(C * C * 9, device="cuda"), torch.zeros(C, device="cuda")
    gw1, gb1 = torch.randn(C * CR * 9, device="cuda"), torch.randn(C, device="cuda")   # accumulate semantics
    gw10, gb10 = gw1.clone(), gb1.clone()
    out = K.conv_bwd_fused(dskip, a, packed, kd, gw, gb, mask=True, pool=(code, dpool), w1=(x1, gw1, gb1))
    torch.cuda.synchronize()
    assert out is None
    assert _rel(gw.cpu(), gw_r.cpu()) < 1e-5 and _rel(gb.cpu(), gb_r.cpu()) < 1e-5
    assert _rel((gw1 - gw10).cpu(), gw1_r.cpu()) < 1e-4, _rel((gw1 - gw10).cpu(), gw1_r.cpu())
    assert _rel((gb1 - gb10).cpu(), gb1_r.cpu()) < 1e-4
    # and against the fp32 autograd reference of conv1's weight gradient from the same g1
    x1n = x1[..., :CR].permute(0, 3, 1, 2).float().cpu().requires_grad_(False)
    w1r = torch.zeros(C, CR, 3, 3, requires_grad=True)
    F.conv2d(x1n, w1r, padding=1).backward(g1.permute(0, 3, 1, 2).float().cpu())
    assert _rel((gw1 - gw10).cpu(), w1r.grad.reshape(-1)) < 1e-4


@pytest.mark.parametrize("N,H,W,Cin,Cout,epi", [
    (2, 5, 64, 32, 32, "stats"), (1, 6, 128, 64, 64, "stats"), (2, 4, 64, 32, 64, "stats"), (1, 5, 64, 64, 32, "stats"),
    (2, 3, 64, 64, 32, "split"), (2, 4, 64, 32, 64, "plain"), (1, 5, 120, 64, 64, "stats"),
])
def test_conv_bwd_fused_batchnorm_modes(hip_lib, N, H, W, Cin, Cout, epi):
    """BatchNorm backward formed in the fused backward's loader (dz from the masked BN-output gradient
    and the BN input z) == bn_bwd's elementwise pass followed by the plain fused backward: the same
    bf16 dz, so dx and the weight / bias gradients agree exactly; dgamma / dbeta equal; with ``stats``
    the per-block (sum dx, sum dx*x) partials of the layer below's BatchNorm match torch sums of dx."""
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(11)
    z = (torch.randn(N, H, W, Cout) * 1.5 + 0.2).to(torch.bfloat16).cuda()
    x = _nhwc(_bf(F.relu(torch.randn(N, Cin, H, W))))
    w = _bf(torch.randn(Cout, Cin, 3, 3) * 0.05)
    packed, ng, kd = _pack_one(1, w)
    res = []
    for fused in (True, False):
        bn = torch.nn.BatchNorm2d(Cout).cuda()
        with torch.no_grad():
            bn.weight.copy_(torch.linspace(0.6, 1.4, Cout))
            bn.bias.copy_(torch.linspace(-0.3, 0.3, Cout))
        y = torch.empty_like(z)
        saved = K.bn_fwd(z, y, bn, train=True)
        torch.manual_seed(12)
        g = (torch.randn(N, H, W, Cout, device="cuda") * (y > 0)).to(torch.bfloat16)   # ReLU-masked
        dgam, dbet = torch.zeros(Cout, device="cuda"), torch.zeros(Cout, device="cuda")
        gw, gb = torch.zeros(Cout * Cin * 9, device="cuda"), torch.zeros(Cout, device="cuda")
        kw = dict(mask=epi == "stats")
        if epi == "split":
            kw.update(dx2=torch.empty(N, H, W, Cin - Cin // 2, dtype=torch.bfloat16, device="cuda"), split=Cin // 2)
        st = None
        if fused:
            coef = K.bn_bwd_coef(g, z, saved, bn, dgam, dbet)
            out = K.conv_bwd_fused(g, x, packed, kd, gw, gb, bn=(z, coef), bn_stats=epi == "stats", **kw)
            if epi == "stats":
                out, st = out
        else:
            dz = K.bn_bwd(g, z, saved, bn, dgam, dbet)
            out = K.conv_bwd_fused(dz, x, packed, kd, gw, gb, **kw)
        dx = torch.cat([out[0], out[1]], dim=3) if epi == "split" else out
        torch.cuda.synchronize()
        res.append((dx.float().cpu(), gw.cpu(), gb.cpu(), dgam.cpu(), dbet.cpu(), st))
    (dxa, gwa, gba, dga, dba, st), (dxb, gwb, gbb, dgb, dbb, _) = res
    assert torch.equal(dxa, dxb)
    assert torch.equal(gwa, gwb) and torch.equal(gba, gbb)
    assert torch.equal(dga, dgb) and torch.equal(dba, dbb)
    if epi == "stats":
        slab, rows = st
        sums = slab.view(rows, 2, Cin).sum(0).cpu()
        xs = x.float().cpu()
        assert _rel(sums[0], dxa.sum((0, 1, 2))) < 1e-3
        assert _rel(sums[1], (dxa * xs).sum((0, 1, 2))) < 1e-3


@pytest.mark.parametrize("sink", [True, False])
@pytest.mark.parametrize("chunks", [2, 4])
def test_first_level_backward_in_image_chunks(hip_lib, chunks, sink):
    """DPA_ENC0_CHUNKS: the first encoder level's fused (pool-folded) backward and the first conv's
    side-stream weight gradient run per image chunk; every gradient equals the one-launch backward up to
    fp32 summation order -- with the slab rows of all chunks reduced once per conv (kernels.SlabSink,
    DPA_NO_CHUNK_SINK=0) or per chunk."""
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.ops import kernels as K
    from distributedpytorch_amd.trainer import SingleDevice
    from distributedpytorch_amd.data.synthetic import synthetic_batch
    torch.manual_seed(0)
    model = build_model("unet")
    st = SingleDevice(TrainConfig(backend="hip", lr=1e-3), model, "cuda:0")
    img, mask = synthetic_batch(8, 128, 128, 3, seed=4)
    x, t = img.cuda(), mask.float().unsqueeze(1).cuda()
    grads = []
    old, old_sink = K.ENC0_CHUNKS, K.CHUNK_SINK
    K.CHUNK_SINK = sink
    try:
        for c in (1, chunks):
            K.ENC0_CHUNKS = c
            st.optimizer.zero_grad()
            (st.forward_loss(x, t) * 8).backward()
            torch.cuda.synchronize()
            grads.append(st.space.grad.detach().clone())
    finally:
        K.ENC0_CHUNKS, K.CHUNK_SINK = old, old_sink
    g0, g1 = grads
    for i, n in enumerate(st.space.names):
        o0, o1 = st.space.slice_of(i)
        a, b = g0[o0:o1].double(), g1[o0:o1].double()
        assert ((a - b).abs().max() / a.abs().max().clamp_min(1e-30)).item() < 1e-4, n
