"""The fp32 hand-written training path (csrc/fp32.hip, ops/fp32.py, models/hip_unet_f32.py) against
plain PyTorch fp32 references: every op forward and backward, and a whole reference-UNet training step
(loss, every parameter gradient).  fp32 MFMA products summed in a permuted K order: relative errors at
the 1e-5 level, not bitwise."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("N,H,W,Cin,Cout,cs", [(2, 16, 24, 32, 32, 32), (1, 9, 13, 64, 96, 64), (2, 8, 8, 3, 32, 4),
                                               (2, 32, 40, 128, 128, 128), (1, 20, 18, 64, 256, 64),
                                               (3, 12, 10, 96, 64, 96)])
def test_conv_relu_fwd_bwd(hip_lib, N, H, W, Cin, Cout, cs):
    from distributedpytorch_amd.models.hip_unet_f32 import _ConvReLU
    torch.manual_seed(Cin + Cout)
    xr = torch.randn(N, Cin, H, W, device="cuda")
    w = (torch.randn(Cout, Cin, 3, 3, device="cuda") / (9 * Cin) ** 0.5).requires_grad_(True)
    b = (torch.randn(Cout, device="cuda") * 0.1).requires_grad_(True)
    ref_x = xr.clone().requires_grad_(True)
    ref = torch.relu(F.conv2d(ref_x, w, b, padding=1))
    g = torch.randn_like(ref)
    gw_ref, gb_ref, gx_ref = torch.autograd.grad(ref, (w, b, ref_x), g)
    xn = torch.zeros(N, H, W, cs, device="cuda")
    xn[..., :Cin] = xr.permute(0, 2, 3, 1)
    xn.requires_grad_(True)
    y = _ConvReLU.apply(xn, w, b, cs)
    assert _rel(y.permute(0, 3, 1, 2), ref) < 1e-5
    gx, gw, gb = torch.autograd.grad(y, (xn, w, b), g.permute(0, 2, 3, 1).contiguous())
    assert _rel(gw, gw_ref) < 1e-5 and _rel(gb, gb_ref) < 1e-5
    assert _rel(gx[..., :Cin].permute(0, 3, 1, 2), gx_ref) < 1e-5


@pytest.mark.parametrize("N,h,w,Cin,Cout,C", [(2, 8, 12, 64, 32, 32), (1, 4, 4, 512, 256, 256)])
def test_up_cat(hip_lib, N, h, w, Cin, Cout, C):
    """[skip ‖ ConvTranspose2d(x)] in one buffer (deconv epilogue into the upper half) vs torch, forward and
    every gradient (the two gradient halves are read in place)."""
    from distributedpytorch_amd.models.hip_unet_f32 import _UpCat
    torch.manual_seed(Cin + C)
    x = torch.randn(N, Cin, h, w, device="cuda").requires_grad_(True)
    sk = torch.randn(N, C, 2 * h, 2 * w, device="cuda").requires_grad_(True)
    wt = (torch.randn(Cin, Cout, 2, 2, device="cuda") / Cin ** 0.5).requires_grad_(True)
    b = (torch.randn(Cout, device="cuda") * 0.1).requires_grad_(True)
    ref = torch.cat([sk, F.conv_transpose2d(x, wt, b, stride=2)], dim=1)
    g = torch.randn_like(ref)
    refs = torch.autograd.grad(ref, (x, sk, wt, b), g)
    xn = x.detach().permute(0, 2, 3, 1).contiguous().requires_grad_(True)
    skn = sk.detach().permute(0, 2, 3, 1).contiguous().requires_grad_(True)
    y = _UpCat.apply(xn, skn, wt, b)
    assert _rel(y.permute(0, 3, 1, 2), ref) < 1e-5
    gx, gsk, gw, gb = torch.autograd.grad(y, (xn, skn, wt, b), g.permute(0, 2, 3, 1).contiguous())
    assert _rel(gx.permute(0, 3, 1, 2), refs[0]) < 1e-5 and _rel(gsk.permute(0, 3, 1, 2), refs[1]) == 0.0
    assert _rel(gw, refs[2]) < 1e-5 and _rel(gb, refs[3]) < 1e-5


@pytest.mark.parametrize("N,H,W,C,strided", [(2, 6, 8, 32, True), (1, 7, 9, 64, False), (3, 4, 4, 4, True)])
def test_enc_out_bwd(hip_lib, N, H, W, C, strided):
    """(y > 0) * (skip grad + max-pool backward) in one pass vs autograd of relu -> (identity, max_pool2d)."""
    from distributedpytorch_amd.ops import fp32 as F32
    torch.manual_seed(N * H + C)
    z = torch.randn(N, C, H, W, device="cuda", requires_grad=True)
    y = torch.relu(z)
    p = F.max_pool2d(y, 2)
    gs = torch.randn_like(y)
    gp = torch.randn_like(p)
    (gz_ref,) = torch.autograd.grad((y, p), (z,), (gs, gp))
    yn = y.detach().permute(0, 2, 3, 1).contiguous()
    pn, code = F32.maxpool2(yn)
    assert _rel(pn.permute(0, 3, 1, 2), p) == 0.0
    gsn = gs.permute(0, 2, 3, 1).contiguous()
    if strided:       # the skip gradient as a channel slice of a wider buffer (cat backward)
        wide = torch.randn(N, H, W, 2 * C, device="cuda")
        wide[..., :C] = gsn
        gsn = wide[..., :C]
    ge = F32.enc_out_bwd(gsn, gp.permute(0, 2, 3, 1).contiguous(), code, yn)
    assert _rel(ge.permute(0, 3, 1, 2), gz_ref) < 1e-6


@pytest.mark.parametrize("N,H,W,Nc,M", [(2, 8, 64, 32, 32), (1, 6, 32, 64, 96), (3, 2, 96, 64, 64), (1, 4, 32, 32, 64)])
def test_wgrad_halo_form(hip_lib, N, H, W, Nc, M):
    """3x3 weight gradient with the input halo staged per 2 x 32-pixel patch (wgrad3_f32_kernel) and the
    generic tap-column form, both vs torch fp32 (weight and bias gradient)."""
    from distributedpytorch_amd.ops import fp32 as F32
    torch.manual_seed(Nc + M + H)
    x = torch.randn(N, Nc, H, W, device="cuda")
    g = torch.randn(N, M, H, W, device="cuda")
    gw_ref = torch.nn.grad.conv2d_weight(x, (M, Nc, 3, 3), g, padding=1)
    gb_ref = g.sum((0, 2, 3))
    A, B = g.permute(0, 2, 3, 1).contiguous(), x.permute(0, 2, 3, 1).contiguous()
    old = F32.USE_WGRAD_HALO
    try:
        for halo in (True, False):
            F32.USE_WGRAD_HALO = halo
            gw = torch.zeros(M, Nc, 3, 3, device="cuda")
            gb = torch.zeros(M, device="cuda")
            F32.wgrad(A, B, gw, gb, KH=3, KW=3, s=1, pad=1)
            assert _rel(gw, gw_ref) < 1e-5 and _rel(gb, gb_ref) < 1e-5, halo
    finally:
        F32.USE_WGRAD_HALO = old


@pytest.mark.parametrize("N,H,W,Cin,Cmid,Cout,cs", [(2, 12, 20, 3, 32, 32, 4), (1, 16, 16, 128, 64, 64, 128)])
def test_double_conv_fwd_bwd(hip_lib, N, H, W, Cin, Cmid, Cout, cs):
    """The fused DoubleConv Function (inner ReLU backward as conv2's dgrad mask epilogue) vs torch fp32."""
    from distributedpytorch_amd.models.hip_unet_f32 import _DoubleConvReLU
    torch.manual_seed(Cin + Cmid)
    xr = torch.randn(N, Cin, H, W, device="cuda")
    w1 = (torch.randn(Cmid, Cin, 3, 3, device="cuda") / (9 * Cin) ** 0.5).requires_grad_(True)
    b1 = (torch.randn(Cmid, device="cuda") * 0.1).requires_grad_(True)
    w2 = (torch.randn(Cout, Cmid, 3, 3, device="cuda") / (9 * Cmid) ** 0.5).requires_grad_(True)
    b2 = (torch.randn(Cout, device="cuda") * 0.1).requires_grad_(True)
    ref_x = xr.clone().requires_grad_(True)
    ref = torch.relu(F.conv2d(torch.relu(F.conv2d(ref_x, w1, b1, padding=1)), w2, b2, padding=1))
    g = torch.randn_like(ref)
    refs = torch.autograd.grad(ref, (ref_x, w1, b1, w2, b2), g)
    xn = torch.zeros(N, H, W, cs, device="cuda")
    xn[..., :Cin] = xr.permute(0, 2, 3, 1)
    xn.requires_grad_(True)
    y = _DoubleConvReLU.apply(xn, w1, b1, w2, b2, cs)
    assert _rel(y.permute(0, 3, 1, 2), ref) < 1e-5
    gx, gw1, gb1, gw2, gb2 = torch.autograd.grad(y, (xn, w1, b1, w2, b2), g.permute(0, 2, 3, 1).contiguous())
    assert _rel(gx[..., :Cin].permute(0, 3, 1, 2), refs[0]) < 1e-5
    for got, want in zip((gw1, gb1, gw2, gb2), refs[1:]):
        assert _rel(got, want) < 1e-5


@pytest.mark.parametrize("N,h,w,Cin,Cout", [(2, 8, 12, 64, 32), (1, 5, 7, 128, 64), (2, 4, 4, 512, 256)])
def test_deconv_fwd_bwd(hip_lib, N, h, w, Cin, Cout):
    from distributedpytorch_amd.models.hip_unet_f32 import _Deconv
    torch.manual_seed(Cin)
    x = torch.randn(N, Cin, h, w, device="cuda").requires_grad_(True)
    wt = (torch.randn(Cin, Cout, 2, 2, device="cuda") / Cin ** 0.5).requires_grad_(True)
    b = (torch.randn(Cout, device="cuda") * 0.1).requires_grad_(True)
    ref = F.conv_transpose2d(x, wt, b, stride=2)
    g = torch.randn_like(ref)
    gx_ref, gw_ref, gb_ref = torch.autograd.grad(ref, (x, wt, b), g)
    xn = x.detach().permute(0, 2, 3, 1).contiguous().requires_grad_(True)
    y = _Deconv.apply(xn, wt, b)
    assert _rel(y.permute(0, 3, 1, 2), ref) < 1e-5
    gx, gw, gb = torch.autograd.grad(y, (xn, wt, b), g.permute(0, 2, 3, 1).contiguous())
    assert _rel(gx.permute(0, 3, 1, 2), gx_ref) < 1e-5 and _rel(gw, gw_ref) < 1e-5 and _rel(gb, gb_ref) < 1e-5


def test_pool_and_head(hip_lib):
    from distributedpytorch_amd.compute import loss_partials_from_probs
    from distributedpytorch_amd.models.hip_unet_f32 import _HeadLoss, _MaxPool
    torch.manual_seed(1)
    x = torch.relu(torch.randn(2, 32, 10, 14, device="cuda")).requires_grad_(True)
    ref = F.max_pool2d(x, 2, 2)
    g = torch.randn_like(ref)
    (gx_ref,) = torch.autograd.grad(ref, (x,), g)
    xn = x.detach().permute(0, 2, 3, 1).contiguous().requires_grad_(True)
    y = _MaxPool.apply(xn)
    assert torch.equal(y.permute(0, 3, 1, 2), ref)
    (gx,) = torch.autograd.grad(y, (xn,), g.permute(0, 2, 3, 1).contiguous())
    assert torch.equal(gx.permute(0, 3, 1, 2), gx_ref)
    # head: 1x1 conv + sigmoid + loss partial sums, and its backward
    yv = torch.randn(2, 32, 16, 16, device="cuda").requires_grad_(True)
    hw = (torch.randn(1, 32, 1, 1, device="cuda") * 0.2).requires_grad_(True)
    hb = torch.randn(1, device="cuda").requires_grad_(True)
    t = (torch.rand(2, 1, 16, 16, device="cuda") > 0.5).float()
    S_ref = loss_partials_from_probs(torch.sigmoid(F.conv2d(yv, hw, hb)), t)
    dS = torch.tensor([0.3, -1.2, 0.7, 0.1], device="cuda")
    g_ref = torch.autograd.grad(S_ref, (yv, hw, hb), dS)
    yn = yv.detach().permute(0, 2, 3, 1).contiguous().requires_grad_(True)
    S = _HeadLoss.apply(yn, hw, hb, t)
    assert _rel(S, S_ref) < 1e-5
    gy, ghw, ghb = torch.autograd.grad(S, (yn, hw, hb), dS)
    assert _rel(gy.permute(0, 3, 1, 2), g_ref[0]) < 1e-4 and _rel(ghw, g_ref[1]) < 1e-4 and _rel(ghb, g_ref[2]) < 1e-4


@pytest.mark.parametrize("hw", [(64, 96), (40, 56)])
def test_unet_fp32_step_matches_torch(hip_lib, hw):
    """Reference UNet (31 layers, 7.76 M parameters) fp32 training step: loss and every gradient of the
    fp32 HIP engine vs stock PyTorch fp32 (TorchBlocks without autocast); (40, 56): the center-crop path."""
    from distributedpytorch_amd.compute import Compute, loss_from_partials
    from distributedpytorch_amd.data.synthetic import synthetic_batch
    from distributedpytorch_amd.models.blocks import TorchBlocks
    from distributedpytorch_amd.models.hip_unet_f32 import HipF32Blocks
    from distributedpytorch_amd.models.unet import build_model
    torch.manual_seed(0)
    model = build_model("unet").cuda()
    img, mask = synthetic_batch(2, hw[0], hw[1], 3, seed=3)
    x, t = img.cuda(), mask.float().unsqueeze(1).cuda()
    if hw == (40, 56):          # the output shrinks to 32 x 48 (reference CenterCrop semantics): crop the target
        t = t[:, :, 4:36, 4:52].contiguous()
    res = []
    for blocks in (TorchBlocks(model, dtype="fp32", channels_last=False), HipF32Blocks(model)):
        model.zero_grad(set_to_none=True)
        comp = Compute(model, blocks)
        S = comp.forward_partials(x, t)
        loss = loss_from_partials(S, t.numel())
        loss.backward()
        torch.cuda.synchronize()
        res.append((loss.item(), {n: p.grad.detach().clone() for n, p in model.named_parameters()}))
    (l0, g0), (l1, g1) = res
    assert abs(l0 - l1) < 1e-5 * abs(l0)
    for n in g0:
        assert _rel(g1[n], g0[n]) < 1e-3, n
