"""Dual conv input (the 32-channel UNet level without a concat buffer): the decoder's first conv reads
its 64 input channels from two dense [N,H,W,32] tensors -- the skip and the up-sampled half --
through ``x2`` of the row-streaming forward (csrc/halo.hip igemm_stream_kernel) and of the fused
backward (csrc/bwd_stream.hip).  Reference behaviour: ``torch.cat([skip, up], dim=1)`` followed by the
DoubleConv (reference model/unet_parts.py:76-95).

Both kernels stage the same LDS images from the two tensors as from the interleaved concat, so the
results must equal the concat-buffer launches bitwise, and match a plain fp32 PyTorch conv.
"""
import pytest
import torch
import torch.nn.functional as F

from test_hip_kernels import _pack_one

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


@pytest.mark.parametrize("N,H,W,Ng", [(2, 20, 512, 32), (2, 33, 96, 32), (1, 16, 256, 64), (3, 8, 136, 64)])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4])
def test_stream_forward_dual_equals_concat(hip_lib, N, H, W, Ng, variant):
    from distributedpytorch_amd.ops import kernels as K
    if variant in (1, 3) and W % 128:
        pytest.skip("128-pixel strips need W % 128 == 0 for this A/B (auto picks 64)")
    g = torch.Generator().manual_seed(N * H + W)
    skip = torch.randn(N, H, W, 32, generator=g).to(torch.bfloat16).cuda()
    up = torch.randn(N, H, W, 32, generator=g).to(torch.bfloat16).cuda()
    w = torch.randn(Ng, 64, 3, 3, generator=g) / 24.0
    b = (torch.randn(Ng, generator=g) * 0.1).cuda()
    wp, _, kf = _pack_one(0, w)
    assert kf == 576
    cat = torch.cat([skip, up], dim=3).contiguous()
    y0 = torch.empty(N, H, W, Ng, dtype=torch.bfloat16, device="cuda")
    y1 = torch.empty_like(y0)
    kw = dict(Ngemm=Ng, Kpad=576, KH=3, KW=3, stride=1, pad=1, Cs=64, out_grid=(N, H, W), bias=b, relu=True,
              path="stream", variant=variant)
    K.igemm(cat, wp, y0, **kw)
    K.igemm(skip, wp, y1, x2=up, **kw)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    ref = torch.relu(F.conv2d(cat.float().permute(0, 3, 1, 2).cpu(), w.to(torch.bfloat16).float(), b.cpu(), padding=1))
    assert _rel(y1.float().cpu(), ref.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("N,H,W,CO", [(2, 24, 512, 32), (2, 17, 192, 32), (1, 16, 128, 64)])
@pytest.mark.parametrize("mode", ["split", "mask"])
def test_fused_backward_dual_equals_concat(hip_lib, N, H, W, CO, mode):
    from distributedpytorch_amd.ops import kernels as K
    if not K.bwd_fused_eligible(64, CO, W):
        pytest.skip("no fused backward for this shape")
    g_ = torch.Generator().manual_seed(W + CO)
    skip = torch.relu(torch.randn(N, H, W, 32, generator=g_)).to(torch.bfloat16).cuda()
    up = torch.relu(torch.randn(N, H, W, 32, generator=g_)).to(torch.bfloat16).cuda()
    g = torch.randn(N, H, W, CO, generator=g_).to(torch.bfloat16).cuda()
    w = torch.randn(CO, 64, 3, 3, generator=g_) / 24.0
    wd, _, kd = _pack_one(1, w)
    cat = torch.cat([skip, up], dim=3).contiguous()
    outs = []
    for dual in (False, True):
        gw = torch.zeros(CO * 64 * 9, device="cuda")
        gb = torch.zeros(CO, device="cuda")
        x, x2 = (skip, up) if dual else (cat, None)
        if mode == "split":
            hi = torch.empty(N, H, W, 32, dtype=torch.bfloat16, device="cuda")
            lo, hi = K.conv_bwd_fused(g, x, wd, kd, gw, gb, mask=False, dx2=hi, split=32, x2=x2)
            dx = torch.cat([lo, hi], dim=3)
        else:
            dx = K.conv_bwd_fused(g, x, wd, kd, gw, gb, mask=True, x2=x2)
        torch.cuda.synchronize()
        outs.append((dx, gw, gb))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]) and torch.equal(outs[0][2], outs[1][2])
    # fp32 anchor of the dual launch
    xc = cat.float().permute(0, 3, 1, 2).cpu().requires_grad_(True)
    wc = w.to(torch.bfloat16).float().requires_grad_(True)
    y = F.conv2d(xc, wc, padding=1)
    y.backward(g.float().permute(0, 3, 1, 2).cpu())
    dx_ref = xc.grad.permute(0, 2, 3, 1)
    if mode == "mask":
        dx_ref = dx_ref * (cat.float().cpu() > 0)
    dx, gw, gb = outs[1]
    assert _rel(dx.float().cpu(), dx_ref) < 1e-2
    assert _rel(gw.view(CO, 64, 3, 3).cpu(), wc.grad) < 1e-3
    assert _rel(gb.cpu(), g.float().sum((0, 1, 2)).cpu()) < 1e-3


def test_unet_step_dual_equals_concat(hip_lib, monkeypatch):
    """A whole UNet training step with the full-resolution level on the dual input == the same step
    with the concat buffer (same values staged in the same order)."""
    from distributedpytorch_amd.compute import loss_from_partials, make_compute
    from distributedpytorch_amd.data.synthetic import synthetic_batch
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.optim import FlatParameterSpace
    from distributedpytorch_amd.ops import kernels as K

    torch.manual_seed(0)
    model = build_model("unet").cuda()
    space = FlatParameterSpace(model)
    comp = make_compute(model, backend="hip", dtype="bf16")
    img, mask = synthetic_batch(2, 64, 256, 3, seed=5)
    x, t = img.cuda(), mask.float().unsqueeze(1).cuda()
    seen = []
    real = K.igemm

    def spy(*a, **kw):
        seen.append(kw.get("x2") is not None)
        return real(*a, **kw)

    monkeypatch.setattr(K, "igemm", spy)

    def run():
        space.zero_grad()
        seen.clear()
        S = comp.forward_partials(x, t)
        loss = loss_from_partials(S, t.numel())
        loss.backward()
        torch.cuda.synchronize()
        return loss.item(), space.grad.clone(), any(seen)

    l1, g1, used1 = run()
    monkeypatch.setattr(K, "USE_DUAL_INPUT", False)
    l0, g0, used0 = run()
    assert used1 and not used0
    assert l0 == l1
    assert torch.allclose(g0, g1, rtol=1e-5, atol=1e-7 * g0.abs().max().item())
