"""Pipeline stage boundaries INSIDE a DoubleConv (cuts ``b + 0.5``, models/blocks.py): the HIP engines'
half-block paths (``enc_a/enc_b/mid_a/mid_b/dec_a/dec_b``) against the same step with whole blocks, on
one GPU (GPipeLocal, every stage on cuda:0).  One microbatch, so the pipelined step is the single-device
step exactly up to the fusions the cut removes (bf16: same values, other kernels / orders)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-30)).item()


@pytest.mark.parametrize("dtype,cuts,model_name", [("bf16", (0, 2.5, 7.5, 10), "unet"),
                                                   ("bf16", (0, 0.5, 4.5, 8.5, 10), "unet"),
                                                   ("bf16", (0, 1.5, 5.5, 10), "unet-bn"),
                                                   ("fp32", (0, 0.5, 4.5, 8.5, 10), "unet")])
def test_half_block_cuts_match_whole_blocks(hip_lib, dtype, cuts, model_name):
    from distributedpytorch_amd.compute import loss_from_partials, make_compute
    from distributedpytorch_amd.data.synthetic import synthetic_batch
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.optim import FlatParameterSpace
    from distributedpytorch_amd.parallel.pipeline import GPipeLocal
    torch.manual_seed(0)
    img, mask = synthetic_batch(2, 64, 96, 3, seed=9)
    x, t = img.cuda(), mask.float().unsqueeze(1).cuda()
    ref = build_model(model_name).cuda()
    state = {k: v.clone() for k, v in ref.state_dict().items()}
    FlatParameterSpace(ref)
    comp = make_compute(ref, backend="hip", dtype=dtype)
    S = comp.forward_partials(x, t)
    loss_ref = loss_from_partials(S, t.numel())
    loss_ref.backward()
    g_ref = {n: p.grad.detach().clone() for n, p in ref.named_parameters()}
    model = build_model(model_name)
    model.load_state_dict(state)
    dev = torch.device("cuda:0")
    pipe = GPipeLocal(model.to(dev), [dev] * (len(cuts) - 1), 1, backend="hip", dtype=dtype, cuts=list(cuts),
                      img_hw=(64, 96))
    loss = pipe.forward_loss(x, t)
    loss.backward()
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == "fp32" else 2e-3
    assert abs(loss.item() - loss_ref.item()) < tol * max(1.0, abs(loss_ref.item()))
    gmax = max(float(g.norm()) for g in g_ref.values())
    for n, p in model.named_parameters():
        assert p.grad is not None, n
        if float(g_ref[n].norm()) < 1e-4 * gmax:
            # a conv bias in front of a BatchNorm: its true gradient is zero (BN removes it), both runs
            # hold rounding noise -- compare magnitudes, not directions
            assert float(p.grad.norm()) < 1e-3 * gmax, n
            continue
        c = _cos(p.grad, g_ref[n])
        assert c > (0.99999 if dtype == "fp32" else 0.999), (n, c)


def test_bn_pipeline_microbatches_keep_skips_plain(hip_lib):
    """the BN engine may keep a full-resolution skip as its BN input z only when the
    consuming decoder level runs in the same ``run_segment`` call.  Under the mirrored (V) placement the
    skip's encoder and decoder levels are two segments of one stage, and with M = 2 microbatches segment 0
    of microbatch 1 (whose ``prep`` resets the engine's hand-over map) runs between them.  Checked three
    ways: (1) bitwise-level equal to the same step with the z hand-over switched off everywhere, (2) close to
    the reference cut (two separate engines, nothing handed over between the levels) on the same
    microbatches, (3) near the stock-PyTorch fp32 pipeline (BatchNorm statistics are per microbatch in all)."""
    from distributedpytorch_amd.data.synthetic import synthetic_batch
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.ops import kernels as K
    from distributedpytorch_amd.parallel.pipeline import GPipeLocal
    from distributedpytorch_amd.parallel.placement import Placement
    torch.manual_seed(0)
    img, mask = synthetic_batch(4, 128, 128, 3, seed=5)
    x, t = img.cuda(), mask.float().unsqueeze(1).cuda()
    base = build_model("unet-bn")
    state = {k: v.clone() for k, v in base.state_dict().items()}
    dev = torch.device("cuda:0")
    v_pl, ref_pl = Placement.mirrored([0, 2, 7, 10]), Placement.contiguous([0, 5, 10])

    def run(backend, dtype, pl):
        m = build_model("unet-bn")
        m.load_state_dict(state)
        pipe = GPipeLocal(m.to(dev), [dev, dev], 2, backend=backend, dtype=dtype, img_hw=(128, 128),
                          placement=pl)
        for s in pipe.spaces:
            s.zero_grad()
        loss = pipe.forward_loss(x, t)
        (loss * x.shape[0]).backward()
        torch.cuda.synchronize()
        return loss.item(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}

    l_hip, g_hip = run("hip", "bf16", v_pl)
    saved = K.BN_SKIP_Z
    K.BN_SKIP_Z = False
    try:
        l_plain, g_plain = run("hip", "bf16", v_pl)
    finally:
        K.BN_SKIP_Z = saved
    assert abs(l_hip - l_plain) <= 1e-5 * abs(l_plain), (l_hip, l_plain)
    for n, g in g_plain.items():
        assert torch.allclose(g_hip[n], g, rtol=1e-4, atol=1e-6 * float(g.abs().max())), n
    l_cut, g_cut = run("hip", "bf16", ref_pl)
    l_ref, g_ref = run("torch", "fp32", v_pl)
    assert abs(l_hip - l_cut) < 2e-3 * abs(l_cut), (l_hip, l_cut)
    assert abs(l_hip - l_ref) < 5e-3 * abs(l_ref), (l_hip, l_ref)
    gmax = max(float(g.norm()) for g in g_ref.values())
    worst = {}
    for n, g in g_ref.items():
        if float(g.norm()) < 1e-4 * gmax:
            continue          # conv bias in front of a BatchNorm: true gradient zero, both hold noise
        worst[n] = (_cos(g_hip[n], g_cut[n]), _cos(g_hip[n], g))
        # V vs reference cut: the same bf16 function on other kernels / fusions (measured >= 0.99997); vs fp32:
        # bf16 storage with BatchNorm backward over 2-image microbatches amplifies rounding (a BN bias at the
        # 16^2 level: 0.895) -> only a gross-error bound
        assert worst[n][0] > 0.999 and worst[n][1] > 0.8, (n, worst[n])
