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
