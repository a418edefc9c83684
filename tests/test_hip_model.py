"""Whole-model parity: the HIP engine (bf16 kernels, explicit backward) vs the reference-semantics
UNet on PyTorch fp32 (CPU), same weights, same batch: loss, every parameter gradient, one Adam
step, and the probability map used for evaluation/Dice."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cos(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-30)).item()


@pytest.mark.parametrize("name,hw", [("unet", (64, 64)), ("unet", (48, 80)), ("unet-xl", (64, 64)), ("unet", (64, 256)),
                                     # the reference's 640x960 aspect (utils/train_utils.py:26): deep levels
                                     # not multiples of 32 (15 / 7.5 / ... strips), ragged row tiles
                                     ("unet", (160, 240)), ("unet", (320, 480))])
def test_hip_unet_matches_torch_fp32(hip_lib, name, hw):
    from distributedpytorch_amd.compute import loss_from_partials, make_compute
    from distributedpytorch_amd.loss import bce_dice_from_probs
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.optim import FlatParameterSpace
    from distributedpytorch_amd.data.synthetic import synthetic_batch

    torch.manual_seed(0)
    ref = build_model(name)
    hip = build_model(name)
    hip.load_state_dict(ref.state_dict())
    img, mask = synthetic_batch(2, hw[0], hw[1], 3, seed=3)
    t = mask.float().unsqueeze(1)

    # reference: fp32 on CPU, reference loss semantics (utils/utils.py:9-25), loss scaled by batch (A11)
    loss_ref = bce_dice_from_probs(ref(img), t)
    (2 * loss_ref).backward()

    hip = hip.cuda()
    space = FlatParameterSpace(hip)
    comp = make_compute(hip, backend="hip", dtype="bf16")
    S = comp.forward_partials(img.cuda(), t.cuda())
    loss = loss_from_partials(S, t.numel())
    (2 * loss).backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - loss_ref.item()) < 2e-2 * abs(loss_ref.item()), (loss.item(), loss_ref.item())
    for (n, p_ref), (_, p) in zip(ref.named_parameters(), hip.named_parameters()):
        g_ref, g = p_ref.grad, p.grad.cpu()
        c = _cos(g, g_ref)
        assert c > 0.98, f"{n}: cosine {c:.4f}"
        r = (g.norm() / g_ref.norm()).item()
        assert 0.9 < r < 1.1, f"{n}: norm ratio {r:.4f}"
    # gradients landed in the flat buffer
    assert space.grad.abs().sum().item() > 0

    with torch.no_grad():
        p_ref = ref(img)
        p = comp.probs(img.cuda()).cpu()
    assert (p - p_ref).abs().max().item() < 3e-2


def test_engine_image_chunking_invariant(hip_lib, monkeypatch):
    """Launches over > 2 GiB tensors are split by image (32-bit buffer offsets).  Force one image per
    launch on a small batch: loss and every gradient must match the unsplit run (per-chunk weight
    gradient slabs only change the fp32 summation order)."""
    from distributedpytorch_amd.compute import loss_from_partials, make_compute
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.optim import FlatParameterSpace
    from distributedpytorch_amd.data.synthetic import synthetic_batch
    from distributedpytorch_amd.ops import kernels as K

    torch.manual_seed(0)
    model = build_model("unet").cuda()
    space = FlatParameterSpace(model)
    comp = make_compute(model, backend="hip", dtype="bf16")
    img, mask = synthetic_batch(3, 64, 128, 3, seed=11)
    x, t = img.cuda(), mask.float().unsqueeze(1).cuda()

    def run():
        space.zero_grad()
        S = comp.forward_partials(x, t)
        loss = loss_from_partials(S, t.numel())
        (3 * loss).backward()
        torch.cuda.synchronize()
        return loss.item(), space.grad.clone()

    l0, g0 = run()
    monkeypatch.setattr(K, "_MAX_BYTES", 1)   # one image per launch
    l1, g1 = run()
    assert abs(l0 - l1) < 1e-5 * abs(l0)
    assert torch.allclose(g0, g1, rtol=1e-3, atol=1e-6 * g0.abs().max().item())


def test_hip_odd_size_center_crop_matches_reference(hip_lib):
    """H, W not divisible by 16: the reference center-crops each skip (model/unet_parts.py:58-74) and
    the output shrinks.  Probabilities, loss and every parameter gradient of the HIP
    engine (cropped skips copied into fresh concat buffers, zero-padded crop gradient) match."""
    from distributedpytorch_amd.compute import loss_from_partials, make_compute
    from distributedpytorch_amd.loss import bce_dice_from_probs
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.optim import FlatParameterSpace
    torch.manual_seed(1)
    ref = build_model("unet")
    hip = build_model("unet")
    hip.load_state_dict(ref.state_dict())
    hip = hip.cuda()
    FlatParameterSpace(hip)
    comp = make_compute(hip, backend="hip", dtype="bf16")
    x = torch.rand(2, 3, 50, 70)
    t = (torch.rand(2, 1, 48, 64) > 0.6).float()
    with torch.no_grad():
        p = comp.probs(x.cuda()).cpu()
    p_ref = ref(x)
    assert p.shape == p_ref.shape == (2, 1, 48, 64)
    assert (p - p_ref.detach()).abs().max().item() < 3e-2
    loss_ref = bce_dice_from_probs(p_ref, t)
    (2 * loss_ref).backward()
    loss = loss_from_partials(comp.forward_partials(x.cuda(), t.cuda()), t.numel())
    (2 * loss).backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - loss_ref.item()) < 2e-2 * abs(loss_ref.item())
    for (n, pr), (_, ph) in zip(ref.named_parameters(), hip.named_parameters()):
        c = _cos(ph.grad.cpu(), pr.grad)
        assert c > 0.98, f"{n}: cosine {c:.4f}"
