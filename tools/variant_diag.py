"""Diagnostic: per-parameter gradient cosine of the HIP engine and of stock torch bf16 autocast vs the
fp32 reference for the BN / bilinear UNet variants."""
import sys
import torch
sys.path.insert(0, ".")
from distributedpytorch_amd.compute import loss_from_partials, make_compute
from distributedpytorch_amd.loss import bce_dice_from_probs
from distributedpytorch_amd.models.unet import build_model
from distributedpytorch_amd.optim import FlatParameterSpace
from distributedpytorch_amd.data.synthetic import synthetic_batch


def cos(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-30)).item()


for variant in sys.argv[1:] or ["bn"]:
    kw = {"batchnorm": "bn" in variant, "bilinear": "bilinear" in variant}
    torch.manual_seed(0)
    ref = build_model("unet", **kw)
    hip = build_model("unet", **kw)
    tb = build_model("unet", **kw)
    hip.load_state_dict(ref.state_dict())
    tb.load_state_dict(ref.state_dict())
    img, mask = synthetic_batch(4, 64, 64, 3, seed=5)
    t = mask.float().unsqueeze(1)
    loss_ref = bce_dice_from_probs(ref(img), t)
    (4 * loss_ref).backward()
    hip = hip.cuda()
    FlatParameterSpace(hip)
    comp = make_compute(hip, backend="hip", dtype="bf16")
    S = comp.forward_partials(img.cuda(), t.cuda())
    loss = loss_from_partials(S, t.numel())
    (4 * loss).backward()
    tb = tb.cuda()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        p = tb(img.cuda())
    lt = bce_dice_from_probs(p.float(), t.cuda())
    (4 * lt).backward()
    print(variant, "loss ref", loss_ref.item(), "hip", loss.item(), "torch-bf16", lt.item())
    for (n, a), (_, b), (_, c) in zip(ref.named_parameters(), hip.named_parameters(), tb.named_parameters()):
        print(f"{n:45s} |g|={a.grad.norm().item():.3e} hip cos {cos(b.grad.cpu(), a.grad):.4f} "
              f"ratio {(b.grad.norm().cpu() / a.grad.norm()).item():.3f}  torch-bf16 cos {cos(c.grad.cpu(), a.grad):.4f}")
