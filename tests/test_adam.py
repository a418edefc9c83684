import math

import pytest
import torch

from distributedpytorch_amd.optim import FlatParameterSpace, FusedAdam, adam_reference
from distributedpytorch_amd.models.unet import build_model


def _torch_adam_ref(n=1000, steps=3, wd=1e-8, device="cpu"):
    torch.manual_seed(0)
    p0 = torch.randn(n)
    gs = [torch.randn(n) for _ in range(steps)]
    p = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([p], lr=1e-3, weight_decay=wd)
    for g in gs:
        p.grad = g.clone()
        opt.step()
    return p0, gs, p.detach()


def test_adam_reference_matches_torch():
    p0, gs, want = _torch_adam_ref()
    p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    for k, g in enumerate(gs, 1):
        adam_reference(p, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 1e-8, 1 - 0.9 ** k, 1 - 0.999 ** k)
    torch.testing.assert_close(p, want, rtol=1e-6, atol=1e-7)


def test_flat_space_views_and_fused_adam_cpu():
    model = build_model("unet-tiny")
    ref = build_model("unet-tiny")
    ref.load_state_dict(model.state_dict())
    space = FlatParameterSpace(model)
    assert space.numel == sum(p.numel() for p in model.parameters())
    opt = FusedAdam(space, lr=1e-3, weight_decay=1e-8)
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-8)
    x = torch.randn(2, 3, 16, 16)
    for _ in range(2):
        opt.zero_grad()
        ropt.zero_grad()
        model(x).sum().backward()
        ref(x).sum().backward()
        # grads landed in the flat buffer
        assert space.grad.abs().sum() > 0
        opt.step()
        ropt.step()
    for (n, a), (_, b) in zip(model.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6, msg=n)


@pytest.mark.gpu
def test_adam_hip_matches_reference(hip_lib):
    from distributedpytorch_amd import ops
    torch.manual_seed(0)
    n = 1_000_003  # odd length exercises the scalar tail
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda")
    m = torch.randn(n, device="cuda").abs() * 0.1
    v = torch.randn(n, device="cuda").abs() * 0.1
    pr, mr, vr = p.cpu().clone(), m.cpu().clone(), v.cpu().clone()
    for k in (1, 2, 3):
        bc1, bc2 = 1 - 0.9 ** k, 1 - 0.999 ** k
        ops.adam_step(p, g, m, v, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2, bc1=bc1, bc2=bc2)
        adam_reference(pr, g.cpu(), mr, vr, 1e-3, 0.9, 0.999, 1e-8, 1e-2, bc1, bc2)
    torch.cuda.synchronize()
    torch.testing.assert_close(p.cpu(), pr, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m.cpu(), mr, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(v.cpu(), vr, rtol=1e-5, atol=1e-6)


def test_device_state_adam_cpu_matches_host_state():
    """Device-state mode (HIP-graph replay form) gives the host-state trajectory, incl. an LR cut."""
    torch.manual_seed(3)
    a, b = build_model("unet-tiny"), build_model("unet-tiny")
    b.load_state_dict(a.state_dict())
    sa, sb = FlatParameterSpace(a), FlatParameterSpace(b)
    oa, ob = FusedAdam(sa, lr=1e-3, weight_decay=1e-8), FusedAdam(sb, lr=1e-3, weight_decay=1e-8)
    ob.enable_device_state()
    for k in range(4):
        if k == 2:
            oa.param_groups[0]["lr"] = ob.param_groups[0]["lr"] = 2e-4
        g = torch.randn(sa.numel)
        sa.grad.copy_(g)
        sb.grad.copy_(g)
        oa.step()
        ob.step()
    assert ob.step_count == oa.step_count == 4 and float(ob._dev_state[0][0]) == 4.0
    torch.testing.assert_close(sb.data, sa.data, rtol=1e-6, atol=1e-7)


@pytest.mark.gpu
def test_adam_hip_device_state_matches_host(hip_lib):
    from distributedpytorch_amd import ops
    torch.manual_seed(0)
    n = 100_003
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda")
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    state = torch.tensor([0.0, 1e-3, 0.0, 0.0], dtype=torch.float64, device="cuda")
    for k in (1, 2, 3):
        ops.adam_step(p, g, m, v, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2,
                      bc1=1 - 0.9 ** k, bc2=1 - 0.999 ** k)
        ops.adam_step_dev(p2, g, m2, v2, state, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2)
    torch.cuda.synchronize()
    assert float(state[0]) == 3.0
    torch.testing.assert_close(p2, p, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(v2, v, rtol=1e-6, atol=1e-7)
