"""Fused first-level forward (csrc/dconv_fwd.hip): conv3x3(8->32)+ReLU -> conv3x3(32->32)+ReLU ->
2x2 max-pool with window codes in one row-streaming kernel, the intermediate kept in an LDS ring.
Bitwise equal to the two streaming kernels it replaces (same MFMA order, same bf16 roundings), and
within bf16 rounding of the fp32 PyTorch reference of the same ops."""
import pytest
import torch
import torch.nn.functional as F

from test_hip_kernels import _bf, _nchw, _pack_one, _rel

pytestmark = pytest.mark.gpu   # calls the kernel directly: runs whether or not the engine enables it


@pytest.mark.parametrize("N,H,W", [(2, 6, 128), (1, 34, 256), (3, 16, 128), (1, 2, 384)])
def test_dconv1_fwd_matches_two_kernels(hip_lib, N, H, W):
    from distributedpytorch_amd.ops import kernels as K
    torch.manual_seed(13)
    img = torch.rand(N, 3, H, W)
    x8 = torch.zeros(N, H, W, 8, dtype=torch.bfloat16, device="cuda")
    x8[..., :3] = img.permute(0, 2, 3, 1).cuda().to(torch.bfloat16)
    w1 = _bf(torch.randn(32, 3, 3, 3) * 0.3)
    w2 = _bf(torch.randn(32, 32, 3, 3) * 0.08)
    b1, b2 = (torch.randn(32) * 0.1).cuda(), (torch.randn(32) * 0.1).cuda()
    p1, _, k1 = _pack_one(0, w1, cin_pad=8)
    p2, _, k2 = _pack_one(0, w2)
    # reference path: igemm_stream8, then igemm_stream with the fused pool epilogue
    a_r = torch.empty(N, H, W, 32, dtype=torch.bfloat16, device="cuda")
    K.igemm(x8, p1, a_r, Ngemm=32, Kpad=k1, KH=3, KW=3, stride=1, pad=1, Cs=8, out_grid=(N, H, W), bias=b1, relu=True)
    cat_r = torch.zeros(N, H, W, 64, dtype=torch.bfloat16, device="cuda")
    pool_r = torch.empty(N, H // 2, W // 2, 32, dtype=torch.bfloat16, device="cuda")
    code_r = torch.empty(N, H // 2, W // 2, 32, dtype=torch.uint8, device="cuda")
    K.igemm(a_r, p2, cat_r[..., :32], Ngemm=32, Kpad=k2, KH=3, KW=3, stride=1, pad=1, Cs=32, out_grid=(N, H, W),
            bias=b2, relu=True, pool=pool_r, pcode=code_r)
    # fused
    a = torch.full_like(a_r, 7.0)
    cat = torch.zeros_like(cat_r)
    pool = torch.full_like(pool_r, 7.0)
    code = torch.full_like(code_r, 255)
    K.dconv1_fwd(x8, p1, k1, b1, p2, k2, b2, a, cat[..., :32], pool, code)
    torch.cuda.synchronize()
    assert torch.equal(a, a_r)
    assert torch.equal(cat, cat_r)                  # skip half written, the other half untouched
    assert torch.equal(pool, pool_r) and torch.equal(code, code_r)
    # fp32 reference of the same ops
    ref = F.relu(F.conv2d(F.relu(F.conv2d(_nchw(x8)[:, :3], w1, b1.cpu(), padding=1)), w2, b2.cpu(), padding=1))
    assert _rel(_nchw(cat[..., :32]), ref) < 2e-2
    assert _rel(_nchw(pool), F.max_pool2d(ref, 2)) < 2e-2
