import torch, sys
sys.path.insert(0, ".")
from distributedpytorch_amd.ops import kernels as K
for (N, H, W, Cin, Cout) in [(1, 8, 128, 64, 128), (2, 5, 128, 32, 32), (1, 33, 64, 64, 64), (2, 16, 64, 128, 256)]:
    torch.manual_seed(3)
    x = torch.randn(N, Cin, H, W).bfloat16().float()
    w = (torch.randn(Cout, Cin, 3, 3) * (2.0 / (9 * Cin)) ** 0.5).bfloat16().float()
    b = torch.randn(Cout) * 0.1
    kf = K.round_up(9 * Cin, 32)
    packed = torch.zeros(Cout, kf)
    packed[:, :9 * Cin] = w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin)
    packed = packed.to(torch.bfloat16).cuda().reshape(-1)
    xh = x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).cuda()
    res = []
    for fused in (True, False):
        bn = torch.nn.BatchNorm2d(Cout).cuda()
        z = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device="cuda")
        stats = [] if fused else None
        K.igemm(xh, packed, z, Ngemm=Cout, Kpad=kf, KH=3, KW=3, stride=1, pad=1, Cs=Cin, out_grid=(N, H, W),
                bias=b.cuda(), relu=False, bn_stats=stats)
        y = torch.empty_like(z)
        saved = K.bn_fwd(z, y, bn, train=True, stats=stats)
        torch.cuda.synchronize()
        zf = z.float()
        res.append((saved.cpu(), zf.mean((0, 1, 2)).cpu()))
    (s1, zm), (s0, _) = res
    d = (s1 - s0).abs()
    print((N, H, W, Cin, Cout), "max abs diff", d.max().item(), "at", d.argmax().item(), "rel", (d / s0.abs().clamp_min(1e-6)).max().item(),
          "mean(fused)-true", (s1[:Cout] - zm).abs().max().item(), "mean(unfused)-true", (s0[:Cout] - zm).abs().max().item(), flush=True)
