#!/usr/bin/env python3
"""Plain-GEMM ceiling for the deep UNet conv shapes: hipBLASLt (torch.matmul, bf16) on the im2col
GEMM (M = pixels, N = Cout, K = 9*Cin) vs our implicit-GEMM kernels.  Tells how far the conv cores
are from what the vendor library reaches on the same M x N x K (no gather, no epilogue)."""
import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t(fn, reps=10):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        s.record(); fn(); e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e) * 1e3)
    ts.sort(); return ts[len(ts) // 2]


B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
for name, H, Cin, Cout in [("L2 128->128", 128, 128, 128), ("L3 256->256", 64, 256, 256),
                           ("L3 512->256", 64, 512, 256), ("mid 512->512", 32, 512, 512), ("sq 8192", 0, 0, 0)]:
    if H:
        M, N, Kd = B * H * H, Cout, 9 * Cin
    else:
        M = N = Kd = 8192
    a = torch.randn(M, Kd, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(Kd, N, device="cuda", dtype=torch.bfloat16)
    us = t(lambda: a @ b)
    print(f"{name:14s} M={M:8d} N={N:4d} K={Kd:5d}  hipBLASLt {us:9.1f} us  {2*M*N*Kd/us/1e6:7.1f} TF", flush=True)
