"""HBM bandwidth probe: read+write copy, read-only reduction and write-only fill on a 4 GiB tensor
(the traffic pattern of the full-resolution UNet layers), to set their kernel times against."""
import torch

def t(fn, reps=10):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps / 1e3

n = 1 << 31                                     # 2^31 bf16 = 4 GiB
x = torch.empty(n, dtype=torch.bfloat16, device="cuda").normal_()
y = torch.empty_like(x)
gb = n * 2 / 1e9
for name, fn, bytes_ in [("copy (read+write)", lambda: y.copy_(x), 2 * gb),
                         ("fill (write)", lambda: y.fill_(1.0), gb),
                         ("sum (read)", lambda: x.sum(dtype=torch.float32), gb),
                         ("add x+y -> y (2 reads + write)", lambda: y.add_(x), 3 * gb)]:
    s = t(fn)
    print(f"{name:32s} {s * 1e3:8.3f} ms  {bytes_ / s / 1e3:6.2f} TB/s", flush=True)
