"""Reference streaming rates on this box (torch elementwise kernels): copy (1R1W) and add (2R1W) over the byte
counts of the 128^2 1x1 layers, to price the 1x1 convs' achieved GB/s against what a plain stream reaches."""
import torch


def t(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1000 * e0.elapsed_time(e1) / iters


d = torch.device("cuda:0")
n = 16 * 128 * 128 * 128
a, b, c = (torch.randn(n, device=d) for _ in range(3))
us = t(lambda: c.copy_(a))
print(f"copy 1R1W {4 * n / 1e6:.0f} MB: {us:.1f} us, {8 * n / us / 1e3:.0f} GB/s")
us = t(lambda: torch.add(a, b, out=c))
print(f"add 2R1W {4 * n / 1e6:.0f} MB each: {us:.1f} us, {12 * n / us / 1e3:.0f} GB/s")
h = torch.randn(n // 2, device=d)
