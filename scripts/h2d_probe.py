"""Host->device copy rates on the box: pageable vs pinned (the PCIe-inclusive rate of DESIGN.md §8).

    python scripts/h2d_probe.py
"""
import time

import torch


def rate(t, dev, reps=5):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t.to(dev, non_blocking=t.is_pinned())
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    for mb in (4.7, 12.6, 50.3):
        n = int(mb * 1e6 / 4)
        pg = torch.rand(n)
        pn = torch.rand(n).pin_memory()
        a, b = rate(pg, dev), rate(pn, dev)
        t0 = time.perf_counter()
        pg.pin_memory()
        c = time.perf_counter() - t0
        print(f"{mb:5.1f} MB: pageable {a * 1e3:7.2f} ms ({mb / a / 1e3:6.2f} GB/s), pinned {b * 1e3:6.2f} ms "
              f"({mb / b / 1e3:6.2f} GB/s), pin_memory() copy {c * 1e3:6.2f} ms")


if __name__ == "__main__":
    main()
