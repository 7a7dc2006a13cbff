"""Per-launch table of every implicit-GEMM conv launch in one training step (HIP-event timed).

    python scripts/layer_table.py [--batch 16] [--size 256]
Prints: us, TFLOP/s (algorithmic), GB/s (algorithmic bytes), geometry; aggregated by geometry.
"""
import argparse
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--amp", action="store_true", help="fp16-operand convs (autocast), as the AMP training mode")
    args = ap.parse_args()
    from hyres_hip.weights import synthetic_state_dict
    from hyres_hip.loss import RateDistortionLoss
    from hyres_hip import ops as O
    from models import ResidualJPEGCompression
    dev = torch.device("cuda:0")
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(dev).train()
    B, S = args.batch, args.size
    x = (torch.randint(0, 256, (B, 3, S, S), generator=torch.Generator().manual_seed(0)).float() / 255).to(dev)
    crit = RateDistortionLoss(lmbda=0.045, alpha=0)

    def step():
        with torch.autocast("cuda", dtype=torch.float16, enabled=args.amp):
            out = net.forward_device(x, x, 0.0)
            loss = crit(out, x)["loss"]
        loss.backward()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    O.SideStream.enabled = False  # time each launch alone (no overlap with the side stream)
    O.BranchStreams.enabled = False
    O.KernelTimer.reset()
    O.KernelTimer.enabled = True
    O.KernelTimer.all_convs = True
    step()
    torch.cuda.synchronize()
    O.KernelTimer.enabled = False
    agg = collections.OrderedDict()
    for desc, a, b, fl, by in O.KernelTimer.table:
        ms = a.elapsed_time(b)
        e = agg.setdefault(desc, [0, 0.0, fl, by])
        e[0] += 1
        e[1] += ms
    tot = sum(v[1] for v in agg.values())
    print(f"total conv+wgrad time {tot:.2f} ms, {sum(v[0] for v in agg.values())} launches")
    print(f"{'ms':>7} {'n':>3} {'us/launch':>9} {'TF/s':>7} {'GB/s':>7}  geometry")
    for d, (n, ms, fl, by) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        us = 1000 * ms / n
        print(f"{ms:7.3f} {n:3d} {us:9.1f} {fl / us / 1e6:7.1f} {by / us / 1e3:7.0f}  {d}")
    # by region: the larger of the two resolutions a launch touches (WGRAD rows: P / Q sides)
    region = collections.Counter()
    for d, (n, ms, fl, by) in agg.items():
        sizes = [int(t.split("x")[0]) for t in d.replace("->", " ").split() if "x" in t and t[0].isdigit()]
        region[max(sizes)] += ms
    print("by resolution (max side touched): " +
          ", ".join(f"{r}^2 {ms:.2f} ms" for r, ms in sorted(region.items(), reverse=True)))


if __name__ == "__main__":
    main()
