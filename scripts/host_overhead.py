"""Host-side enqueue cost vs GPU time of one training step, plus eval (encode+decode) forward timings.

    python scripts/host_overhead.py [--batch 16] [--size 256]
Prints one JSON line per measurement: host enqueue ms (no sync), synced step ms, eval forward ms at
bs=16 256x256 and at Kodak size 768x512 (bs=1).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    from hyres_hip.weights import synthetic_state_dict
    from hyres_hip.loss import RateDistortionLoss
    from hyres_hip.optim import FusedAdam
    from models import ResidualJPEGCompression
    dev = torch.device("cuda:0")
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(dev).train()
    main_p = [p for n, p in sorted(net.named_parameters()) if not n.endswith(".quantiles")]
    opt = FusedAdam(main_p, lr=3e-4, max_grad_norm=1.0)
    B, S = args.batch, args.size
    x = (torch.randint(0, 256, (B, 3, S, S), generator=torch.Generator().manual_seed(0)).float() / 255).to(dev)
    crit = RateDistortionLoss(lmbda=0.045, alpha=0)

    def step():
        out = net.forward_device(x, x, 0.0)
        crit(out, x)["loss"].backward()
        opt.step()
        opt.zero_grad()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    host, full = [], []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e3)
        full.append((t2 - t0) * 1e3)
    print(json.dumps({"what": "train_step", "host_enqueue_ms": sorted(host), "synced_ms": sorted(full)}))

    net.eval()
    for (b, h, w, tag) in ((B, S, S, "eval_bs16_256"), (1, 512, 768, "eval_kodak_768x512")):
        xe = torch.rand(b, 3, h, w, device=dev)
        with torch.no_grad():
            for _ in range(2):
                net.forward_device(xe, xe, 0.0)
            torch.cuda.synchronize()
            ts, hs = [], []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                net.forward_device(xe, xe, 0.0)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
                hs.append((t1 - t0) * 1e3)
        ms = min(ts)
        print(json.dumps({"what": tag, "ms": round(ms, 3), "host_enqueue_ms": round(min(hs), 3),
                          "mpix_s": round(b * h * w / ms / 1e3, 3)}))


if __name__ == "__main__":
    main()
