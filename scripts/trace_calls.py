"""List the launches of one eager C2 train step (bs16 256x256) that call the given C-ABI entry points, with
the model call site and size of each, to find gradient adds / elementwise passes that could be fused away.

    python3 scripts/trace_calls.py [--fn hyres_add2d --fn hyres_prelu_bwd] [--batch 16 --size 256]
"""
import argparse
import collections
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"), REPO]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fn", action="append", default=None)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    args = ap.parse_args()
    fns = set(args.fn or ["hyres_add2d", "hyres_prelu_bwd", "hyres_relu_bwd_2d"])
    from hyres_hip import _lib as L
    from hyres_hip.loss import RateDistortionLoss
    from hyres_hip.weights import synthetic_state_dict
    from models import ResidualJPEGCompression
    dev = torch.device("cuda:0")
    net = ResidualJPEGCompression(jpeg_quality=50)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(dev).train()
    g = torch.Generator().manual_seed(1926)
    x_cpu = torch.randint(0, 256, (args.batch, 3, args.size, args.size), generator=g).float() / 255
    jpeg, bpp = net.jpeg(x_cpu)
    x, jpeg = x_cpu.to(dev), jpeg.to(dev)
    crit = RateDistortionLoss(lmbda=0.045, alpha=0)
    seen = collections.Counter()
    orig = L.call

    def call(fn, *a):
        if fn in fns:
            st = [f for f in traceback.extract_stack()[:-1] if "hyres_hip" in f.filename or "models" in f.filename]
            site = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in reversed(st[-4:]))
            ints = [v for v in a if isinstance(v, int) and v < (1 << 32)]
            seen[(fn, site, tuple(ints[:6]))] += 1
        return orig(fn, *a)

    L.call = call
    out = net.forward_device(x, jpeg, torch.full((), float(bpp), device=dev), False)
    c = crit(out, x)
    c["loss"].backward()
    torch.cuda.synchronize()
    L.call = orig
    for (fn, site, ints), n in sorted(seen.items(), key=lambda kv: kv[0][1]):
        print(f"{n:3d}x {fn} ints={ints}  {site}")


if __name__ == "__main__":
    main()
