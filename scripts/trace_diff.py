"""Stage-by-stage comparison of the HIP forward (eval) against the oracle at a given image size.

    python scripts/trace_diff.py --H 128 --W 192
Prints the normwise relative error of every traced activation (models' Trace hooks vs oracle trace).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=128)
    ap.add_argument("--W", type=int, default=192)
    ap.add_argument("--B", type=int, default=1)
    a = ap.parse_args()
    from helpers import build_model, oracle_from, recipe_state_dict
    from hyres_hip import ops as O
    net, _ = build_model()
    dev = torch.device("cuda:0")
    net = net.to(dev).eval()
    g = torch.Generator().manual_seed(7)
    base = F.interpolate(torch.rand(a.B, 3, max(a.H // 32, 1), max(a.W // 32, 1), generator=g), size=(a.H, a.W),
                         mode="bilinear", align_corners=False)
    x = ((base * 0.8 + 0.2 * torch.rand(a.B, 3, a.H, a.W, generator=g)) * 255).floor() / 255
    jpeg, jb = net.jpeg(x)
    O.Trace.nodes = {}
    with torch.no_grad():
        out = net(x, jpeg=(jpeg, jb))
    torch.cuda.synchronize()
    hip = {k: O.Trace.value(k).cpu() for k in O.Trace.nodes}
    O.Trace.nodes = None
    orc, _ = oracle_from(recipe_state_dict())
    T = {}
    with torch.no_grad():
        ref = orc.forward(x, jpeg, float(jb), training=False, trace=T)
    T["x_hat"] = ref["x_hat"]
    for k in sorted(hip):
        if k not in T:
            print(f"{k:24s} (no oracle trace)")
            continue
        h, r = hip[k].double(), T[k].double()
        if h.shape != r.shape:
            print(f"{k:24s} shape {tuple(h.shape)} vs {tuple(r.shape)}")
            continue
        err = float((h - r).abs().max() / r.abs().max().clamp_min(1e-30))
        print(f"{k:24s} {err:.3e}  {tuple(h.shape)}")
    e = float((out["x_hat"].cpu() - ref["x_hat"]).abs().max())
    print("x_hat max abs err", e)


if __name__ == "__main__":
    main()
