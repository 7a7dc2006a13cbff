"""Sweep the forward-conv tile / split-K choice and the weight-gradient split plan (hyres_conv_tuning) over
the C2 step's small-grid geometries.

    python scripts/tile_sweep.py [--iters 30] [--f16] [--wgrad]
For each geometry: the heuristic's time, then every candidate; HIP-event timed (forward: fused epilogue;
--wgrad: weight + bias gradient incl. the split-K reduce).
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"))

import torch  # noqa: E402

# (H, Ci, Co, K, stride, res): 32^2 region of g_a/g_s AttentionBlock(192), h_a/h_s, param_aggregation,
# plus their dgrad shapes (a dgrad of Ci->Co is a Co->Ci conv) and two 64^2 / 128^2 references
GEOMS = [
    (32, 96, 96, 3, 1, False),
    (32, 192, 96, 1, 1, False),
    (32, 96, 192, 1, 1, True),
    (32, 768, 640, 1, 1, False),
    (32, 640, 512, 1, 1, False),
    (32, 512, 384, 1, 1, False),
    (32, 384, 512, 1, 1, False),
    (32, 192, 384, 3, 1, False),
    (32, 384, 192, 3, 1, False),
    (32, 192, 128, 3, 1, False),
    (64, 64, 64, 3, 1, False),
    (64, 128, 64, 1, 1, False),
    (64, 64, 128, 1, 1, True),
    (128, 128, 64, 1, 1, False),
    (128, 64, 128, 1, 1, True),
]
# weight gradients (H, Ci, Co, K[, stride]): P = dY [.., Co], Q = X [.., Ci]
WGEOMS = [
    (32, 96, 96, 3), (32, 96, 192, 1), (32, 192, 96, 1), (32, 192, 384, 5), (32, 192, 384, 3),
    (32, 768, 640, 1), (32, 512, 384, 1), (64, 64, 64, 3), (64, 128, 64, 1), (128, 64, 64, 3), (256, 64, 64, 3),
]
# the image-side 3-channel layers (refine conv 3->64 / 64->3 at 256^2, g_a's 5x5 s2 3->128)
WGEOMS3 = [(256, 3, 64, 3, 1), (256, 64, 3, 3, 1), (256, 3, 128, 5, 2)]
TILES = [0, 1, 2, 3, 4]
SPLITS = [0, 512, 1024, 2048]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--f16", action="store_true")
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--wgrad", action="store_true")
    ap.add_argument("--three", action="store_true", help="--wgrad over the 3-channel layers, incl. max split")
    a = ap.parse_args()
    if a.wgrad:
        return sweep_wgrad(a)
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    lib = L.load()
    dev = torch.device("cuda:0")

    def tune(k, v):
        L.check(lib.hyres_conv_tuning(k, v, None), "tuning")

    def timeit(x, w, b, res, K, s):
        ctx = torch.autocast("cuda", dtype=torch.float16) if a.f16 else torch.autocast("cuda", enabled=False)
        with ctx:
            y = O.conv2d(None, x, w, b, stride=s, pad=K // 2, act=L.ACT_RELU, res=res)
            for _ in range(2):
                y = O.conv2d(None, x, w, b, stride=s, pad=K // 2, act=L.ACT_RELU, res=res, out=y)
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                y = O.conv2d(None, x, w, b, stride=s, pad=K // 2, act=L.ACT_RELU, res=res, out=y)
            e1.record()
        torch.cuda.synchronize()
        return 1000 * e0.elapsed_time(e1) / a.iters

    geoms = [(256, 3, 64, 3, 1, False), (256, 3, 128, 5, 2, False)] if a.three else GEOMS
    for H, Ci, Co, K, s, r in geoms:
        x = O.Node(torch.randn(a.B, H, H, Ci, device=dev), rg=False)
        w = torch.randn(Co, Ci, K, K, device=dev) / (Ci * K * K) ** 0.5
        b = torch.randn(Co, device=dev)
        res = O.Node(torch.randn(a.B, H // s, H // s, Co, device=dev), rg=False) if r else None
        tune(0, -1), tune(1, -1)
        base = timeit(x, w, b, res, K, s)
        flops = 2.0 * a.B * (H // s) ** 2 * K * K * Ci * Co
        rows = []
        for t in TILES:
            for sp in SPLITS:
                tune(0, t)
                tune(1, sp if sp else 0)
                rows.append((timeit(x, w, b, res, K, s), t, sp))
        tune(0, -1), tune(1, -1)
        rows.sort()
        best = rows[0]
        print(f"B{a.B} {H}x{H}x{Ci}->{Co} K{K}{' +res' if r else ''}{' f16' if a.f16 else ''}: heuristic {base:.1f} us "
              f"({flops / base / 1e6:.1f} TF/s) | best tile {best[1]} split {best[2]}: {best[0]:.1f} us "
              f"({flops / best[0] / 1e6:.1f} TF/s) | top3 " +
              " ".join(f"t{t}/s{sp}:{us:.1f}" for us, t, sp in rows[:3]), flush=True)


def sweep_wgrad(a):
    import ctypes
    from hyres_hip import _lib as L
    lib = L.load()
    dev = torch.device("cuda:0")

    def tune(k, v):
        L.check(lib.hyres_conv_tuning(k, v, None), "tuning")

    for geom in (WGEOMS3 if a.three else WGEOMS):
        H, Ci, Co, K = geom[:4]
        st = geom[4] if len(geom) > 4 else 1
        d = L.WgradDesc()
        L.check(lib.hyres_wgrad_desc_conv2d(ctypes.byref(d), a.B, H, H, Ci, Ci, Co, Co, K, K, st, K // 2, 1), "desc")
        d.f16_operands = int(a.f16)
        Ho = (H + 2 * (K // 2) - K) // st + 1
        P = torch.randn(a.B, Ho, Ho, Co, device=dev)
        Q = torch.randn(a.B, H, H, Ci, device=dev)
        dst = torch.zeros(Co, Ci, K, K, device=dev)
        db = torch.zeros(Co, device=dev)

        def timeit():
            nb = lib.hyres_wgrad_workspace_bytes(ctypes.byref(d))
            ws = torch.empty(max(nb, 16) // 4 + 4, device=dev)
            args = (ctypes.byref(d), P.data_ptr(), Q.data_ptr(), dst.data_ptr(), db.data_ptr(), ws.data_ptr(),
                    ws.numel() * 4, L.stream())
            for _ in range(2):
                L.check(lib.hyres_conv_wgrad(*args), "wgrad")
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                lib.hyres_conv_wgrad(*args)
            e1.record()
            torch.cuda.synchronize()
            return 1000 * e0.elapsed_time(e1) / a.iters

        for k in (3, 4, 5, 6):
            tune(k, -1)
        base = timeit()
        rows = []
        if a.three:
            for tb in (2048, 8192, 32768):
                for mc in (2, 4, 8):
                    for msx in (512, 2048, 8192):
                        tune(3, tb), tune(4, mc), tune(6, msx)
                        rows.append((timeit(), tb, mc, msx))
        else:
            for tb in (1024, 2048, 4096):
                for mc in (2, 4, 8):
                    for nt in (-1, 1):
                        tune(3, tb), tune(4, mc), tune(5, nt)
                        rows.append((timeit(), tb, mc, nt))
        for k in (3, 4, 5, 6):
            tune(k, -1)
        rows.sort()
        flops = 2.0 * a.B * Ho * Ho * K * K * Ci * Co
        us, tb, mc, nt = rows[0]
        print(f"WGRAD B{a.B} {H}x{H} {Ci}->{Co} K{K}{' f16' if a.f16 else ''}: heuristic {base:.1f} us "
              f"({flops / base / 1e6:.1f} TF/s) | best blocks {tb} minchunks {mc} {'maxsplit' if a.three else 'nt'} {nt}: {us:.1f} us "
              f"({flops / us / 1e6:.1f} TF/s) | top3 " +
              " ".join(f"b{b}/c{c}/n{n}:{u:.1f}" for u, b, c, n in rows[:3]), flush=True)


if __name__ == "__main__":
    main()
