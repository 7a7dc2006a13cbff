"""Microbenchmark one conv weight gradient (hyres_conv_wgrad: kernel + split reduce) with HIP events,
with and without the fused bias gradient.

    python scripts/wgrad_micro.py [--B 16 --H 128 --Ci 64 --Co 128 --K 1 --iters 30]
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--H", type=int, default=128)
    ap.add_argument("--Ci", type=int, default=64)
    ap.add_argument("--Co", type=int, default=128)
    ap.add_argument("--K", type=int, default=1)
    ap.add_argument("--dil", type=int, default=1)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--f16", action="store_true", help="AMP: fp16 operands (f16 MFMA)")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--ab", default=None, help="key=v1,v2: time each value of hyres_conv_tuning key and compare the "
                                               "gradients bit for bit (e.g. 15=1,2)")
    a = ap.parse_args()
    from hyres_hip import _lib as L
    dev = torch.device("cuda:0")
    x = torch.randn(a.B, a.H, a.H, a.Ci, device=dev)
    gy = torch.randn(a.B, a.H // a.stride, a.H // a.stride, a.Co, device=dev)
    dw = torch.zeros(a.Co, a.Ci, a.K, a.K, device=dev)
    db = torch.zeros(a.Co, device=dev)
    d = L.WgradDesc()
    L.call("hyres_wgrad_desc_conv2d", ctypes.byref(d), a.B, a.H, a.H, a.Ci, a.Ci, a.Co, a.Co, a.K, a.K, a.stride, a.dil * (a.K // 2), a.dil)
    d.f16_operands = int(a.f16)
    d.sm = a.Ci * a.K * a.K
    nb = L.load().hyres_wgrad_workspace_bytes(ctypes.byref(d))
    ws = torch.empty(nb // 4 + 16, device=dev)
    if a.ab:
        key, vals = a.ab.split("=")
        res = {}
        for v in vals.split(","):
            L.call("hyres_conv_tuning", int(key), int(v), None)

            def run():
                dw.zero_()
                db.zero_()
                L.call("hyres_conv_wgrad", ctypes.byref(d), gy.data_ptr(), x.data_ptr(), dw.data_ptr(), db.data_ptr(),
                       ws.data_ptr(), nb, L.stream())
            for _ in range(10):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = 1000 * e0.elapsed_time(e1) / a.iters
            res[v] = (dw.clone(), db.clone())
            byts = 4.0 * a.B * a.H * a.H * (a.Ci + a.Co)
            print(f"wgrad key{key}={v} B{a.B} {a.H}^2 {a.Ci}->{a.Co} K{a.K} d{a.dil} bias=1: {us:.1f} us, "
                  f"{byts / us / 1e3:.0f} GB/s (incl. zeroing)")
        vs = list(res.values())
        same = all(torch.equal(r[0], vs[0][0]) and torch.equal(r[1], vs[0][1]) for r in vs[1:])
        print(f"wgrad key{key} variants bit-identical: {same}")
        return
    for bias in (False, True):
        def run():
            L.call("hyres_conv_wgrad", ctypes.byref(d), gy.data_ptr(), x.data_ptr(), dw.data_ptr(),
                   db.data_ptr() if bias else None, ws.data_ptr(), nb, L.stream())
        for _ in range(10):  # (3 left the first-measured configuration ~10 % slow: clock ramp)
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = 1000 * e0.elapsed_time(e1) / a.iters
        flops = 2.0 * a.B * a.H * a.H * a.K * a.K * a.Ci * a.Co
        byts = 4.0 * a.B * a.H * a.H * (a.Ci + a.Co)
        print(f"wgrad{' f16' if a.f16 else ''} B{a.B} {a.H}^2 {a.Ci}->{a.Co} K{a.K} d{a.dil} bias={int(bias)}: {us:.1f} us, {flops / us / 1e6:.1f} TFLOP/s, "
              f"{byts / us / 1e3:.0f} GB/s")


if __name__ == "__main__":
    main()
