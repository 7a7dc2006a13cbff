"""Microbenchmark one conv geometry (forward, fused epilogue) with HIP events; for PMC passes.

    python scripts/conv_micro.py [--B 16 --H 128 --Ci 64 --Co 64 --K 3 --stride 1 --iters 50]
"""
import argparse
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
    ap.add_argument("--Co", type=int, default=64)
    ap.add_argument("--K", type=int, default=3)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--dil", type=int, default=1)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--relu", action="store_true")
    ap.add_argument("--res", action="store_true", help="fused residual add (RU / RBB tail)")
    ap.add_argument("--mask", action="store_true",
                    help="1x1 with the ReLU-mask epilogue (the input-gradient into a ReLU output), fp32 only")
    ap.add_argument("--f16", action="store_true", help="fp16 operands (autocast)")
    ap.add_argument("--tile", type=int, default=-1, help="force a conv tile (hyres_conv_tuning key 0)")
    ap.add_argument("--bf6", action="store_true", help="fp32 GEMM on the bf16 MFMA (hyres_conv_tuning key 7; default here: native)")
    ap.add_argument("--io16", action="store_true", help="fp16 activations in HBM (X, Y, residual; implies --f16)")
    ap.add_argument("--no-stream-h", action="store_true", help="fp16 1x1 on the tiled kernel (hyres_conv_tuning key 8 = 0)")
    ap.add_argument("--no-stream-b6", action="store_true",
                    help="bf16x6 fp32 1x1 on the tiled kernel (hyres_conv_tuning key 10 = 0)")
    ap.add_argument("--stream-cm", type=int, default=1,
                    help="streaming bf16x6 1x1 access mode (hyres_conv_tuning key 11: 0 MFMA layout, 1 LDS-staged epilogue)")
    ap.add_argument("--deconv", action="store_true", help="compressai deconv (ConvTranspose2d k5 s2 p2 op1, 4 phases)")
    ap.add_argument("--wres-v", type=int, default=0, help="conv3x3_wres_bf6_kernel variant (hyres_conv_tuning key 12)")
    a = ap.parse_args()
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    if a.tile >= 0:
        L.call("hyres_conv_tuning", 0, a.tile, None)
    L.call("hyres_conv_tuning", 7, 1 if a.bf6 else 0, None)  # the native fp32 MFMA unless --bf6
    L.call("hyres_conv_tuning", 8, 0 if a.no_stream_h else 1, None)
    L.call("hyres_conv_tuning", 10, 0 if a.no_stream_b6 else 1, None)
    L.call("hyres_conv_tuning", 11, a.stream_cm, None)
    L.call("hyres_conv_tuning", 12, a.wres_v, None)
    if a.io16:
        a.f16 = True
    dev = torch.device("cuda:0")
    adt = torch.float16 if a.io16 else torch.float32
    x = O.Node(torch.randn(a.B, a.H, a.H, a.Ci, device=dev).to(adt), rg=False)
    w = torch.randn(a.Co, a.Ci, a.K, a.K, device=dev) / (a.Ci * a.K * a.K) ** 0.5
    b = torch.randn(a.Co, device=dev)
    act = L.ACT_RELU if a.relu else L.ACT_NONE
    res = O.Node(torch.randn(a.B, a.H // a.stride, a.H // a.stride, a.Co, device=dev).to(adt), rg=False) if a.res else None
    if a.mask:  # low-level launch: the mask operand (a ReLU output) rides in aux0, as ops.relu_mask_epilogue sets it
        assert a.K == 1 and not a.io16
        yo = torch.relu(torch.randn(a.B, a.H, a.H, a.Co, device=dev))
        y = torch.empty(a.B, a.H, a.H, a.Co, device=dev)
        g = O._geom("hyres_geom_conv2d", a.B, a.H, a.H, a.Ci, a.Ci, a.Co, a.Co, 1, 1, 1, 0, 1)
        e = L.Epilogue()
        e.kind = L.EPI_BIAS
        e.act = L.ACT_RELU_MASK
        e.aux0, e.ld0 = yo.data_ptr(), a.Co
        for _ in range(3):
            O._launch_conv(g, x.ptr(), w.view(a.Co, a.Ci), a.Ci, y.data_ptr(), e)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            O._launch_conv(g, x.ptr(), w.view(a.Co, a.Ci), a.Ci, y.data_ptr(), e)
        e1.record()
        torch.cuda.synchronize()
        us = 1000 * e0.elapsed_time(e1) / a.iters
        byts = 4.0 * a.B * a.H * a.H * (a.Ci + 2 * a.Co)
        print(f"conv B{a.B} {a.H}x{a.H}x{a.Ci} -> {a.H}x{a.H}x{a.Co} K1 +mask{' bf16x6' if a.bf6 else ''}: {us:.1f} us, "
              f"{2.0 * a.B * a.H * a.H * a.Ci * a.Co / us / 1e6:.1f} TFLOP/s, {byts / us / 1e3:.0f} GB/s")
        return
    if a.deconv:
        wd = torch.randn(a.Ci, a.Co, 5, 5, device=dev) / (a.Ci * 25) ** 0.5
        for _ in range(3):
            y = O.deconv2d(None, x, wd, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            y = O.deconv2d(None, x, wd, b, out=y)
        e1.record()
        torch.cuda.synchronize()
        us = 1000 * e0.elapsed_time(e1) / a.iters
        flops = 2.0 * a.B * a.H * a.H * 25 * a.Ci * a.Co
        print(f"deconv B{a.B} {a.H}x{a.H}x{a.Ci} -> {2 * a.H}x{2 * a.H}x{a.Co} K5{' bf16x6' if a.bf6 else ''}: {us:.1f} us, "
              f"{flops / us / 1e6:.1f} TFLOP/s")
        return
    ctx = torch.autocast("cuda", dtype=torch.float16) if a.f16 else torch.autocast("cuda", enabled=False)
    import contextlib
    with ctx, (O.f16_region() if a.io16 else contextlib.nullcontext()):
        for _ in range(3):
            y = O.conv2d(None, x, w, b, stride=a.stride, pad=a.dil * (a.K // 2), dil=a.dil, act=act, res=res)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            y = O.conv2d(None, x, w, b, stride=a.stride, pad=a.dil * (a.K // 2), dil=a.dil, act=act, res=res, out=y)
        e1.record()
    torch.cuda.synchronize()
    us = 1000 * e0.elapsed_time(e1) / a.iters
    Ho = y.H
    flops = 2.0 * a.B * Ho * Ho * a.K * a.K * a.Ci * a.Co
    es = 2.0 if a.io16 else 4.0
    byts = es * (a.B * a.H * a.H * a.Ci + a.B * Ho * Ho * a.Co * (2 if a.res else 1)) + 4.0 * a.K * a.K * a.Ci * a.Co
    print(f"conv B{a.B} {a.H}x{a.H}x{a.Ci} -> {Ho}x{Ho}x{a.Co} K{a.K} s{a.stride}{f' d{a.dil}' if a.dil > 1 else ''}{' +res' if a.res else ''}{' f16' if a.f16 else ''}{' io16' if a.io16 else ''}{' tiled' if a.no_stream_h or a.no_stream_b6 else ''}{f' cm{a.stream_cm}' if a.stream_cm != 1 else ''}{f' wres-v{a.wres_v}' if a.wres_v else ''}{' bf16x6' if a.bf6 else ''}: {us:.1f} us, "
          f"{flops / us / 1e6:.1f} TFLOP/s, {byts / us / 1e3:.0f} GB/s")


if __name__ == "__main__":
    main()
