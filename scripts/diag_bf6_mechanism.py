"""Signature of the bf16x6 cross-kernel interference (DESIGN §4 "Cross-kernel interference").

The library's conv3x3_wres_bf6_kernel runs on the main stream in its DIAGNOSTIC unguarded build (hyres_conv_tuning
key 9 = 0: 224 VGPRs per wave, a 64-register hole per SIMD) or its default guarded one (256), while a side stream
runs victims against their results computed alone:
  * the library's bilinear x1/2 resize (bilinear_fwd_kernel<4,false>: packed-fp32 VALU, v_pk_mul_f32 / v_pk_fma_f32),
  * torch elementwise kernels (a + b, a * 0.25 + b * 0.75, and a copy).
For every wrong bilinear output it records the wave position: the kernel's thread i = ow * 16 + c / 4 of its output
row, lane = i % 64, so one 16-lane group (one pass of the 16-wide SIMD over a wave64 instruction) = the 16 channel
groups of one output pixel; which float4 component (c % 4) is wrong; and which of the four 0.25-weighted source taps
the error equals (+tap: the tap counted twice, -tap: the tap lost).

    python scripts/diag_bf6_mechanism.py [reps] [--guarded]
"""
import os
import sys
from collections import Counter

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "hyres-residual-enhanced-hybrid-image-compression_amd"))

from hyres_hip import _lib as L  # noqa: E402
from hyres_hip import ops as O  # noqa: E402
from hyres_hip import refine_ops as R  # noqa: E402


def main(argv):
    reps = int(argv[0]) if argv and argv[0].isdigit() else 20
    guarded = "--guarded" in argv
    lib = L.load()
    lib.hyres_conv_tuning(7, 1, None)  # bf16x6
    lib.hyres_conv_tuning(9, 1 if guarded else 0, None)
    D = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(71)
    B, H, W, C = 2, 256, 256, 64
    feat = O.to_nhwc((torch.rand((B, C, H, W), generator=g) * 2 - 1).to(D))
    other = O.to_nhwc((torch.rand((B, C, H, W), generator=g) * 2 - 1).to(D))
    w = torch.nn.Parameter(((torch.rand((C, C, 3, 3), generator=g) * 2 - 1) * (C * 9) ** -0.5).to(D))
    b = ((torch.rand((C,), generator=g) * 2 - 1) * 0.1).to(D)
    slope = torch.full((1,), 0.25, device=D)
    ta = (torch.rand((4 << 20,), generator=g) * 2 - 1).to(D)
    tb = (torch.rand((4 << 20,), generator=g) * 2 - 1).to(D)
    side = torch.cuda.Stream(device=D)

    def conv():
        return O.conv2d(None, feat, w, b, pad=1, act=L.ACT_PRELU, slope=slope)

    def victims():
        return [R.bilinear(None, other, H // 2, W // 2, 2.0, 2.0).v for _ in range(3)] + \
               [ta + tb, ta * 0.25 + tb * 0.75, ta.clone()]

    names = ["bilinear#1", "bilinear#2", "bilinear#3", "torch a+b", "torch a*.25+b*.75", "torch copy"]
    with torch.no_grad():
        y0 = conv().v.clone()
        ref = [t.clone() for t in victims()]
        torch.cuda.synchronize()
        src = other.v  # [B, H, W, C] NHWC
        wrong = Counter()
        reps_hit = Counter()
        conv_bad = 0
        events = []  # (rep, victim, b, oh, ow) -> components, taps
        for r in range(reps):
            fork = torch.cuda.Event()
            fork.record()
            y = conv()
            side.wait_event(fork)
            with torch.cuda.stream(side):
                got = victims()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            conv_bad += int((y.v != y0).sum())
            for k, (gv, rv) in enumerate(zip(got, ref)):
                bad = (gv != rv)
                n = int(bad.sum())
                if not n:
                    continue
                wrong[names[k]] += n
                reps_hit[names[k]] += 1
                if k >= 3:
                    continue
                idx = bad.nonzero().tolist()  # [b, oh, ow, c]
                by_px = {}
                for bb, oh, ow, c in idx:
                    err = float(gv[bb, oh, ow, c] - rv[bb, oh, ow, c])
                    taps = [float(src[bb, 2 * oh + dy, 2 * ow + dx, c]) for dy in (0, 1) for dx in (0, 1)]
                    m = "other"
                    for t, tv in enumerate(taps):
                        if abs(abs(err) - 0.25 * abs(tv)) < 1e-6 * max(1.0, abs(tv)):
                            m = f"{'+' if err * tv > 0 else '-'}tap{t}"
                    by_px.setdefault((bb, oh, ow), []).append((c, m))
                for (bb, oh, ow), lst in by_px.items():
                    events.append((r, k, bb, oh, ow, lst))
    print(f"unguarded={not guarded} reps={reps}: conv output changed in {conv_bad} elements")
    for nm in names:
        print(f"  {nm:20s} wrong {wrong[nm]:8d} in {reps_hit[nm]:3d}/{reps} reps")
    if events:
        lanes = Counter(len(e[5]) for e in events)
        comps = Counter(c % 4 for e in events for c, _ in e[5])
        cgroups = Counter(len({c // 4 for c, _ in e[5]}) for e in events)
        taps = Counter(m for e in events for _, m in e[5])
        lanegrp = Counter(e[4] % 4 for e in events)
        print(f"  bilinear events (one output pixel = one 16-lane group of a wave): {len(events)}")
        print(f"    wrong elements per event: {dict(sorted(lanes.items()))}")
        print(f"    distinct lanes (channel groups) per event: {dict(sorted(cgroups.items()))}")
        print(f"    float4 component (c % 4): {dict(sorted(comps.items()))}")
        print(f"    error = 0.25 x tap: {dict(sorted(taps.items()))}")
        print(f"    16-lane group within the wave (ow % 4): {dict(sorted(lanegrp.items()))}")
        for e in events[:12]:
            print(f"    rep {e[0]} {names[e[1]]} b{e[2]} oh {e[3]} ow {e[4]}: " +
                  ", ".join(f"c{c}:{m}" for c, m in sorted(e[5])[:8]) + (" ..." if len(e[5]) > 8 else ""))
    lib.hyres_conv_tuning(9, 1, None)


if __name__ == "__main__":
    main(sys.argv[1:])
