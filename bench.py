"""HyRES residual-codec hot path on MI355X: training-step throughput (BASELINE.json configs[1]).

One step = the C2 workload: N=128 M=192 ResidualJPEGCompression, bs=16 synthetic 256x256 RGB per GPU,
train mode (noisequant=False), forward (residual -> LightWeightCheckerboard -> MultiScaleRefine -> clamp)
+ RateDistortionLoss(lambda=0.045) + backward + clip_grad_norm(1.0) + Adam + aux (quantiles) Adam step,
every kernel from libhyres_hip.  JPEG (a host CPU stage) is precomputed before the timed region so the
inputs are resident in HBM; its host cost is reported separately (``jpeg_host_ms_per_image``).
Metric: Mpixels/s = B*H*W*world / step time (whole job).  Multi-GPU: one process per GPU, batches
shard over ranks (weak scaling), gradients all-reduced over RCCL (hyres_hip.ddp).

    python bench.py [--gpus N --steps K --warmup W]
"""
from __future__ import annotations

import argparse
import ctypes
import faulthandler
import json
import math
import os
import sys
import time

# a host-side crash prints the Python stacks of every thread to stderr (DESIGN §13 "Open")
faulthandler.enable()

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, REPO)

import torch  # noqa: E402

MI355X_FP32_PEAK_TFLOPS = 157.3  # dense fp32 (vector == matrix), MI355X_MICROARCH.md
MI355X_HBM_TBPS = 8.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--lmbda", type=float, default=0.045)
    ap.add_argument("--jpeg-quality", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0)
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of HIP-graph replay")
    ap.add_argument("--no-eval", action="store_true", help="skip the encode+decode (eval) legs")
    ap.add_argument("--no-host-jpeg", action="store_true", help="skip the with-host-JPEG legs")
    ap.add_argument("--no-amp", action="store_true", help="skip the f16-amp (train.sh --mixed-precision) leg")
    ap.add_argument("--jpeg-procs", type=int, default=None, help="JPEG worker processes (default min(8, cpus))")
    ap.add_argument("--fp32-gemm", choices=["default", "native", "bf16x6"], default="default",
                    help="fp32 conv GEMMs: the native fp32 MFMA or the bf16x6 split (hyres_conv_tuning key 7)")
    return ap.parse_args()


def cpu_baseline(args, budget_s):
    """The oracle (torch-CPU fp32 restatement of the reference hot path, oracle/ — ``kind: port``) on the
    host cores: the same train step (fwd + RD loss + bwd) on a bounded sample (batch 2 at 256x256, the JPEG
    stage's real output as input), timed with mkldnn on and off (the reference's src/training.py:7-9 turns
    it off)."""
    from oracle import Oracle, rd_loss
    from hyres_hip.weights import synthetic_state_dict
    from models import ResidualJPEGCompression
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    net = ResidualJPEGCompression(jpeg_quality=args.jpeg_quality)
    sd = synthetic_state_dict(net.state_dict())
    for k, v in sd.items():
        if v.is_floating_point() and not k.endswith(("pedestal", "bound", "mask", "target", "scale_bound")):
            v.requires_grad_(True)
    orc = Oracle(sd)
    B, S = 2, args.size
    g = torch.Generator().manual_seed(1926)
    x = torch.randint(0, 256, (B, 3, S, S), generator=g).float() / 255
    jpeg, jpeg_bpp = net.jpeg(x)
    noise = {"z": torch.rand(B, 128, S // 32, S // 32) - 0.5, "y": torch.rand(B, 192, S // 8, S // 8) - 0.5}
    res = {}
    for tag, mk in (("mkldnn_on", True), ("mkldnn_off", False)):
        prev = torch.backends.mkldnn.enabled
        torch.backends.mkldnn.enabled = mk
        times = []
        t_end = time.time() + budget_s / 2
        try:
            while True:
                t0 = time.time()
                out = orc.forward(x, jpeg, jpeg_bpp, training=True, noisequant=False, noise=noise)
                crit = rd_loss(out, x, args.lmbda)
                crit["loss"].backward()
                times.append(time.time() - t0)
                if time.time() > t_end or len(times) >= 10:
                    break
        finally:
            torch.backends.mkldnn.enabled = prev
        t = min(times[1:]) if len(times) > 1 else times[0]
        res[tag] = {"value": round(B * S * S / t / 1e6, 4), "steps": len(times)}
    # configs[0] (C1): the reference's CPU forward only, one 256x256 image, eval (models/hyres.py:23-77)
    x1, j1 = x[:1], jpeg[:1]
    c1 = []
    with torch.no_grad():
        for _ in range(4):
            t0 = time.time()
            orc.forward(x1, j1, jpeg_bpp, training=False)
            c1.append(time.time() - t0)
    t1 = min(c1[1:])
    return {"value": res["mkldnn_on"]["value"], "unit": "Mpixels/s", "cores": threads, "kind": "port",
            "value_mkldnn_off": res["mkldnn_off"]["value"],
            "c1_eval_forward": {"ms": round(1000 * t1, 1), "mpix_s": round(S * S / t1 / 1e6, 4),
                                "sample": f"configs[0]: oracle eval forward, 1x3x{S}x{S}, min over 3 runs after one "
                                          f"warm-up, {threads} threads"},
            "sample": f"oracle (torch-CPU fp32 port of the reference math) train step (fwd+RD loss+bwd) at batch "
                      f"{B}x{S}x{S} on the JPEG stage's output, min over {res['mkldnn_on']['steps']} / "
                      f"{res['mkldnn_off']['steps']} steps with mkldnn on / off, {threads} threads; the reference "
                      f"itself cannot run here (compressai absent)"}


# scripts/check.sh <tag> pmc: the fp32 line's dominant kernel, and the AMP leg's dominant kernel from the same passes;
# committed PMC summaries, newest first: the first one collected for the kernel being priced is used
# (r7w: the final round-6 build after the late folds; r6x: the round-6 build before them; r6o: an earlier round-6 build, the D = 1 weight-resident launches; r5f: the bf16x6 weight-resident conv incl. its dilation-2 launches; r5s: before those; r4i: its round-4 build;
# r4b: the native fp32 one)
PMC_TRAFFIC = [os.path.join(REPO, "profiles", f) for f in
               os.environ.get("HYRES_PMC_TRAFFIC",
                              "r7w_pmc_traffic.json,r6x_pmc_traffic.json,r6o_pmc_traffic.json,r5f_pmc_traffic.json,r5s_pmc_traffic.json,r4i_pmc_traffic.json,r4b_pmc_traffic.json").split(",")]
PMC_TRAFFIC_AMP = [os.path.join(REPO, "profiles", f) for f in
                   os.environ.get("HYRES_PMC_TRAFFIC_AMP", "r7w_pmc_traffic_amp.json,r6x_pmc_traffic_amp.json,r6o_pmc_traffic_amp.json,r5f_pmc_traffic_amp.json,r5s_pmc_traffic_amp.json").split(",")]
EAGER_TIMED = 3  # eager steps behind the live per-launch roofline timing
# N > 1 default: the graphed step cut at the "hyper" marker with the finished segments' all-reduce between the two
# replays; HYRES_DIST_MODE=graph+allreduce (reduce after one replay) / eager-overlap select the others
DIST_DEFAULT = "graph+overlap"
SPLIT_AT = ("hyper",)


# bf16x6 (csrc/conv.hip bf6_mfma): each fp32 product from six bf16 MFMA products -> the fp32-equivalent ceiling of
# a bf16x6 kernel is the dense bf16 MFMA peak / 6
MI355X_BF16_PEAK_TFLOPS = 2500.0
BF6_PEAK_TFLOPS = MI355X_BF16_PEAK_TFLOPS / 6
FP32_GEMM_NOTE = {
    "bf16x6": "fp32 conv GEMMs on the bf16 MFMA: each fp32 operand split into three bf16 pieces (24 significant bits), "
              "the six cross products with i + j <= 2 accumulated in fp32 — per-product error ~2^-25 relative, below "
              "the fp32 MFMA's own 2^-24 rounding; measured error vs fp64 equal to the native fp32 kernel's "
              "(tests/test_bf6_gpu.py) and the fp32 parity suite / C2 fp64-oracle test pass unchanged with it. "
              "The reference's own fp32 convs run with PyTorch's default cudnn.allow_tf32=True (10-bit mantissa "
              "operands) on its NVIDIA hardware. Covers forward, input-gradient and the halo-staged / 1x1 weight "
              "gradients (the generic tap-folded weight-gradient kernel stays on the fp32 MFMA).",
    "native": "fp32 conv GEMMs on the native fp32 MFMA (v_mfma_f32_32x32x2_f32)",
}


def kernel_peak(kernel):
    """The peak a kernel's fp32 flops are priced against: the bf16x6 ceiling for the bf16x6 kernels, else the dense
    fp32 MFMA peak."""
    return BF6_PEAK_TFLOPS if ("bf6" in kernel or "b6_kernel" in kernel or "b6db_kernel" in kernel) else MI355X_FP32_PEAK_TFLOPS


def peak_note(kernel):
    if kernel_peak(kernel) == BF6_PEAK_TFLOPS:
        return ("bf16x6 ceiling: 2500 TF/s dense bf16 MFMA / 6 bf16 products per fp32 product = 416.7 fp32-equivalent "
                "TF/s (frac_vs_native_fp32_peak: the same rate against the 157.3 TF/s fp32 MFMA)")
    return "dense fp32 MFMA peak"


def kernel_label(kernel):
    """What the dominant kernel is: the VALU narrow-output kernel (Co <= 4) and the streaming 1x1 kernel are
    not the implicit-GEMM tile kernel."""
    if kernel.startswith("conv_narrow"):
        return "narrow-output conv (Co <= 4), fp32 VALU FMA — not MFMA; priced against the MFMA peak as an upper bound"
    if kernel.startswith("conv1x1_stream"):
        if kernel.replace(" ", "").endswith(",true>"):
            return "streaming 1x1 conv, fp16-rounded operands on the fp32 MFMA (autocast), HBM-bound"
        return "streaming 1x1 conv, fp32 MFMA, weights resident in LDS"
    if kernel.startswith("conv3x3_wres_bf6"):
        return "weight-resident persistent 3x3 conv, fp32 via bf16x6 on the bf16 MFMA, split weights in LDS, halo tiles"
    if kernel.startswith("conv_fwd_b6"):
        return "implicit-GEMM conv, fp32 via bf16x6 on the bf16 MFMA, fused epilogue"
    if kernel.startswith("conv3x3_wres_f32"):
        return "weight-resident persistent 3x3 conv, fp32 MFMA, fp32 weights in LDS, halo tiles"
    if kernel.startswith("conv3x3_wres_f16"):
        return "weight-resident persistent 3x3 conv, f16 MFMA, fp16 halo tiles in LDS"
    if kernel.startswith("conv3x3_halo_f16"):
        return "halo-staged 3x3 conv, f16 MFMA"
    if kernel.startswith("conv_fwd_h_kernel"):
        io = kernel.replace(" ", "").rstrip(">").split(",")[-1]
        return (f"implicit-GEMM conv, f16 MFMA, fp16 activations in HBM (io {io}: bit 0 X, bit 1 Y/residual/aux), "
                "fused epilogue")
    if "true>" in kernel.replace(" ", "").split(",")[-1]:
        return "implicit-GEMM conv, f16 MFMA, fused epilogue"
    return "implicit-GEMM conv, fp32 MFMA, fused epilogue"


def traffic_bytes_per_launch(kernel, path=None):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC passes of this same
    command (scripts/pmc_traffic.py: 2 x FETCH_SIZE + WRITE_SIZE, separate passes, gfx950 FETCH_SIZE
    correction); None when that summary is absent or was collected for another kernel."""
    paths = path or PMC_TRAFFIC
    for p in [paths] if isinstance(paths, str) else paths:
        try:
            with open(p) as f:
                d = json.load(f)
            if kernel is not None and kernel in d["kernel"]:
                return d["traffic_bytes_per_launch"]
        except (OSError, KeyError, ValueError):
            pass
    return None


def eval_legs(net, x, jpeg, jpeg_bpp, args, reps=20):
    """Encode+decode (eval forward, SURVEY §8d: "Mpix/s = B*H*W / wall time of one step: forward (eval)
    for encode+decode") at the bench batch (configs[1] shape) and at Kodak size 768x512 (configs[4],
    fp32), device-only (JPEG precomputed), HIP-graph replay and eager."""
    from hyres_hip.graphs import CapturedStep
    net.eval()
    res = {}
    g = torch.Generator().manual_seed(1926)
    xk = torch.randint(0, 256, (1, 3, 512, 768), generator=g).float() / 255.0
    jk, bk = net.jpeg(xk)
    dev = x.device
    # C3's batch (bs=32): the bench batch twice, the second half mirrored (synthetic timing input)
    x2 = torch.cat([x, torch.flip(x, dims=[3])]).contiguous()
    j2 = torch.cat([jpeg, torch.flip(jpeg, dims=[3])]).contiguous()
    legs = (("bs%d_%dx%d" % (x.shape[0], x.shape[2], x.shape[3]), x, jpeg, jpeg_bpp),
            ("bs%d_%dx%d" % (x2.shape[0], x.shape[2], x.shape[3]), x2, j2, jpeg_bpp),
            ("kodak_1x768x512", xk.to(dev), jk.to(dev), bk))
    for tag, xe, je, be in legs:
        cap = CapturedStep(net, xe, je, be)
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(reps):
            cap.replay()
        torch.cuda.synchronize()
        ms = (time.time() - t0) * 1000 / reps
        with torch.no_grad():
            for _ in range(2):
                net.forward_device(xe, je, be)
            torch.cuda.synchronize()
            t0 = time.time()
            for _ in range(5):
                net.forward_device(xe, je, be)
            torch.cuda.synchronize()
        ems = (time.time() - t0) * 1000 / 5
        npx = xe.shape[0] * xe.shape[2] * xe.shape[3]
        res[tag] = {"ms": round(ms, 3), "mpix_s": round(npx / ms / 1e3, 3), "eager_ms": round(ems, 3)}
        cap.close()  # no replay output is held here (graphs.py lifetime rule)
        del cap
    # configs[4] precision: inference under torch.autocast(float16) -> fp16-operand f16 MFMA convs
    with torch.autocast("cuda", dtype=torch.float16):
        for tag, xe, je, be in [(t + "_autocast_f16", a, b, c) for t, a, b, c in legs]:
            cap = CapturedStep(net, xe, je, be)
            torch.cuda.synchronize()
            t0 = time.time()
            for _ in range(reps):
                cap.replay()
            torch.cuda.synchronize()
            ms = (time.time() - t0) * 1000 / reps
            npx = xe.shape[0] * xe.shape[2] * xe.shape[3]
            res[tag] = {"ms": round(ms, 3), "mpix_s": round(npx / ms / 1e3, 3)}
            cap.close()
            del cap
    # A/B of the fused ResidualUnit / RBB inference kernel (csrc/ru_fused.hip): the bench batch under autocast with
    # the three-conv chain instead
    from hyres_hip import ops as O
    O.RU_FUSED = False
    try:
        with torch.autocast("cuda", dtype=torch.float16):
            cap = CapturedStep(net, x, jpeg, jpeg_bpp)
            torch.cuda.synchronize()
            t0 = time.time()
            for _ in range(reps):
                cap.replay()
            torch.cuda.synchronize()
            ms = (time.time() - t0) * 1000 / reps
            cap.close()
            del cap
    finally:
        O.RU_FUSED = True
    res[legs[0][0] + "_autocast_f16_ru_unfused"] = {"ms": round(ms, 3), "mpix_s": round(x.shape[0] * x.shape[2] *
                                                                                       x.shape[3] / ms / 1e3, 3)}
    res["analysis_synthesis_bs%d" % x.shape[0]] = analysis_synthesis(net, x, reps)
    res["kodak_codec"] = codec_leg(net, xk.to(dev), jk.to(dev))
    # configs[4]: the same codec under autocast (fp16 MFMA operands, fp16 activations above the latent)
    with torch.autocast("cuda", dtype=torch.float16):
        res["kodak_codec_autocast_f16"] = codec_leg(net, xk.to(dev), jk.to(dev))
    net.train()
    return res


MI355X_F16_PEAK_TFLOPS = 2500.0  # dense f16 MFMA (MI355X_MICROARCH.md), no sparsity


def amp_leg(net, opt, aux_opt, crit, x, jpeg, jpeg_bpp, args):
    """train.sh's actual configuration (--mixed-precision, src/utils/engine.py:23-82): the C2 step under
    torch.autocast(float16) — every conv / deconv / GDN contraction and its input-gradient on the f16 MFMA
    (v_mfma_f32_32x32x16_f16, fp16 operands, fp32 accumulation; the f16_region's activations stored fp16 in
    HBM as autocast's conv outputs are, activation gradients fp32) —
    with the device GradScaler (scaled loss, unscale-before-clip, skip on inf/NaN, backoff/growth), as a HIP
    graph.  Reported beside the fp32 headline; dtype "f16-amp"."""
    from hyres_hip.graphs import CapturedStep
    from hyres_hip.optim import DeviceGradScaler
    from hyres_hip import ops as O
    dev = x.device
    scaler = DeviceGradScaler(dev)
    cap = CapturedStep(net, x, jpeg, jpeg_bpp, noisequant=False, criterion=crit, zero_grad=opt.zero_grad, amp=True,
                       loss_scale=scaler.scale)

    def step():
        c = cap.replay()[1]
        opt.step(grad_scaler=scaler)
        scaler.update(opt.sumsq)
        nan = opt.sumsq.clone()
        opt.zero_grad()
        aux = net.aux_loss()
        aux.backward()
        aux_opt.step(skip_if_nan=nan)
        aux_opt.zero_grad()
        return c

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(args.steps):
        c = step()
    torch.cuda.synchronize()
    ms = (time.time() - t0) * 1000 / args.steps
    loss = float(c["loss"].detach())
    c = None  # a replay output (graph pool): dropped before the graph is closed
    B, _, H, W = x.shape
    # dominant f16 kernel, live (one eager AMP step, HIP events per launch, as for the fp32 line)
    O.KernelTimer.reset()
    O.KernelTimer.enabled = True
    with torch.autocast("cuda", dtype=torch.float16):
        out = net.forward_device(x, jpeg, jpeg_bpp, noisequant=False)
        cc = crit(out, x)
    (cc["loss"] * scaler.scale.reshape(())).backward()
    torch.cuda.synchronize()
    O.KernelTimer.enabled = False
    ks = O.KernelTimer.summary()
    # the dominant f16-MFMA-bound kernel (intensity above the f16 ridge 2500 / 8 = 312 FLOP/B) as well
    ks_mfma = O.KernelTimer.summary(pick=lambda k, v: v[1] / max(v[2], 1.0) >= F16_RIDGE)
    opt.zero_grad()
    nrep = max(5, args.steps // 2)
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(nrep):
        cap.replay()
        opt.zero_grad()
    torch.cuda.synchronize()
    ms_a = (time.time() - t0) * 1000 / nrep
    del out, cc  # the eager step's outputs (regular pool) — nothing of the graph's is held now
    cap.close()
    del cap
    # round-4 A/B on the same box: the step with the unfused ResidualUnits, and with fp32 activation gradients and
    # the unfused ResidualUnits (round 3's AMP path) — the gains of the fused RU forward and of fp16 gradients
    def ab(f16_grad, ru_fused):
        saved = (O.AMP_F16_GRAD, O.RU_FUSED)
        O.AMP_F16_GRAD, O.RU_FUSED = f16_grad, ru_fused
        try:
            scaler_b = DeviceGradScaler(dev)
            cap_b = CapturedStep(net, x, jpeg, jpeg_bpp, noisequant=False, criterion=crit, zero_grad=opt.zero_grad,
                                 amp=True, loss_scale=scaler_b.scale)
            torch.cuda.synchronize()
            t0 = time.time()
            for _ in range(nrep):
                cap_b.replay()
                opt.zero_grad()
            torch.cuda.synchronize()
            ms_ab = (time.time() - t0) * 1000 / nrep
            cap_b.close()
            del cap_b
        finally:
            O.AMP_F16_GRAD, O.RU_FUSED = saved
        return ms_ab

    ms_u = ab(True, False)
    ms_b = ab(False, False)
    opt.zero_grad()
    return {"dtype": "f16-amp", "value": round(B * H * W / ms / 1e3, 4), "unit": "Mpixels/s", "ms_per_step": round(ms, 3),
            "fwd_bwd_ms": round(ms_a, 3), "ab_unfused_ru_fwd_bwd_ms": round(ms_u, 3),
            "ab_fp32_grads_unfused_ru_fwd_bwd_ms": round(ms_b, 3),
            "loss": loss, "loss_scale": scaler.get_scale(),
            "roofline": with_traffic(roofline_of(ks, MI355X_F16_PEAK_TFLOPS, F16_RIDGE), ks["kernel"]),
            "roofline_f16_mfma_kernel": roofline_of(ks_mfma, MI355X_F16_PEAK_TFLOPS, F16_RIDGE),
            "note": "fp16 operands / fp32 accumulation (f16 MFMA; the HBM-bound 1x1 layers on the fp32 MFMA with "
                    "fp16-rounded operands); weight gradients "
                    + ("f16" if os.environ.get("HYRES_AMP_WGRAD_F16", "1") == "1" else "fp32")}


def with_traffic(r, kernel):
    """The AMP leg's roofline entry with its PMC-measured HBM bytes per launch (profiles/r4i_pmc_traffic_amp.json)."""
    if r is not None:
        r["traffic"] = traffic_bytes_per_launch(kernel, PMC_TRAFFIC_AMP)
    return r


MI355X_HBM_PEAK_GBS = 8000.0
F16_RIDGE = MI355X_F16_PEAK_TFLOPS * 1e12 / (MI355X_HBM_PEAK_GBS * 1e9)


def roofline_of(ks, peak_tflops, ridge):
    """Roofline entry of a KernelTimer summary: MFMA-bound (TFLOP/s vs the dense peak) when its algorithmic
    intensity is above the ridge, else HBM-bound (algorithmic GB/s vs 8 TB/s)."""
    if not ks.get("kernel") or ks["total_ms"] <= 0:
        return None
    inten = ks["flops_per_launch"] / max(ks["bytes_per_launch"], 1.0)
    sec = ks["total_ms"] * 1e-3
    base = {"kernel": f"{ks['kernel']} ({kernel_label(ks['kernel'])})", "avg_launch_us": round(ks["avg_us"], 2),
            "launches_per_step": ks["launches"], "flops_per_launch": ks["flops_per_launch"],
            "algorithmic_bytes_per_launch": ks["bytes_per_launch"], "intensity_flop_per_byte": round(inten, 2)}
    if inten >= ridge:
        ach = ks["flops"] / sec / 1e12
        base.update(bound="mfma", achieved=round(ach, 3), peak=peak_tflops, unit="TFLOP/s",
                    frac=round(ach / peak_tflops, 4))
    else:
        ach = ks["bytes_per_launch"] * ks["launches"] / sec / 1e9
        base.update(bound="hbm", achieved=round(ach, 1), peak=MI355X_HBM_PEAK_GBS, unit="GB/s",
                    frac=round(ach / MI355X_HBM_PEAK_GBS, 4))
    return base


def family_rooflines(by_variant, steps, peak_tflops, ridge, top=6):
    """Every conv kernel family (template instantiation) of the live step on its own roofline — the dominant
    kernel is one line; these are the rest of the conv GPU time. Per family: launches and GPU ms per step, the
    achieved FLOP and algorithmic-byte rates over its HIP-event time, its mean intensity, and the fraction of
    the roof that bounds it (MFMA above the ridge, HBM below). Largest ``top`` families by time."""
    out = []
    for k, (ms, flops, nbytes, n) in sorted(by_variant.items(), key=lambda kv: -kv[1][0])[:top]:
        if ms <= 0:
            continue
        sec = ms * 1e-3
        tf, gbs = flops / sec / 1e12, nbytes / sec / 1e9
        inten = flops / max(nbytes, 1.0)
        if kernel_peak(k) != peak_tflops:  # a bf16x6 family: its own (fp32-equivalent) MFMA ceiling and ridge
            peak_k = kernel_peak(k)
            ridge_k = peak_k * 1e12 / (MI355X_HBM_PEAK_GBS * 1e9)
        else:
            peak_k, ridge_k = peak_tflops, ridge
        bound = "mfma" if inten >= ridge_k else "hbm"
        out.append({"kernel": k, "launches_per_step": round(n / steps, 1), "ms_per_step": round(ms / steps, 3),
                    "avg_launch_us": round(1000.0 * ms / n, 2), "tflops": round(tf, 2), "gbs": round(gbs, 1),
                    "intensity_flop_per_byte": round(inten, 2), "bound": bound,
                    "frac": round(tf / peak_k if bound == "mfma" else gbs / MI355X_HBM_PEAK_GBS, 4)})
    return out


def host_jpeg_legs(net, step_eager_cpu, x_cpu, reps=5, step_graph_cpu=None):
    """SURVEY §8d "reported twice" / §8f f2: the host JPEG stage alone (1 thread, a thread pool, worker
    processes) and the C2 train step WITH the host JPEG stage inline, eager, as train.sh runs it
    (``model(d)`` on a CPU batch: JPEG round trip on the host, H2D copy, device step), then the same with
    the next batch's JPEG prefetched in the background (src/utils/engine.py's pipelining)."""
    from hyres_hip import jpeg_host
    from models.utils.turbo_jpeg_compression import TurboJPEGCompression
    B = x_cpu.shape[0]
    res = {"backend": net.jpeg.backend}
    pool, nprocs = jpeg_host.pool()
    for tag, workers, use_procs in (("threads_1", 1, False), ("threads_16", 16, False), ("procs", 0, True)):
        if use_procs and pool is None:
            continue
        j = TurboJPEGCompression(quality=net.jpeg.quality, workers=max(workers, 1))
        saved = jpeg_host._POOL
        if not use_procs:
            jpeg_host._POOL = None
        try:
            j(x_cpu)
            t0 = time.time()
            for _ in range(3):
                j(x_cpu)
            res[f"ms_per_image_{tag}" if not use_procs else f"ms_per_image_procs_{nprocs}"] = round(
                (time.time() - t0) * 1000 / (3 * B), 3)
        finally:
            jpeg_host._POOL = saved
    # eager train step with JPEG inline (two alternating CPU batches so a prefetch is never stale)
    xs = [x_cpu, torch.flip(x_cpu, dims=[3]).contiguous()]
    for tag, prefetch in (("with_host_jpeg", False), ("with_host_jpeg_prefetch", True)):
        step_eager_cpu(xs[0], None)
        torch.cuda.synchronize()
        t0 = time.time()
        for i in range(reps):
            step_eager_cpu(xs[i % 2], xs[(i + 1) % 2] if prefetch else None)
        torch.cuda.synchronize()
        ms = (time.time() - t0) * 1000 / reps
        res[tag] = {"ms_per_step": round(ms, 3), "mpix_s": round(B * x_cpu.shape[2] * x_cpu.shape[3] / ms / 1e3, 3)}
    if step_graph_cpu is not None:
        # src/utils/engine.py's default: host JPEG (prefetched) + H2D + the replayed forward/loss/backward graph
        step_graph_cpu(xs[0], xs[1])
        torch.cuda.synchronize()
        t0 = time.time()
        for i in range(reps):
            step_graph_cpu(xs[i % 2], xs[(i + 1) % 2])
        torch.cuda.synchronize()
        ms = (time.time() - t0) * 1000 / reps
        res["with_host_jpeg_prefetch_graph"] = {"ms_per_step": round(ms, 3),
                                                "mpix_s": round(B * x_cpu.shape[2] * x_cpu.shape[3] / ms / 1e3, 3)}
    return res


def codec_leg(net, xk, jk, reps=3):
    """configs[4] / BASELINE.md §1: LightWeightCheckerboard.compress / decompress self-timers (transforms +
    rANS, JPEG and MultiScaleRefine excluded — the span of the README's 0.476 s / 0.286 s) on one Kodak-size
    768x512 residual, best of ``reps``; bpp from the strings. Synthetic image and recipe weights: the bpp is
    not comparable with a trained model's."""
    rm = net.residual_model
    net.update(force=True)
    residual = (xk - jk).contiguous()
    enc, dec = [], []
    for _ in range(reps):
        c = rm.compress(residual)
        d = rm.decompress(c["strings"], c["shape"])
        torch.cuda.synchronize()
        enc.append(c["time"])
        dec.append(d["time"])
    nbits = 8 * sum(len(s) for part in (c["strings"][0][0], c["strings"][0][1], c["strings"][1]) for s in part)
    e, dd = min(enc) * 1000, min(dec) * 1000
    return {"encode_ms": round(e, 2), "decode_ms": round(dd, 2), "residual_bpp": round(nbits / (512 * 768), 4),
            "readme_encode_ms": 476.0, "readme_decode_ms": 286.0,
            "speedup_vs_readme": round((476.0 + 286.0) / (e + dd), 2)}


def analysis_synthesis(net, x, reps):
    """North-star target (BASELINE.json): the N=128/M=192 analysis + synthesis pass (g_a on the residual,
    g_s on y_hat; models/checkerboard.py:35-58) at bs=16 256x256, forward, as a HIP graph. Fraction of the
    HBM roofline = SURVEY §8d ledger bytes (1.836 GB per image: g_a 0.918 + g_s 0.918) / t / 8 TB/s;
    FLOP rate from the same ledger (40.66 GFLOP per image)."""
    from hyres_hip import ops as O
    rm = net.residual_model
    B, _, H, W = x.shape
    with torch.no_grad():
        xn = O.to_nhwc(x - 0.5, rg=False)
        yh = O.Node.new(B, H // 8, W // 8, rm.M, x.device, rg=False)
        yh.v.copy_(torch.randn(yh.v.shape, generator=torch.Generator().manual_seed(3)).to(x.device))
        for _ in range(2):
            rm.g_a.hip(None, xn)
            rm.g_s.hip(None, yh)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            rm.g_a.hip(None, xn)
            rm.g_s.hip(None, yh)
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        ms = (time.time() - t0) * 1000 / reps
        g.reset()  # the capture's g_a / g_s outputs were dropped inside .hip(): nothing of its pool is held
        del g
    ledger = B * 1.836e9
    res = {"ms": round(ms, 3), "ledger_bytes": ledger, "hbm_frac": round(ledger / (ms * 1e-3) / 8e12, 4),
           "tflops": round(B * 40.66e9 / (ms * 1e-3) / 1e12, 2),
           "mfma_fp32_frac": round(B * 40.66e9 / (ms * 1e-3) / 1e12 / MI355X_FP32_PEAK_TFLOPS, 4),
           "target": "north_star: >= 0.40 of the HBM roofline, i.e. <= 9.2 ms at bs=16"}
    # the SAME pass's HBM bytes measured with PMC counters (scripts/as_traffic.py, profiles/r6k_as_traffic.json: round 6 build, scripts/check.sh phase "as"):
    # the fused kernels move far fewer bytes than the eager per-op ledger, so the honest HBM fraction is lower —
    # this pass is MFMA-bound (mfma_fp32_frac), not HBM-bound
    try:
        with open(os.path.join(REPO, "profiles", "r6k_as_traffic.json")) as f:
            pmc = json.load(f)
        if pmc.get("ledger_bytes_per_pass") == ledger:
            res["pmc_bytes"] = pmc["bytes_per_pass"]
            res["hbm_frac_pmc"] = round(pmc["bytes_per_pass"] / (ms * 1e-3) / 8e12, 4)
    except (OSError, KeyError, ValueError):
        pass
    return res


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # host JPEG worker processes: spawned before this process touches the GPU (hyres_hip.jpeg_host); only
    # the N = 1 run times the host JPEG legs, so N > 1 ranks code their one setup batch in-process (no
    # 8 workers per rank on a full node)
    from hyres_hip import jpeg_host
    jpeg_host.start(args.jpeg_procs if world == 1 else 0)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1 or os.environ.get("HYRES_BENCH_FORCE_DIST") == "1"  # rehearse the RCCL path at N=1
    # rehearsal knobs for the N>1 path on a one-GPU box: HYRES_BENCH_ONE_GPU=1 puts every rank on device 0,
    # HYRES_BENCH_BACKEND=gloo replaces RCCL (which refuses two ranks on one device); defaults = the real run
    if os.environ.get("HYRES_BENCH_ONE_GPU") == "1":
        local = 0
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group(os.environ.get("HYRES_BENCH_BACKEND", "nccl"))
    dev = torch.device("cuda", local)

    from hyres_hip import _lib as L
    if args.fp32_gemm != "default":
        L.call("hyres_conv_tuning", 7, 1 if args.fp32_gemm == "bf16x6" else 0, None)
    from hyres_hip.weights import synthetic_state_dict
    from hyres_hip.loss import RateDistortionLoss
    from hyres_hip.optim import FusedAdam
    from hyres_hip import ops as O
    from models import ResidualJPEGCompression

    net = ResidualJPEGCompression(jpeg_quality=args.jpeg_quality)
    torch.nn.Module.load_state_dict(net, synthetic_state_dict(net.state_dict()), strict=True)
    net = net.to(dev).train()
    main_names = [n for n, p in sorted(net.named_parameters()) if not n.endswith(".quantiles")]
    main_p = [p for n, p in sorted(net.named_parameters()) if not n.endswith(".quantiles")]
    aux_p = [p for n, p in sorted(net.named_parameters()) if n.endswith(".quantiles")]
    opt = FusedAdam(main_p, lr=3e-4, max_grad_norm=1.0)
    aux_opt = FusedAdam(aux_p, lr=3e-4)
    reducer = None
    # N > 1: the captured forward/backward replays on every rank and the flat gradient is all-reduced over
    # RCCL; HYRES_DIST_MODE=eager-overlap (or --no-graph) selects the eager step with overlapped collectives.
    dist_mode = None
    if dist:
        # default "graph+overlap" (round 6): the step captured as two graphs cut at the "hyper" backward marker, the
        # finished refine / g_s / hyperprior segments' all-reduce launched between the two replays (no event node
        # inside a graph, no extra stream); "graph+allreduce": one replay, then the whole flat gradient;
        # "eager-overlap": the eager step with each segment's all-reduce started at its backward-progress marker
        dist_mode = "eager-overlap" if args.no_graph else os.environ.get("HYRES_DIST_MODE", DIST_DEFAULT)
        assert dist_mode in ("eager-overlap", "graph+allreduce", "graph+overlap"), dist_mode
    if dist:
        # RCCL all-reduce of refine / g_s / hyperprior gradient segments launched from backward-progress
        # markers (overlapped with the rest of backward), the remainder (g_a) after backward
        from hyres_hip.ddp import FlatGradReducer, HYRES_SEGMENTS
        reducer = FlatGradReducer(opt.flat, world, names=main_names, segments=HYRES_SEGMENTS)
        if dist_mode == "eager-overlap":
            reducer.overlap()
    crit = RateDistortionLoss(lmbda=args.lmbda, alpha=0)

    B, S = args.batch, args.size
    g = torch.Generator().manual_seed(1926 + rank)
    x_cpu = torch.randint(0, 256, (B, 3, S, S), generator=g).float() / 255.0
    t0 = time.time()
    jpeg_cpu, jpeg_bpp = net.jpeg(x_cpu)
    jpeg_ms = (time.time() - t0) * 1000 / B
    x = x_cpu.to(dev)
    jpeg = jpeg_cpu.to(dev)

    graphed = None
    if not args.no_graph and dist_mode != "eager-overlap":
        # forward + RD loss + backward captured once as a HIP graph (hyres_hip.graphs); the optimiser,
        # the RCCL all-reduce and the aux step stay eager (a handful of launches)
        from hyres_hip.graphs import CapturedStep
        # graph+overlap: the capture is cut at the "hyper" backward-progress marker; between the two replays the
        # refine / g_s / hyperprior gradient segments start their RCCL all-reduce, which runs while g_a's backward
        # (the second graph) computes
        graphed = CapturedStep(net, x, jpeg, jpeg_bpp, noisequant=False, criterion=crit, zero_grad=opt.zero_grad,
                               capture_error_mode="thread_local" if dist else "global",
                               split_at=SPLIT_AT if dist_mode == "graph+overlap" else ())

    def fwd_bwd(eager=False, gr=None):
        gr = gr or graphed
        if gr is not None and not eager:
            between = reducer.launch_segments if (reducer is not None and gr.split_at) else None
            return gr.replay(between=between)[1]
        out = net.forward_device(x, jpeg, jpeg_bpp, noisequant=False)
        c = crit(out, x)
        c["loss"].backward()
        return c

    def step(eager=False, gr=None):
        c = fwd_bwd(eager, gr)
        if reducer is not None:
            reducer.all_reduce()
        opt.step()
        opt.zero_grad()
        aux = net.aux_loss()
        aux.backward()
        aux_opt.step()
        aux_opt.zero_grad()
        return c

    def step_eager_cpu(xc, x_next):
        """train.sh's path: model(d) on a CPU batch (host JPEG inline), eager, + loss/backward/optimiser."""
        if x_next is not None:
            net.jpeg.prefetch(x_next)
        out = net(xc, noisequant=False)
        c = crit(out, xc.to(dev, non_blocking=True))
        c["loss"].backward()
        opt.step()
        opt.zero_grad()
        aux = net.aux_loss()
        aux.backward()
        aux_opt.step()
        aux_opt.zero_grad()

    def step_graph_cpu(xc, x_next):
        """The drop-in loop's graphed step (src/utils/engine.py _GraphedStep): JPEG on the host for a CPU
        batch (the next one prefetched), H2D, replay, optimiser."""
        net.jpeg.prefetch(x_next)
        dec, bpp = net.jpeg(xc)
        graphed.replay(xc.to(dev), dec.to(dev), float(bpp))
        opt.step()
        opt.zero_grad()
        aux = net.aux_loss()
        aux.backward()
        aux_opt.step()
        aux_opt.zero_grad()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.time()
    for i in range(args.steps):
        c = step()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    elapsed = time.time() - t0
    loss_val = float(c["loss"].detach())
    c = None  # replay outputs live in the graph's pool: none may be held when the graph is closed
    # dominant-kernel roofline, measured live with HIP events (on the stream each conv launch goes to:
    # torch's current stream, also inside the branch streams) around every conv_fwd_kernel launch of one
    # eager step of the same workload right after the timed region (a graph replay cannot carry
    # per-kernel host events); the instantiation with the largest total time is reported
    # (averaged over EAGER_TIMED steps: one step's concurrent-branch overlap varies run to run)
    def timed_steps():
        O.KernelTimer.reset()
        O.KernelTimer.enabled = True
        for _ in range(EAGER_TIMED):
            step(eager=True)
        torch.cuda.synchronize()
        O.KernelTimer.enabled = False
        r = O.KernelTimer.summary()
        r["launches"] //= EAGER_TIMED
        r["by_variant_ms"] = {k: round(v / EAGER_TIMED, 3) for k, v in r.get("by_variant_ms", {}).items()}
        r["families"] = family_rooflines(r.get("by_variant", {}), EAGER_TIMED, MI355X_FP32_PEAK_TFLOPS,
                                         MI355X_FP32_PEAK_TFLOPS * 1e12 / (MI355X_HBM_PEAK_GBS * 1e9))
        return r

    ks = timed_steps()
    # the same kernel without the concurrent branches' contention (branch and side streams off):
    # its intrinsic rate, reported next to the live one
    O.BranchStreams.enabled = O.SideStream.enabled = False
    ks_iso = timed_steps()
    O.BranchStreams.enabled = O.SideStream.enabled = True
    if dist:
        t = torch.tensor([elapsed], device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t)
    ms = elapsed * 1000 / args.steps
    value = world * B * S * S * args.steps / elapsed / 1e6

    achieved = ks["flops"] / (ks["total_ms"] * 1e-3) / 1e12 if ks["total_ms"] > 0 else 0.0
    # the same instantiation's entry in the isolated steps (it need not be the top kernel there)
    iso = iso_us = None
    ent = ks_iso.get("by_variant", {}).get(ks["kernel"])
    if ent is not None and ent[0] > 0:
        iso = ent[1] / (ent[0] * 1e-3) / 1e12
        iso_us = 1000.0 * ent[0] / ent[3]


    if rank != 0:
        if graphed is not None:
            graphed.close()
        if dist:
            tdist.destroy_process_group()
        return
    # the fp32 convs' GEMM (hyres_conv_tuning key 7: 1 bf16x6, 0 the native fp32 MFMA); the same step is re-captured
    # and timed once more on the other GEMM (A/B on this box)
    cur = ctypes.c_int(0)
    L.call("hyres_conv_tuning", 7, 1, ctypes.byref(cur))  # read (and restore) the current mode
    L.call("hyres_conv_tuning", 7, cur.value, None)
    fp32_gemm = "bf16x6" if cur.value == 1 else "native"
    other = None
    if world == 1 and graphed is not None:
        from hyres_hip.graphs import CapturedStep
        L.call("hyres_conv_tuning", 7, 1 - cur.value, None)
        try:
            gn = CapturedStep(net, x, jpeg, jpeg_bpp, noisequant=False, criterion=crit, zero_grad=opt.zero_grad)
            for _ in range(args.warmup):
                step(gr=gn)
            torch.cuda.synchronize()
            t0 = time.time()
            for _ in range(args.steps):
                step(gr=gn)
            torch.cuda.synchronize()
            ms_n = (time.time() - t0) * 1000 / args.steps
            gn.close()
            del gn
            name = "native" if cur.value == 1 else "bf16x6"
            other = {"fp32_gemm": name, "ms_per_step": round(ms_n, 3), "value": round(B * S * S / ms_n / 1e3, 4),
                     "note": f"the same graphed C2 step with the fp32 convs on the {name} GEMM, timed after the "
                             "headline on this box"}
        finally:
            L.call("hyres_conv_tuning", 7, cur.value, None)
    # the same step with the concurrent branch streams off (every kernel on the main stream), A/B on this box
    serial = None
    if world == 1 and graphed is not None:
        from hyres_hip.graphs import CapturedStep
        O.BranchStreams.enabled = False
        try:
            gs = CapturedStep(net, x, jpeg, jpeg_bpp, noisequant=False, criterion=crit, zero_grad=opt.zero_grad)
            for _ in range(args.warmup):
                step(gr=gs)
            torch.cuda.synchronize()
            t0 = time.time()
            for _ in range(args.steps):
                step(gr=gs)
            torch.cuda.synchronize()
            ms_s = (time.time() - t0) * 1000 / args.steps
            gs.close()
            del gs
            serial = {"ms_per_step": round(ms_s, 3), "value": round(B * S * S / ms_s / 1e3, 4),
                      "note": "the same graphed C2 step with MultiScaleRefine's / AttentionBlock's branches on one "
                              "stream, timed after the headline on this box"}
        finally:
            O.BranchStreams.enabled = True
    evals = None
    if world == 1 and not args.no_eval:
        evals = eval_legs(net, x, jpeg, jpeg_bpp, args)
    amp = None
    if world == 1 and not args.no_amp:
        amp = amp_leg(net, opt, aux_opt, crit, x, jpeg, jpeg_bpp, args)
    host = None
    if world == 1 and not args.no_host_jpeg:
        host = host_jpeg_legs(net, step_eager_cpu, x_cpu, step_graph_cpu=step_graph_cpu if graphed is not None else None)
    if graphed is not None:
        graphed.close()  # every CapturedStep of this run is closed explicitly (DESIGN §13 "Open")
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, args.cpu_baseline_seconds)
    line = {
        "metric": "Mpixels/s encode+decode (N=128,M=192,256\u00d7256) at 1/2/4/8 GPU; bpp+PSNR parity",
        "metric_definition": ("BASELINE.json's metric, measured on configs[1] (the workload it is quoted on): one "
                              "step = forward (g_a 'encode' + hyperprior + checkerboard context + g_s 'decode' + "
                              "MultiScaleRefine) + RD-loss backward + clip + Adam + aux Adam at bs=16 per GPU, "
                              "device-only (host JPEG precomputed). This TRAIN-STEP rate is stricter than "
                              "SURVEY §8d's 'encode+decode' = eval-forward rate, which is reported as "
                              "'encode_decode_eval' (eval.bs16_256x256; C3's bs=32 in eval.bs32_256x256); the "
                              "with-host-JPEG rates are in 'host_jpeg'"),
        "encode_decode_eval": None if not evals else {
            k: evals[k]["mpix_s"] for k in evals if k.startswith("bs") and "mpix_s" in evals[k]},
        "value": round(value, 4),
        "unit": "Mpixels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic uniform 8-bit RGB, recipe-initialised weights (no checkpoint ships)",
        "config": {"workload": "C2 train step (configs[1]): ResidualJPEGCompression N=128 M=192, fwd+bwd+"
                               "optimizer, lambda=0.045, noisequant=False, JPEG q50 precomputed on host",
                   "global_batch": B * world, "image": [S, S], "parallelism": f"dp{world}"},
        "fp32_gemm": fp32_gemm,
        "fp32_gemm_note": FP32_GEMM_NOTE[fp32_gemm],
        "fp32_gemm_ab": other,
        "branch_streams_off_ab": serial,
        "roofline": {"bound": "mfma", "kernel": f"{ks['kernel']} ({kernel_label(ks['kernel'])})",
                     "achieved": round(achieved, 3), "peak": kernel_peak(ks["kernel"]), "unit": "TFLOP/s",
                     "peak_note": peak_note(ks["kernel"]),
                     "frac": round(achieved / kernel_peak(ks["kernel"]), 4),
                     "frac_vs_native_fp32_peak": round(achieved / MI355X_FP32_PEAK_TFLOPS, 4),
                     "traffic": traffic_bytes_per_launch(ks["kernel"]),
                     "launches_per_step": ks["launches"], "avg_launch_us": round(ks["avg_us"], 2),
                     "flops_per_launch": ks["flops_per_launch"],
                     "algorithmic_bytes_per_launch": ks["bytes_per_launch"],
                     "timing": f"HIP events around each launch of {EAGER_TIMED} eager steps after the timed region",
                     "achieved_isolated": None if iso is None else round(iso, 3),
                     "frac_isolated": None if iso is None else round(iso / kernel_peak(ks["kernel"]), 4),
                     "avg_launch_us_isolated": None if iso_us is None else round(iso_us, 2),
                     "ms_by_variant": ks.get("by_variant_ms"),
                     "families": ks.get("families")},
        "graph": graphed is not None,
        "dist_mode": dist_mode,
        "eval": evals,
        "cpu_baseline": cpu,
        "jpeg_host_ms_per_image": round(jpeg_ms, 3),
        "host_jpeg": host,
        "amp": amp,
        "loss": loss_val,
    }
    print(json.dumps(line))
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
