"""Register-allocation guards read from libhyres_hip.so's code-object metadata (host tools only, no GPU).

DESIGN §4 "Cross-kernel interference": waves of other kernels sharing SIMDs with conv3x3_wres_bf6_kernel computed
wrong values while its allocation (224 VGPRs x 2 waves per SIMD) left a 64-register hole; the kernel therefore takes
the whole file. These tests keep that guard from silently disappearing (a compiler update or an edit of the kernel's
asm line) and list every persistent 512-thread kernel whose allocation still leaves room for another kernel's waves.
"""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "scripts"))
import kernel_meta  # noqa: E402

SO = os.path.join(os.path.dirname(HERE), "hyres-residual-enhanced-hybrid-image-compression_amd", "hyres_hip",
                  "libhyres_hip.so")

pytestmark = pytest.mark.skipif(not (kernel_meta.available() and os.path.exists(SO)),
                                reason="ROCm LLVM tools or the built library absent")


@pytest.fixture(scope="module")
def meta():
    return {k["name"]: k for k in kernel_meta.kernels(SO)}


def _find(meta, fragment):
    hits = [k for n, k in meta.items() if fragment in n]
    assert hits, fragment
    return hits


def test_wres_bf6_takes_the_whole_vgpr_file(meta):
    # GUARD = true: every instantiation a default launch can pick (the variants of hyres_conv_tuning key 12)
    ks = _find(meta, "conv3x3_wres_bf6_kernelILb1E")
    assert len(ks) == 5  # key 12 variants 0..3 and the dilation-2 build of variant 1
    for k in ks:
        r = kernel_meta.residency(k)
        assert k["threads"] == 512 and k["alloc"] == 256, k
        assert r["waves_per_simd"] == 2 and r["hole_vgprs"] == 0, r
        assert k["scratch"] == 0
    # the diagnostic instantiation (hyres_conv_tuning key 9 = 0) keeps the allocation that showed the interference
    (d,) = _find(meta, "conv3x3_wres_bf6_kernelILb0E")
    assert d["alloc"] == 224 and kernel_meta.residency(d)["hole_vgprs"] == 64, d


def test_other_cvt_mfma_persistent_kernels_take_the_whole_vgpr_file(meta):
    """ru_fused_f16_kernel beside a side-stream bilinear showed the same interference in its 232-VGPR build (round 5,
    scripts/bf6_interference_repro.hip ru); it and every weight-resident f16 3x3 now leave no hole."""
    (k,) = _find(meta, "ru_fused_f16_kernelILb1E")
    assert k["alloc"] == 256 and kernel_meta.residency(k)["hole_vgprs"] == 0, k
    (d,) = _find(meta, "ru_fused_f16_kernelILb0E")  # diagnostic build
    assert d["alloc"] == 232, d
    for k in _find(meta, "conv3x3_wres_f16_kernel") + _find(meta, "conv3x3_wres_f32_kernel"):
        assert k["alloc"] == 256 and kernel_meta.residency(k)["hole_vgprs"] == 0, k


def test_no_default_path_kernel_uses_scratch(meta):
    # a spill or a register array demoted to scratch memory is a performance bug on these kernels
    bad = [n for n, k in meta.items() if k["scratch"] and ("conv" in n or "wgrad" in n or "ru_fused" in n)]
    assert not bad, bad


# The diagnostic builds that keep the allocation which showed the interference (hyres_conv_tuning key 9 = 0): never
# launched by a default or user-selectable production mode, only by the co-residency tests and the reproducer.
DIAGNOSTIC_HOLES = ("conv3x3_wres_bf6_kernelILb0E", "ru_fused_f16_kernelILb0E")


def test_lds_limited_512_thread_kernels_leave_no_hole(meta):
    """The guard's predicate (DESIGN §4 "Cross-kernel interference"), asserted: every LDS-limited 512-thread kernel —
    the persistent / one-or-two-blocks-per-CU shape of all three observed hogs (bf16x6 and f16 kernels that convert with
    v_cvt_pk_*, and the native fp32-MFMA conv3x3_wres_f32_kernel, which does not) — allocates the whole VGPR file of its
    SIMDs, in every mode a user can select (HYRES_FP32_GEMM=native runs the native wgrad1x1_kernel<..., G = 2>). Only the
    diagnostic builds are exempt."""
    rows, bad = [], []
    for n, k in sorted(meta.items()):
        if k["threads"] != 512:
            continue
        r = kernel_meta.residency(k)
        if not r["lds_limited"]:
            continue
        rows.append(n)
        if r["hole_vgprs"] and not any(d in n for d in DIAGNOSTIC_HOLES):
            bad.append((kernel_meta.demangle([n])[0], k["alloc"], r["hole_vgprs"]))
    assert not bad, bad
    names = {kernel_meta.demangle([n])[0].split("(")[0].split("::")[-1].split("<")[0] for n in rows}
    assert {"conv3x3_wres_bf6_kernel", "ru_fused_f16_kernel", "conv3x3_wres_f32_kernel", "conv3x3_wres_f16_kernel",
            "wgrad1x1_kernel"} <= names, names


@pytest.fixture(scope="module")
def disasm():
    return kernel_meta.disassembly(SO)


def test_cvt_mfma_kernels_with_a_hole_are_256_thread(meta, disasm):
    """Kernels that convert with v_cvt_pk_* AND run MFMAs while leaving a hole of >= 40 VGPRs (room for the 40-VGPR
    side-stream bilinear): all are 256-thread multi-block kernels — the shape measured as no hog (the bf16x6 weight
    gradients and implicit GEMM beside all five victims: 0 wrong values in 20 runs each, profiles/r5t_repro_wgrad_hogs.txt)
    — apart from the diagnostic builds. A new or recompiled 512-thread cvt + MFMA kernel with a hole fails here."""
    offenders = []
    for n, ins in disasm.items():
        k = meta.get(n)
        if k is None or any(d in n for d in DIAGNOSTIC_HOLES):
            continue
        ops = {i.split()[0] for i in ins}
        if not (any(o.startswith("v_cvt_pk") for o in ops) and any(o.startswith("v_mfma") for o in ops)):
            continue
        if kernel_meta.residency(k)["hole_vgprs"] >= 40 and k["threads"] != 256:
            offenders.append(kernel_meta.demangle([n])[0])
    assert not offenders, offenders


def test_hand_issued_lds_reads_are_waited_for_before_use(disasm):
    """conv3x3_wres_bf6_kernel's V & 1 path issues ds_read_b128 through inline asm and waits with hand-counted
    lgkmcnt values; the compiler treats the asm outputs as ready at once. Scan every kernel's ISA: no instruction may read
    or overwrite the destination VGPRs of an LDS read before an s_waitcnt has retired it (kernel_meta.lds_read_hazards;
    compiler-issued reads pass by construction, so the whole library is the calibration)."""
    assert kernel_meta.lds_read_hazards(["ds_read_b128 v[4:7], v1", "v_mov_b32 v8, v5", "s_waitcnt lgkmcnt(0)"])
    assert not kernel_meta.lds_read_hazards(["ds_read_b128 v[4:7], v1", "s_waitcnt lgkmcnt(0)", "v_mov_b32 v8, v5"])
    hand = [n for n in disasm if "conv3x3_wres_bf6_kernel" in n and ("Li1ELi" in n or "Li3ELi" in n)]
    assert len(hand) >= 3, hand  # V = 1 and 3 (dilation 1), V = 1 dilation 2
    for n in hand:
        assert sum(1 for i in disasm[n] if i.startswith("ds_read_b128")) >= 54, n  # 9 taps x 6 fragments, unrolled
    bad = {n: h[:2] for n, ins in disasm.items() for h in [kernel_meta.lds_read_hazards(ins)] if h}
    assert not bad, bad


def test_stream_b6_kernels_fill_the_vgpr_file(meta):
    """conv1x1_stream_b6_kernel (bf16x6 streaming 1x1, round 5) converts with v_cvt_pk_bf16_f32 and runs bf16 MFMAs:
    every instantiation (either epilogue path) allocates exactly 256 VGPRs (2 waves per SIMD) — no hole — and spills
    nothing; the round-6 SA_BWD (NT = 6), ROWSCALE (KS = 12) and 128 -> 128 (NT = 4, KS = 8) forms, one block per CU by
    their LDS, take all 512."""
    ks = _find(meta, "conv1x1_stream_b6_kernel")
    # (NT, KS) in {(2, 4), (4, 4), (2, 8)} x 8 epilogue-operand sets x coalesced epilogue on / off, + <6, 4, 8 | 12, true>
    # + the ROWSCALE form <2, 12, 16, true> + <4, 8, 0 | 2> (128 -> 128) x coalesced on / off + <6, 4, 40, true>
    # (SA_BWD with the scale-1 PReLU mask)
    assert len(ks) == 56
    for k in ks:
        full = 512 if ("kernelILi6E" in k["name"] or "ELi12E" in k["name"] or "kernelILi4ELi8E" in k["name"]) else 256
        assert k["alloc"] == full and kernel_meta.residency(k)["hole_vgprs"] == 0 and k["scratch"] == 0, k
