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


def test_persistent_kernels_with_room_beside_them(meta):
    """Every LDS-limited 512-thread (persistent, one block per CU) kernel and the VGPRs per SIMD its two waves leave
    to other kernels; a 40-register wave (the side-stream bilinear) fits in a hole of >= 40."""
    rows = []
    for n, k in sorted(meta.items()):
        if k["threads"] != 512:
            continue
        r = kernel_meta.residency(k)
        if r["lds_limited"]:
            rows.append((kernel_meta.demangle([n])[0], k["alloc"], r["hole_vgprs"]))
    for name, alloc, hole in rows:
        print(f"{name[:64]:64s} alloc {alloc:3d}  hole {hole:3d}{'  <- another kernel wave fits' if hole >= 40 else ''}")
    names = {r[0].split("(")[0].split("::")[-1].split("<")[0] for r in rows}
    assert {"conv3x3_wres_bf6_kernel", "ru_fused_f16_kernel", "conv3x3_wres_f32_kernel"} <= names


def test_stream_b6_kernels_fill_the_vgpr_file(meta):
    """conv1x1_stream_b6_kernel (bf16x6 streaming 1x1, round 5) converts with v_cvt_pk_bf16_f32 and runs bf16 MFMAs:
    every instantiation (either epilogue path) allocates exactly 256 VGPRs (2 waves per SIMD) — no hole — and spills nothing."""
    ks = _find(meta, "conv1x1_stream_b6_kernel")
    assert len(ks) == 48  # (NT, KS) in {(2, 4), (4, 4), (2, 8)} x 8 epilogue-operand sets x coalesced epilogue on / off
    for k in ks:
        assert k["alloc"] == 256 and kernel_meta.residency(k)["hole_vgprs"] == 0 and k["scratch"] == 0, k
