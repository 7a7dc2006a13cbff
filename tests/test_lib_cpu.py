"""CPU: the C-ABI library loads and exports every symbol include/hyres_hip.h declares (no kernel calls)."""
import os
import re

import pytest

from conftest import REPO


def header_functions():
    src = open(os.path.join(REPO, "include", "hyres_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_\s\*]*?\b(hyres_[a-z0-9_]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_library_exports_every_header_symbol():
    from hyres_hip import _lib as L
    lib = L.load()
    names = header_functions()
    assert len(names) > 50
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding declares a signature for each of them
    unbound = [n for n in names if n not in L.exported_symbols()]
    assert not unbound, unbound
    assert lib.hyres_version() >= 10000


def test_geometry_helpers_without_gpu():
    """Pure host functions: geometry / workspace planning need no device."""
    import ctypes
    from hyres_hip import _lib as L
    lib = L.load()
    g = L.ConvGeom()
    assert lib.hyres_geom_deconv2d(ctypes.byref(g), 2, 8, 8, 128, 128, 64, 64, 5, 2) == 0
    assert g.nphase == 4 and g.ntaps == 25 and [g.ntap[i] for i in range(4)] == [9, 6, 6, 4]
    assert (g.Ho, g.Wo) == (16, 16)
    assert lib.hyres_geom_conv2d_dgrad(ctypes.byref(g), 2, 16, 16, 3, 3, 128, 128, 5, 5, 2, 2, 1) == 0
    assert g.nphase == 4 and g.ntaps == 25 and (g.Hq, g.Wq) == (8, 8)
    d = L.WgradDesc()
    assert lib.hyres_wgrad_desc_conv2d(ctypes.byref(d), 16, 128, 128, 64, 64, 64, 64, 3, 3, 1, 1, 1) == 0
    assert lib.hyres_wgrad_workspace_bytes(ctypes.byref(d)) > 0
    # error path: unsupported stride-3 dgrad reports a shape error with a message
    rc = lib.hyres_geom_conv2d_dgrad(ctypes.byref(g), 1, 9, 9, 4, 4, 4, 4, 3, 3, 3, 1, 1)
    assert rc == 1001 and b"stride 2" in lib.hyres_last_error_string()


def test_product_path_has_no_oracle_imports():
    pkg = os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd")
    offenders = []
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                txt = open(os.path.join(root, f)).read()
                if re.search(r"^\s*(from|import)\s+oracle", txt, flags=re.M):
                    offenders.append(os.path.join(root, f))
    assert not offenders, offenders


# ------------------------------------------------------------------ entropy coding (host side of f1)
def _cdf_call(pmf):
    import ctypes
    import numpy as np
    from hyres_hip import _lib as L
    p = np.ascontiguousarray(pmf, dtype=np.float32)
    out = np.zeros(len(p) + 1, dtype=np.int32)
    L.check(L.load().hyres_pmf_to_quantized_cdf(p.ctypes.data, len(p), 16, out.ctypes.data), "cdf")
    return out.tolist()


def test_pmf_to_quantized_cdf_matches_restatement():
    """hyres_pmf_to_quantized_cdf == compressai's pmf_to_quantized_cdf (oracle/entropy_coding.py), incl.
    zero-probability symbols that must steal a frequency unit; the result is a valid 16-bit CDF."""
    import numpy as np
    from oracle.entropy_coding import gc_tables, pmf_to_quantized_cdf
    rng = np.random.default_rng(5)
    cases = [rng.random(n).astype(np.float32) for n in (2, 7, 40)]
    cases.append(np.array([0.5, 0.0, 0.0, 0.5, 1e-9], np.float32))
    z = rng.random(30).astype(np.float32)
    z[::3] = 0
    cases.append(z)
    for p in cases:
        p = p / p.sum()
        got = _cdf_call(p)
        assert got == pmf_to_quantized_cdf(p)
        assert got[0] == 0 and got[-1] == 65536 and all(b > a for a, b in zip(got, got[1:]))
    cdf, lengths, offsets = gc_tables([0.11, 1.0, 17.3, 256.0])
    assert list(lengths) == [2 * (-o) + 3 for o in offsets] and cdf[:, 0].tolist() == [0] * 4


def test_rans_roundtrip_and_bitstream_matches_restatement():
    """hyres_rans_encode/decode_with_indexes: decode(encode(s)) == s, including symbols outside every CDF's
    range (bypass escape), and the byte string equals the rans64 restatement's."""
    import ctypes
    import numpy as np
    from hyres_hip import _lib as L
    from oracle.entropy_coding import gc_tables, rans_decode, rans_encode
    lib = L.load()
    cdf, lengths, offsets = gc_tables(np.exp(np.linspace(np.log(0.11), np.log(256), 64)).astype(np.float32))
    rng = np.random.default_rng(11)
    n = 3000
    idx = rng.integers(0, 64, n).astype(np.int32)
    sym = np.round(rng.normal(0, 1, n) * np.exp(np.linspace(np.log(0.11), np.log(256), 64))[idx]).astype(np.int32)
    sym[::97] = np.int32(5000)   # far outside: bypass
    sym[5::131] = np.int32(-777)
    cdf = np.ascontiguousarray(cdf, np.int32)
    lengths = np.ascontiguousarray(lengths, np.int32)
    offsets = np.ascontiguousarray(offsets, np.int32)
    ln = ctypes.c_longlong(0)
    L.check(lib.hyres_rans_encode_with_indexes(sym.ctypes.data, idx.ctypes.data, n, cdf.ctypes.data, cdf.shape[1],
                                               lengths.ctypes.data, offsets.ctypes.data, 64, None, 0,
                                               ctypes.byref(ln)), "enc")
    buf = np.zeros(ln.value, np.uint8)
    L.check(lib.hyres_rans_encode_with_indexes(sym.ctypes.data, idx.ctypes.data, n, cdf.ctypes.data, cdf.shape[1],
                                               lengths.ctypes.data, offsets.ctypes.data, 64, buf.ctypes.data,
                                               buf.size, ctypes.byref(ln)), "enc")
    ref = rans_encode(sym.tolist(), idx.tolist(), cdf.tolist(), lengths.tolist(), offsets.tolist())
    assert buf.tobytes() == ref
    dec = np.zeros(n, np.int32)
    L.check(lib.hyres_rans_decode_with_indexes(buf.ctypes.data, buf.size, idx.ctypes.data, n, cdf.ctypes.data,
                                               cdf.shape[1], lengths.ctypes.data, offsets.ctypes.data, 64,
                                               dec.ctypes.data), "dec")
    assert np.array_equal(dec, sym)
    assert rans_decode(ref, idx.tolist(), cdf.tolist(), lengths.tolist(), offsets.tolist()) == sym.tolist()


def test_conv_kernel_name_follows_the_launch_routing():
    """hyres_conv_kernel_name (the profiler label bench.py's roofline line uses) reports the launcher's
    own tile choice: 128x64 tiles for 3x3 64-channel layers, half-height tiles for short-K 1x1 layers,
    the VALU narrow kernel for <= 4 output channels, split-K / fp16 / GDN-square flags."""
    import ctypes
    from hyres_hip import _lib as L
    from hyres_hip.ops import _geom, conv_variant
    e = L.Epilogue()
    e.kind = L.EPI_BIAS
    g3 = _geom("hyres_geom_conv2d", 16, 128, 128, 64, 64, 64, 64, 3, 3, 1, 1, 1)
    g3b = _geom("hyres_geom_conv2d", 16, 128, 128, 96, 96, 64, 64, 3, 3, 1, 1, 1)  # Ci = 96: implicit GEMM
    # bf16x6 on the bf16 MFMA (hyres_conv_tuning key 7 = 1, the default)
    old = ctypes.c_int(0)
    L.call("hyres_conv_tuning", 7, 1, ctypes.byref(old))
    try:
        assert old.value == 1  # the default
        assert conv_variant(g3, e, False) == "conv3x3_wres_bf6_kernel"
        assert conv_variant(g3b, e, False) == "conv_fwd_b6_kernel<2, 1, 2, 2, 0, false>"
        assert conv_variant(g3b, e, True) == "conv_fwd_b6_kernel<2, 1, 2, 2, 0, true>"
        L.call("hyres_conv_tuning", 7, 0, None)  # the native fp32 MFMA
        _native_routing(L, e, g3, g3b, _geom, conv_variant)
    finally:
        L.call("hyres_conv_tuning", 7, old.value, None)


def _native_routing(L, e, g3, g3b, _geom, conv_variant):
    # fp32 3x3 with Ci = 64, W % 64 == 0 and >= 2 tiles per block: the weight-resident persistent kernel
    assert conv_variant(g3, e, False) == "conv3x3_wres_f32_kernel"
    assert conv_variant(g3b, e, False) == "conv_fwd_kernel<2, 1, 2, 2, 0, false, false>"
    assert conv_variant(g3b, e, True) == "conv_fwd_kernel<2, 1, 2, 2, 0, true, false>"
    g1 = _geom("hyres_geom_conv2d", 16, 128, 128, 64, 64, 128, 128, 1, 1, 1, 0, 1)
    assert conv_variant(g1, e, False) == "conv1x1_stream_kernel<4, 8>"  # K <= 128 1x1, >= 64k pixels
    g1b = _geom("hyres_geom_conv2d", 16, 256, 256, 192, 192, 64, 64, 1, 1, 1, 0, 1)  # K = 192: not short
    assert conv_variant(g1b, e, False) == "conv_fwd_kernel<2, 1, 2, 2, 0, false, false>"
    g1c = _geom("hyres_geom_conv2d", 16, 128, 128, 128, 128, 64, 64, 1, 1, 1, 0, 1)
    assert conv_variant(g1c, e, False) == "conv1x1_stream_kernel<2, 16>"
    gn = _geom("hyres_geom_conv2d", 16, 256, 256, 64, 64, 3, 3, 3, 3, 1, 1, 1)
    assert conv_variant(gn, e, False) == "conv_narrow_strip_kernel<3, 1>"
    gs = _geom("hyres_geom_conv2d", 16, 256, 256, 3, 3, 64, 64, 3, 3, 1, 1, 1)  # Ci = 3: scalar path
    assert conv_variant(gs, e, False) == "conv_fwd_kernel<1, 1, 2, 2, 2, false, false>"
    e.square_input = 1
    g2 = _geom("hyres_geom_conv2d", 16, 128, 128, 128, 128, 128, 128, 1, 1, 1, 0, 1)
    assert conv_variant(g2, e, False) == "conv_fwd_kernel<1, 2, 2, 2, 1, false, false>"
    e.square_input = 0
    e.f16_operands = 1
    # autocast 3x3, Ci = 64, >= 2 tiles of 4 x 64 pixels per CU: the weight-resident persistent kernel; fewer
    # tiles or Ci != 64: the halo-staged kernel; W % 64 != 0: the implicit-GEMM tiles
    assert conv_variant(g3, e, False) == "conv3x3_wres_f16_kernel<0>"
    gh = _geom("hyres_geom_conv2d", 2, 64, 64, 64, 64, 64, 64, 3, 3, 1, 1, 1)
    assert conv_variant(gh, e, False) == "conv3x3_halo_f16_kernel<0>"
    gh2 = _geom("hyres_geom_conv2d", 16, 128, 128, 96, 96, 64, 64, 3, 3, 1, 1, 1)
    assert conv_variant(gh2, e, False) == "conv3x3_halo_f16_kernel<0>"
    gw = _geom("hyres_geom_conv2d", 16, 32, 32, 64, 64, 64, 64, 3, 3, 1, 1, 1)
    assert conv_variant(gw, e, False) == "conv_fwd_kernel<1, 1, 2, 2, 0, false, true>"
    # autocast 1x1 (K <= 128, >= 64k pixels): the streaming kernel on fp16-rounded operands
    assert conv_variant(g1, e, False) == "conv1x1_stream_kernel<4, 8, true>"
    # small grids (<= 65536 output pixels): 64-row tiles; f16 takes 128x128 from 192 channels up
    e.f16_operands = 0
    s3 = _geom("hyres_geom_conv2d", 16, 32, 32, 96, 96, 96, 96, 3, 3, 1, 1, 1)
    assert conv_variant(s3, e, False) == "conv_fwd_kernel<1, 1, 2, 2, 0, false, false>"
    s5 = _geom("hyres_geom_conv2d", 16, 32, 32, 512, 512, 384, 384, 1, 1, 1, 0, 1)
    assert conv_variant(s5, e, False) == "conv_fwd_kernel<1, 2, 2, 2, 0, false, false>"
    e.f16_operands = 1
    assert conv_variant(s5, e, False) == "conv_fwd_kernel<2, 2, 2, 2, 0, false, true>"
    assert conv_variant(s3, e, False) == "conv_fwd_kernel<1, 1, 2, 2, 0, false, true>"
    # fp16 activations (autocast inference): conv_fwd_h_kernel<tile, mode, split, io>
    e.io_f16 = 3
    assert conv_variant(g3, e, False) == "conv3x3_wres_f16_kernel<3>"
    assert conv_variant(g1b, e, False) == "conv_fwd_h_kernel<2, 1, 2, 2, 0, false, 3>"
    # 1x1 K <= 128 with fp16 X and Y on >= 16384 pixels: the fp16 streaming kernel (not the fp32 one)
    assert conv_variant(g1, e, False) == "conv1x1_stream_h_kernel<4, 4>"
    e.square_input = 1  # (GDN's square prologue stays on the tiles)
    assert conv_variant(g1, e, False) == "conv_fwd_h_kernel<1, 2, 2, 2, 1, false, 3>"
    e.square_input = 0
    e.io_f16 = 2
    e.f16_operands = 0
    assert conv_variant(gs, e, False) == "conv_fwd_h_kernel<1, 1, 2, 2, 2, false, 2>"  # fp32 image in, fp16 out


def test_conv_plan_split_follows_the_tile():
    """Split-K engages only when the chosen tile leaves < 512 blocks and K has >= 8 chunks; the workspace
    query covers the larger of the fp32 / f16 plans."""
    import ctypes
    from hyres_hip import _lib as L
    from hyres_hip.ops import _geom
    lib = L.load()
    e = L.Epilogue()
    e.kind = L.EPI_BIAS

    def plan(g):
        t, n = ctypes.c_int(), ctypes.c_int()
        L.check(lib.hyres_conv_plan(ctypes.byref(g), ctypes.byref(e), ctypes.byref(t), ctypes.byref(n)), "plan")
        return t.value, n.value
    s3 = _geom("hyres_geom_conv2d", 16, 32, 32, 96, 96, 96, 96, 3, 3, 1, 1, 1)     # 256 x 2 = 512 blocks
    assert plan(s3) == (4, 1) and lib.hyres_conv_workspace_bytes(ctypes.byref(s3)) == 0
    h = _geom("hyres_geom_conv2d", 16, 32, 32, 128, 128, 128, 128, 5, 5, 2, 2, 1)  # 16^2 out: 64 x 2 blocks
    t, ns = plan(h)
    assert t == 4 and ns == 4
    assert lib.hyres_conv_workspace_bytes(ctypes.byref(h)) >= ns * 16 * 16 * 16 * 128 * 4
    big = _geom("hyres_geom_conv2d", 16, 128, 128, 64, 64, 64, 64, 3, 3, 1, 1, 1)
    assert plan(big) == (1, 1)


def test_fp32_gemm_env_switch():
    """HYRES_FP32_GEMM selects the fp32 convs' GEMM at library load: bf16x6 (default, hyres_conv_tuning key 7 = 1)
    or the native fp32 MFMA (key 7 = 0); anything else is refused."""
    import os
    import subprocess
    import sys
    from conftest import PKG
    code = ("import ctypes, sys; sys.path.insert(0, %r); from hyres_hip import _lib as L; o = ctypes.c_int(-1); "
            "L.call('hyres_conv_tuning', 7, 1, ctypes.byref(o)); print(o.value)") % PKG
    for env, want in ((None, "1"), ("bf16x6", "1"), ("native", "0")):
        e = dict(os.environ)
        e.pop("HYRES_FP32_GEMM", None)
        if env is not None:
            e["HYRES_FP32_GEMM"] = env
        out = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stderr
        assert out.stdout.strip().splitlines()[-1] == want, (env, out.stdout)
    e = dict(os.environ, HYRES_FP32_GEMM="tf32")
    out = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "HYRES_FP32_GEMM" in out.stderr


def test_bench_prices_each_kernel_with_its_own_pmc_summary():
    """bench.py's roofline ``traffic`` comes from the committed PMC summary collected for the kernel it prices
    (bf16x6 and native weight-resident convs, the AMP kernel), and is None for a kernel no summary covers."""
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    for kernel, paths in (("conv3x3_wres_bf6_kernel", b.PMC_TRAFFIC), ("conv3x3_wres_f32_kernel", b.PMC_TRAFFIC),
                          ("conv_fwd_h_kernel<1, 2, 2, 2, 0, false, 3>", b.PMC_TRAFFIC_AMP)):
        got = b.traffic_bytes_per_launch(kernel, paths)
        want = next(json.load(open(p))["traffic_bytes_per_launch"] for p in paths
                    if os.path.exists(p) and kernel in json.load(open(p))["kernel"])
        assert got == want and got > 0
    assert b.traffic_bytes_per_launch("no_such_kernel") is None
    assert b.traffic_bytes_per_launch(None) is None
