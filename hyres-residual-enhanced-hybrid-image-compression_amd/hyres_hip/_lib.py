"""ctypes binding of libhyres_hip.so (the C-ABI declared in include/hyres_hip.h).

The library is loaded from this directory (built in-tree by ``__graft_entry__.build()`` /
``python -m hyres_hip.build``).  There is NO fallback: if the shared object is missing or no GPU is
visible, every op raises — the product path never silently runs anything else.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
# HYRES_LIB_PATH: an alternative build for A/B timing runs (scripts only; the default is the in-tree library)
LIB_PATH = os.environ.get("HYRES_LIB_PATH") or os.path.join(HERE, "libhyres_hip.so")

MAX_TAPS = 49
WPREP_CONV, WPREP_CONV_DGRAD, WPREP_DECONV, WPREP_DECONV_DGRAD = 0, 1, 2, 3
EPI_BIAS, EPI_GDN, EPI_IGDN, EPI_GDN_BWD, EPI_IGDN_BWD, EPI_ROWSCALE, EPI_SA_BWD = 0, 1, 2, 3, 4, 5, 6
ACT_NONE, ACT_RELU, ACT_PRELU, ACT_RELU_MASK, ACT_PRELU_MASK = 0, 1, 2, 3, 4
PRELU_PARTIALS = 2048  # HYRES_PRELU_PARTIALS
IO_X16, IO_Y16, IO_AUX16 = 1, 2, 4  # hyres_epilogue.io_f16 bits (fp16 activations in HBM)
EB_REC = 64


class ConvGeom(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("B", "Hi", "Wi", "Ci", "ldx", "Ho", "Wo", "Co", "ldy", "nphase", "Hq", "Wq",
                 "osh", "osw", "ish", "isw")] + [
        ("oph", ctypes.c_int * 4), ("opw", ctypes.c_int * 4), ("ntap", ctypes.c_int * 4),
        ("tap0", ctypes.c_int * 4), ("ntaps", ctypes.c_int),
        ("dh", ctypes.c_int * MAX_TAPS), ("dw", ctypes.c_int * MAX_TAPS),
        ("kh", ctypes.c_int * MAX_TAPS), ("kw", ctypes.c_int * MAX_TAPS)]


class Epilogue(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("act", ctypes.c_int), ("accumulate", ctypes.c_int),
                ("square_input", ctypes.c_int),
                ("bias", ctypes.c_void_p), ("res", ctypes.c_void_p), ("ldres", ctypes.c_int),
                ("slope", ctypes.c_void_p),
                ("aux0", ctypes.c_void_p), ("ld0", ctypes.c_int),
                ("aux1", ctypes.c_void_p), ("ld1", ctypes.c_int),
                ("aux2", ctypes.c_void_p), ("ld2", ctypes.c_int),
                ("out2", ctypes.c_void_p), ("ldo2", ctypes.c_int), ("f16_operands", ctypes.c_int),
                ("io_f16", ctypes.c_int)]


class WgradDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("B", "Hq", "Wq", "M", "ldp", "N", "ldq", "Hqq", "Wqq", "sq", "ntaps")] + [
        ("dh", ctypes.c_int * MAX_TAPS), ("dw", ctypes.c_int * MAX_TAPS),
        ("sm", ctypes.c_int), ("sn", ctypes.c_int), ("st", ctypes.c_int),
        ("square_q", ctypes.c_int), ("accumulate", ctypes.c_int), ("f16_operands", ctypes.c_int),
        ("io_f16", ctypes.c_int)]


WGRAD_MAX_JOBS = 48


class WgradJob(ctypes.Structure):
    """hyres_wgrad_job: one deferred split-K slab reduce (include/hyres_hip.h)."""
    _fields_ = [("slab", ctypes.c_void_p), ("dst", ctypes.c_void_p)] + [
        (n, ctypes.c_int) for n in ("nsplit", "ntaps", "M", "N", "sm", "sn", "st", "accumulate", "lanes",
                                    "reserved")]


_P = ctypes.c_void_p
_I = ctypes.c_int
_LL = ctypes.c_longlong
_F = ctypes.c_float
_D = ctypes.c_double
_ULL = ctypes.c_ulonglong
_PP = ctypes.POINTER(ctypes.c_void_p)

# name -> (restype, argtypes)
_SIGS = {
    "hyres_version": (_I, []),
    "hyres_last_error_string": (ctypes.c_char_p, []),
    "hyres_geom_conv2d": (_I, [ctypes.POINTER(ConvGeom)] + [_I] * 12),
    "hyres_geom_conv2d_dgrad": (_I, [ctypes.POINTER(ConvGeom)] + [_I] * 12),
    "hyres_geom_deconv2d": (_I, [ctypes.POINTER(ConvGeom)] + [_I] * 9),
    "hyres_geom_deconv2d_dgrad": (_I, [ctypes.POINTER(ConvGeom)] + [_I] * 9),
    "hyres_geom_filter_taps": (_I, [ctypes.POINTER(ConvGeom), ctypes.POINTER(ctypes.c_ubyte), _I]),
    "hyres_conv_weight_prep": (_I, [ctypes.POINTER(ConvGeom), _P, _P, _I, _I, _I, _I, _I, _I, _P, _P]),
    "hyres_prep_desc_bytes": (_LL, []),
    "hyres_prep_desc_fill": (_I, [_P, ctypes.POINTER(ConvGeom), _P, _P, _I, _I, _I, _I, _I, _LL,
                                  ctypes.POINTER(_LL)]),
    "hyres_conv_weight_prep_batch": (_I, [_P, _I, _LL, _P]),
    "hyres_conv_forward": (_I, [ctypes.POINTER(ConvGeom), _P, _P, _I, _P, ctypes.POINTER(Epilogue), _P, _LL,
                                _P]),
    "hyres_conv_workspace_bytes": (_LL, [ctypes.POINTER(ConvGeom)]),
    "hyres_conv_kernel_name": (_I, [ctypes.POINTER(ConvGeom), ctypes.POINTER(Epilogue), _I, ctypes.c_char_p, _I]),
    "hyres_conv_tuning": (_I, [_I, _I, _P]),
    "hyres_conv_plan": (_I, [ctypes.POINTER(ConvGeom), ctypes.POINTER(Epilogue), _P, _P]),
    "hyres_wgrad_desc_conv2d": (_I, [ctypes.POINTER(WgradDesc)] + [_I] * 12),
    "hyres_wgrad_desc_deconv2d": (_I, [ctypes.POINTER(WgradDesc)] + [_I] * 9),
    "hyres_wgrad_workspace_bytes": (_LL, [ctypes.POINTER(WgradDesc)]),
    "hyres_conv_wgrad": (_I, [ctypes.POINTER(WgradDesc), _P, _P, _P, _P, _P, _LL, _P]),
    "hyres_conv_wgrad_deferred": (_I, [ctypes.POINTER(WgradDesc), _P, _P, _P, _P, _P, _LL, ctypes.POINTER(WgradJob),
                                       ctypes.POINTER(ctypes.c_int), _P]),
    "hyres_wgrad_reduce_jobs": (_I, [ctypes.POINTER(WgradJob), _I, _P]),
    "hyres_ru_fused_f16_ok": (_I, [_I, _I, _I, _I]),
    "hyres_ru_fused_f16": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P]),
    "hyres_colsum": (_I, [_P, _I, _I, _I, _P, _I, _P, _LL, _P]),
    "hyres_colsum_workspace_bytes": (_LL, [_I, _I]),
    "hyres_colsum_f16": (_I, [_P, _I, _I, _I, _P, _I, _P, _LL, _P]),
    "hyres_nchw_to_nhwc": (_I, [_P, _P, _I, _I, _I, _I, _I, _P]),
    "hyres_nhwc_to_nchw": (_I, [_P, _I, _P, _I, _I, _I, _I, _P]),
    "hyres_axpby": (_I, [_P, _P, _F, _P, _LL, _P]),
    "hyres_add_clamp01": (_I, [_P, _P, _P, _LL, _P]),
    "hyres_add_clamp01_bwd": (_I, [_P, _P, _P, _I, _LL, _P]),
    "hyres_relu_bwd": (_I, [_P, _P, _P, _LL, _P]),
    "hyres_relu_bwd_2d": (_I, [_P, _I, _P, _I, _P, _I, _LL, _I, _P]),
    "hyres_prelu_bwd": (_I, [_P, _I, _P, _I, _P, _I, _LL, _I, _P, _P, _P, _LL, _P]),
    "hyres_attn_gate_fwd": (_I, [_P, _P, _P, _P, _LL, _P]),
    "hyres_attn_gate_fwd_f16": (_I, [_P, _P, _P, _P, _LL, _P]),
    "hyres_attn_gate_bwd": (_I, [_P, _P, _P, _P, _P, _LL, _P]),
    "hyres_attn_gate_bwd_relu": (_I, [_P, _P, _P, _P, _P, _LL, _P]),
    "hyres_attn_gate_bwd_f16": (_I, [_P, _P, _P, _P, _P, _LL, _I, _P]),
    "hyres_attn_gate_bwd_relu_f16": (_I, [_P, _P, _P, _P, _P, _LL, _I, _P]),
    "hyres_relu_bwd_2d_f16": (_I, [_P, _I, _P, _I, _P, _I, _LL, _I, _I, _P]),
    "hyres_prelu_bwd_f16": (_I, [_P, _I, _P, _I, _P, _I, _LL, _I, _P, _P, _P, _LL, _I, _P]),
    "hyres_gdn_dnorm_f16": (_I, [_P, _P, _P, _P, _LL, _I, _I, _I, _P]),
    "hyres_se_bwd_f16": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _LL, _I, _P]),
    "hyres_spatial_attn_bwd_f16": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _LL, _I, _P]),
    "hyres_accumulate": (_I, [_P, _P, _LL, _P]),
    "hyres_accumulate_f16": (_I, [_P, _P, _LL, _P]),
    "hyres_scale": (_I, [_P, _P, _F, _P, _LL, _I, _P]),
    "hyres_add2d": (_I, [_P, _I, _P, _I, _LL, _I, _I, _P]),
    "hyres_add2d_f16": (_I, [_P, _I, _P, _I, _LL, _I, _I, _I, _P]),
    "hyres_mul": (_I, [_P, _P, _P, _LL, _P]),
    "hyres_zero": (_I, [_P, _LL, _P]),
    "hyres_gdn_reparam_fwd": (_I, [_P, _P, _P, _P, _I, _P]),
    "hyres_gdn_reparam_bwd": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _P]),
    "hyres_gdn_dnorm": (_I, [_P, _P, _P, _P, _LL, _I, _I, _P]),
    "hyres_uniform_noise": (_I, [_P, _LL, _ULL, _ULL, _P]),
    "hyres_uniform_noise_dev": (_I, [_P, _LL, _P, _ULL, _P]),
    "hyres_quantize": (_I, [_P, _I, _P, _LL, _P]),
    "hyres_gc_symbols": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _I, _P, _I, _P, _P, _P]),
    "hyres_gc_dequant": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _I, _I, _P]),
    "hyres_eb_symbols": (_I, [_P, _I, _P, _I, _I, _I, _I, _P, _P, _I, _I, _P]),
    "hyres_pmf_to_quantized_cdf": (_I, [_P, _I, _I, _P]),
    "hyres_rans_encode_with_indexes": (_I, [_P, _P, _LL, _P, _I, _P, _P, _I, _P, _LL, ctypes.POINTER(_LL)]),
    "hyres_rans_decode_with_indexes": (_I, [_P, _LL, _P, _LL, _P, _I, _P, _P, _I, _P]),
    "hyres_ckbd_anchor_fwd": (_I, [_P, _P, _I, _P, _P, _I, _I, _I, _I, _P]),
    "hyres_ckbd_nonanchor_gc_fwd": (_I, [_P, _P, _P, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P,
                                         _I, _I, _I, _I, _P]),
    "hyres_ckbd_gc_bwd": (_I, [_P, _P, _P, _P, _P, _I, _P, _P, _I, _P, _I, _I, _I, _I, _I, _P]),
    "hyres_ckbd_anchor_bwd": (_I, [_P, _P, _I, _I, _I, _I, _P]),
    "hyres_eb_pack": (_I, [_PP, _PP, _PP, _P, _P, _I, _P]),
    "hyres_eb_fwd": (_I, [_P, _P, _P, _I, _P, _P, _P, _LL, _I, _P]),
    "hyres_eb_bwd": (_I, [_P, _P, _P, _P, _P, _I, _I, _P, _P, _LL, _I, _P]),
    "hyres_eb_workspace_bytes": (_LL, [_LL, _I]),
    "hyres_eb_unpack_grad": (_I, [_P, _I, _PP, _PP, _PP, _PP, _PP, _P, _I, _I, _P]),
    "hyres_eb_aux_loss": (_I, [_P, _P, _P, _P, _P, _I, _P]),
    "hyres_bilinear_fwd": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _F, _F, _I, _P]),
    "hyres_bilinear_bwd": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _F, _F, _I, _P]),
    "hyres_bilinear_bwd_f16": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _F, _F, _I, _P]),
    "hyres_bilinear_bwd_prelu_workspace_bytes": (_LL, [_I, _I, _I, _I]),
    "hyres_bilinear_bwd_prelu": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _F, _F, _P, _I, _P, _P, _P, _LL, _I, _P]),
    "hyres_se_fwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _LL, _P]),
    "hyres_se_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _LL, _P]),
    "hyres_se_bwd_prelu": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _LL, _P]),
    "hyres_se_bwd_prelu_f16": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _LL, _I, _P]),
    "hyres_se_workspace_bytes": (_LL, [_I, _I, _I]),
    "hyres_spatial_attn_fwd": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "hyres_bilinear_fwd_f16": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _F, _F, _P]),
    "hyres_se_fwd_f16": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _LL, _P]),
    "hyres_spatial_attn_fwd_f16": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "hyres_spatial_attn_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _LL, _P]),
    "hyres_spatial_attn_workspace_bytes": (_LL, [_I, _I, _I]),
    "hyres_sa_fold_workspace_bytes": (_LL, [_LL, _I]),
    "hyres_sa_fold_bwd": (_I, [_P, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _LL, _I, _P, _LL, _P]),
    "hyres_sa_fold_bwd_f16": (_I, [_P, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _LL, _I, _P, _LL, _I, _P]),
    "hyres_spatial_attn_bwd_map": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _LL, _P]),
    "hyres_sum_log": (_I, [_P, _LL, _P, _P, _LL, _P]),
    "hyres_sum_sqdiff": (_I, [_P, _P, _LL, _P, _P, _LL, _P]),
    "hyres_reduce_workspace_bytes": (_LL, [_LL]),
    "hyres_scale_recip": (_I, [_P, _P, _F, _P, _LL, _P]),
    "hyres_scale_diff": (_I, [_P, _P, _P, _F, _P, _LL, _P]),
    "hyres_sumsq": (_I, [_P, _LL, _P, _P, _LL, _P]),
    "hyres_rd_finalize": (_I, [_P, _P, _F, _LL, _LL, _PP, _P]),
    "hyres_rd_bwd_coef": (_I, [_P, _P, _P, _P, _P, _P, _F, _LL, _LL, _P, _P]),
    "hyres_adam_step": (_I, [_P, _P, _P, _P, _LL, _D, _D, _D, _D, _P, _P, _D, _P, _I, _P]),
    "hyres_grad_scaler_update": (_I, [_P, _P, _P, _P, _D, _D, _I, _P]),
    "hyres_normalize_fwd": (_I, [_P, _P, _LL, _I, _P, _P, _P]),
    "hyres_normalize_bwd": (_I, [_P, _P, _LL, _I, _P, _P, _I, _P]),
    "hyres_relu_fwd": (_I, [_P, _P, _LL, _P]),
    "hyres_maxpool2_fwd": (_I, [_P, _P, _P, _I, _I, _I, _I, _P]),
    "hyres_maxpool2_bwd": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "hyres_absdiff_workspace_bytes": (_LL, [_LL]),
    "hyres_absdiff_mean": (_I, [_P, _P, _LL, _P, _I, _P, _LL, _P]),
    "hyres_absdiff_bwd": (_I, [_P, _P, _P, _LL, _P, _I, _P]),
}

_lib: Optional[ctypes.CDLL] = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libhyres_hip.so (no GPU needed to load; kernels need one to run)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"libhyres_hip.so not found at {path}: build it first (python __graft_entry__.py build or "
            f"python -m hyres_hip.build). There is no CPU/torch fallback for the HIP hot path.")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    # HYRES_FP32_GEMM: the fp32 convs' GEMM — bf16x6 (the library default: the three-way bf16 split on the bf16 MFMA)
    # or native (the fp32 MFMA); hyres_conv_tuning key 7
    mode = os.environ.get("HYRES_FP32_GEMM", "bf16x6")
    if mode not in ("bf16x6", "native"):
        raise ValueError(f"HYRES_FP32_GEMM={mode!r}: 'bf16x6' or 'native'")
    lib.hyres_conv_tuning(7, 1 if mode == "bf16x6" else 0, None)
    # HYRES_TUNE="key=value,...": A/B overrides of other hyres_conv_tuning keys (include/hyres_hip.h HYRES_TUNE_*)
    for kv in filter(None, os.environ.get("HYRES_TUNE", "").split(",")):
        k, v = kv.split("=")
        if lib.hyres_conv_tuning(int(k), int(v), None) != 0:
            raise ValueError(f"HYRES_TUNE: bad key {kv!r}")
    return lib


def exported_symbols():
    return list(_SIGS.keys())


class HipError(RuntimeError):
    pass


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().hyres_last_error_string()
        raise HipError(f"libhyres_hip {what} failed ({rc}): {msg.decode() if msg else ''}")


def call(name: str, *args):
    rc = getattr(load(), name)(*args)
    check(rc, name)


def stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def ptr_array(ts):
    arr = (ctypes.c_void_p * len(ts))(*[t.data_ptr() if t is not None else None for t in ts])
    return arr


def require_device(t: torch.Tensor) -> None:
    if not t.is_cuda:
        raise RuntimeError("hyres_hip ops need tensors on a ROCm GPU (no CPU fallback)")
