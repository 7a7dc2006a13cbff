"""The fp16-activation streaming 1x1 conv (csrc/conv.hip conv1x1_stream_h_kernel: io_f16 = 3, Ci / Co in {64, 96, 128},
>= 16384 pixels, no streamed epilogue operand) and, for the layers WITH one (residual, ReLU mask, old y),
conv1x1_stream_hf_kernel (round 6: operands a co tile ahead, row-shaped epilogue through LDS), which must equal the
f16 tiles it replaces bit for bit (hyres_conv_tuning key 17 = 0 routes them back). Against torch float64 on the same fp16 values (X fp16, W rounded to fp16, fp32 bias, fp16 residual / mask /
old y), rounded to fp16 once at the end: within one fp16 ulp of the output plus fp32 summation-order slack (2e-3
max-norm); strided X / Y and a ragged pixel count; the routing checked by name."""
import ctypes

import pytest
import torch

from helpers import rel_err

pytestmark = pytest.mark.gpu


def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


def _rand(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(shape, generator=g) * 2 - 1) * scale


@pytest.mark.parametrize("case", [
    # P (pixels), Ci, Co, act, res, acc, ld pad
    (16384, 64, 128, "relu", False, False, 0),
    (16384, 128, 64, "none", False, False, 0),
    (4 * 64 * 64 + 17, 96, 96, "relu", False, False, 0),  # ragged last 32-pixel tile
    (16384, 128, 128, "none", False, False, 24),            # strided X / Y rows
    (16384, 64, 128, "relu", True, False, 0),               # residual
    (16384, 128, 64, "mask", False, True, 0),               # dgrad: ReLU mask + accumulate
    (16384, 64, 128, "mask", True, True, 32),               # residual + mask + accumulate, strided
    (4 * 64 * 64 + 17, 128, 128, "relu", True, False, 0),    # residual, ragged last tile
    (65536, 64, 64, "none", False, True, 0),                # accumulate only
    (16384, 128, 128, "mask", False, False, 8),             # mask only, strided
])
def test_stream_h_matches_torch(case):
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    P, Ci, Co, act, use_res, acc, pad = case
    D = dev()
    ldx, ldy = Ci + pad, Co + pad
    x = _rand((P, ldx), 1).half().to(D)
    w = _rand((Co, Ci), 2, Ci ** -0.5).to(D)
    b = _rand((Co,), 3, 0.1).to(D)
    res = _rand((P, ldy), 4).half().to(D) if use_res else None
    mask = _rand((P, ldy), 5).half().to(D) if act == "mask" else None
    y0 = _rand((P, ldy), 6).half().to(D)
    y = y0.clone()
    g = O._geom("hyres_geom_conv2d", 1, 1, P, Ci, ldx, Co, ldy, 1, 1, 1, 0, 1)
    e = L.Epilogue()
    e.kind = L.EPI_BIAS
    e.act = {"none": L.ACT_NONE, "relu": L.ACT_RELU, "mask": L.ACT_RELU_MASK}[act]
    e.bias = b.data_ptr()
    if res is not None:
        e.res, e.ldres = res.data_ptr(), ldy
    if mask is not None:
        e.aux0, e.ld0 = mask.data_ptr(), ldy
    e.accumulate = int(acc)
    e.f16_operands = 1
    e.io_f16 = L.IO_X16 | L.IO_Y16
    streamed = res is not None or mask is not None or acc
    want = "conv1x1_stream_hf_kernel" if streamed else "conv1x1_stream_h_kernel"
    assert O.conv_variant(g, e, False).startswith(want), O.conv_variant(g, e, False)
    L.call("hyres_conv_forward", ctypes.byref(g), x.data_ptr(), w.data_ptr(), Ci, y.data_ptr(), ctypes.byref(e),
           None, 0, L.stream())
    torch.cuda.synchronize()
    if streamed:  # the f16 tiles it replaces: the same products and epilogue, bit for bit
        yt = y0.clone()
        L.call("hyres_conv_tuning", 17, 0, None)
        try:
            assert O.conv_variant(g, e, False).startswith("conv_fwd_h_kernel"), O.conv_variant(g, e, False)
            L.call("hyres_conv_forward", ctypes.byref(g), x.data_ptr(), w.data_ptr(), Ci, yt.data_ptr(),
                   ctypes.byref(e), None, 0, L.stream())
            torch.cuda.synchronize()
        finally:
            L.call("hyres_conv_tuning", 17, 1, None)
        assert torch.equal(y, yt), float((y.float() - yt.float()).abs().max())
    ref = x[:, :Ci].double() @ w.half().double().t() + b.double()
    if res is not None:
        ref = ref + res[:, :Co].double()
    if act == "relu":
        ref = ref.clamp_min(0)
    elif act == "mask":
        ref = ref * (mask[:, :Co].double() > 0)
    if acc:
        ref = ref + y0[:, :Co].double()
    ref = ref.half().double()
    err = rel_err(y[:, :Co].double().cpu(), ref.cpu())
    print(case, f"max-norm error vs fp64 {err:.2e}")
    assert err < 2e-3
    if pad:  # the padding columns are untouched
        assert torch.equal(y[:, Co:], y0[:, Co:])
