"""conv1x1_stream_b6_kernel (csrc/conv.hip, round 5): the fp32 1x1 convs of the ResidualUnits / RBBs and their
input-gradients (models/layers/attention.py:11-30, compressai ResidualBottleneckBlock at models/checkerboard.py:38-56)
on a per-wave streaming kernel with bf16x6 products, every epilogue operand issued a co tile ahead.

Against float64 torch, through the C-ABI (hyres_conv_forward with a hand-built epilogue, so every operand combination
the model's forward and backward use is reached): the three shapes (Ci, Co) in {(64, 128), (128, 64), (64, 64)} x
all eight combinations of residual / ReLU mask / accumulate, with ReLU, PReLU or no activation and the pre-activation
copy (out2), on a ragged pixel count (5 x 117 x 117 = 68,445: the last 32-pixel tile is partial), with the coalesced
(LDS-staged, hyres_conv_tuning key 11 = 1) and the MFMA-layout epilogue. Bar: normwise error
vs fp64 <= 2e-6 and no worse than twice the tiled implicit GEMM's on the same call (hyres_conv_tuning key 10 = 0).
"""
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


def _run(Ci, Co, F, act, out2, stream_on, ce=1):
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    D = dev()
    B, H, W = 5, 117, 117
    P = B * H * W
    x = _rand((P, Ci), 1).to(D)
    w = _rand((Co, Ci, 1, 1), 2, Ci ** -0.5).to(D)
    b = _rand((Co,), 3, 0.1).to(D)
    res = _rand((P, Co), 4).to(D)
    mask = _rand((P, Co), 5).to(D)
    old = _rand((P, Co), 6).to(D)
    slope = torch.full((1,), 0.25, device=D)
    y = old.clone() if F & 4 else torch.full((P, Co), float("nan"), device=D)
    pre = torch.full((P, Co), float("nan"), device=D)
    g = O._geom("hyres_geom_conv2d", B, H, W, Ci, Ci, Co, Co, 1, 1, 1, 0, 1)
    w2 = torch.empty((Co, Ci), device=D)
    L.call("hyres_conv_weight_prep", ctypes.byref(g), w.data_ptr(), w2.data_ptr(), 0, Ci, Co, 1, 1, 0, None, L.stream())
    e = L.Epilogue()
    e.kind, e.bias = L.EPI_BIAS, b.data_ptr()
    e.act = L.ACT_RELU_MASK if F & 2 else act
    if F & 1:
        e.res, e.ldres = res.data_ptr(), Co
    if F & 2:
        e.aux0, e.ld0 = mask.data_ptr(), Co
    e.accumulate = 1 if F & 4 else 0
    e.slope = slope.data_ptr()
    if out2:
        e.out2, e.ldo2 = pre.data_ptr(), Co
    old_key, old_ce = ctypes.c_int(0), ctypes.c_int(0)
    L.call("hyres_conv_tuning", 10, 1 if stream_on else 0, ctypes.byref(old_key))
    L.call("hyres_conv_tuning", 11, ce, ctypes.byref(old_ce))
    try:
        name = O.conv_variant(g, e, False)
        L.call("hyres_conv_forward", ctypes.byref(g), x.data_ptr(), w2.data_ptr(), Ci, y.data_ptr(), ctypes.byref(e),
               None, 0, L.stream())
        torch.cuda.synchronize()
    finally:
        L.call("hyres_conv_tuning", 10, old_key.value, None)
        L.call("hyres_conv_tuning", 11, old_ce.value, None)
    # float64 reference of the epilogue order: acc + bias (+ res) -> out2 -> act / mask -> (+ old)
    r = x.double() @ w.double().reshape(Co, Ci).t() + b.double()
    if F & 1:
        r = r + res.double()
    ref_pre = r.clone()
    if F & 2:
        r = torch.where(mask.double() > 0, r, torch.zeros_like(r))
    elif act == L.ACT_RELU:
        r = torch.relu(r)
    elif act == L.ACT_PRELU:
        r = torch.where(r >= 0, r, 0.25 * r)
    if F & 4:
        r = r + old.double()
    errs = [rel_err(y.double().cpu(), r.cpu())]
    if out2:
        errs.append(rel_err(pre.double().cpu(), ref_pre.cpu()))
    return name, max(errs)


@pytest.mark.parametrize("Ci,Co,F", [(c, o, f) for (c, o) in ((64, 128), (128, 64), (64, 64)) for f in range(8)]
                         + [(128, 128, 0), (128, 128, 2)])
def test_stream_b6_matches_fp64(Ci, Co, F):
    """(128, 128) (round 6): the operand-free and ReLU-mask forms only (one wave per SIMD by its LDS)."""
    from hyres_hip import _lib as L
    acts = [L.ACT_RELU, L.ACT_PRELU, L.ACT_NONE]
    act = acts[(F + Ci // 64) % 3]
    out2 = F in (1, 4, 7)
    name_s, err_s = _run(Ci, Co, F, act, out2, True)
    name_m, err_m = _run(Ci, Co, F, act, out2, True, ce=0)
    name_t, err_t = _run(Ci, Co, F, act, out2, False)
    print(f"{Ci}->{Co} F={F} act={act} out2={out2}: {name_s} {err_s:.2e}, {name_m} {err_m:.2e}, {name_t} {err_t:.2e}")
    assert name_s.startswith("conv1x1_stream_b6_kernel<") and name_s.endswith(", true>"), name_s
    assert name_m.startswith("conv1x1_stream_b6_kernel<") and name_m.endswith(", false>"), name_m
    assert not name_t.startswith("conv1x1_stream_b6"), name_t
    for err in (err_s, err_m):
        assert err < 2e-6 and err <= 2 * err_t + 1e-9


def _run_sab(acc, stream_on):
    """The HYRES_EPI_SA_BWD input-gradient of MultiScaleRefine's fusion 1x1 (64 -> 192): y = (W^T g + gm[p][0]) +
    (n == argmax[p] ? gm[p][1] : 0) (+ old y), through the C-ABI on the streaming kernel or the implicit GEMM."""
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    D = dev()
    B, H, W = 5, 117, 117
    P, Ci, Co = B * H * W, 64, 192
    x = _rand((P, Ci), 11).to(D)
    w = _rand((Co, Ci, 1, 1), 12, Ci ** -0.5).to(D)
    gm = _rand((P, 2), 13).to(D)
    am = torch.randint(0, Co, (P,), generator=torch.Generator().manual_seed(14), dtype=torch.int32).to(D)
    old = _rand((P, Co), 15).to(D)
    y = old.clone() if acc else torch.full((P, Co), float("nan"), device=D)
    g = O._geom("hyres_geom_conv2d", B, H, W, Ci, Ci, Co, Co, 1, 1, 1, 0, 1)
    w2 = torch.empty((Co, Ci), device=D)
    L.call("hyres_conv_weight_prep", ctypes.byref(g), w.data_ptr(), w2.data_ptr(), 0, Ci, Co, 1, 1, 0, None, L.stream())
    e = L.Epilogue()
    e.kind = L.EPI_SA_BWD
    e.aux0, e.ld0 = gm.data_ptr(), 2
    e.aux2 = am.data_ptr()
    e.accumulate = int(acc)
    old_key = ctypes.c_int(0)
    L.call("hyres_conv_tuning", 21, 1 if stream_on else 0, ctypes.byref(old_key))
    try:
        name = O.conv_variant(g, e, False)
        L.call("hyres_conv_forward", ctypes.byref(g), x.data_ptr(), w2.data_ptr(), Ci, y.data_ptr(), ctypes.byref(e),
               None, 0, L.stream())
        torch.cuda.synchronize()
    finally:
        L.call("hyres_conv_tuning", 21, old_key.value, None)
    r = x.double() @ w.double().reshape(Co, Ci).t() + gm[:, :1].double()
    r = r + torch.where(torch.arange(Co, device=D)[None, :] == am[:, None].long(), gm[:, 1:].double(),
                        torch.zeros((), dtype=torch.float64, device=D))
    if acc:
        r = r + old.double()
    return name, rel_err(y.double().cpu(), r.cpu())


@pytest.mark.parametrize("acc", [False, True])
def test_stream_b6_sa_bwd_matches_fp64(acc):
    """conv1x1_stream_b6_kernel<6, 4, 8 | acc> (round 6, hyres_conv_tuning key 21): the SA_BWD input-gradient 64 -> 192
    on a ragged pixel count vs fp64 (2e-6 normwise, no worse than twice the implicit GEMM it replaces on the same
    call)."""
    name_s, err_s = _run_sab(acc, True)
    name_t, err_t = _run_sab(acc, False)
    print(f"SA_BWD 64->192 acc={acc}: {name_s} {err_s:.2e}, {name_t} {err_t:.2e}")
    assert name_s == f"conv1x1_stream_b6_kernel<6, 4, {8 | (4 if acc else 0)}, true>", name_s
    assert not name_t.startswith("conv1x1_stream_b6"), name_t
    assert err_s < 2e-6 and err_s <= 2 * err_t + 1e-9, (err_s, err_t)


def _run_rowscale(act, stream_on):
    """The HYRES_EPI_ROWSCALE forward of MultiScaleRefine's fusion 1x1 with SpatialAttention folded (192 -> 64):
    y = act(attn[p] * (W x)[p] + b), out2 = the pre-activation, through the C-ABI on the streaming kernel or the
    implicit GEMM."""
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    D = dev()
    B, H, W = 5, 117, 117
    P, Ci, Co = B * H * W, 192, 64
    x = _rand((P, Ci), 21).to(D)
    w = _rand((Co, Ci, 1, 1), 22, Ci ** -0.5).to(D)
    b = _rand((Co,), 23, 0.1).to(D)
    sc = torch.rand(P, generator=torch.Generator().manual_seed(24)).to(D)
    slope = torch.full((1,), 0.25, device=D)
    y = torch.full((P, Co), float("nan"), device=D)
    pre = torch.full((P, Co), float("nan"), device=D)
    g = O._geom("hyres_geom_conv2d", B, H, W, Ci, Ci, Co, Co, 1, 1, 1, 0, 1)
    w2 = torch.empty((Co, Ci), device=D)
    L.call("hyres_conv_weight_prep", ctypes.byref(g), w.data_ptr(), w2.data_ptr(), 0, Ci, Co, 1, 1, 0, None, L.stream())
    e = L.Epilogue()
    e.kind = L.EPI_ROWSCALE
    e.act = act
    e.bias = b.data_ptr()
    e.slope = slope.data_ptr()
    e.aux1, e.ld1 = sc.data_ptr(), 1
    e.out2, e.ldo2 = pre.data_ptr(), Co
    old_key = ctypes.c_int(0)
    L.call("hyres_conv_tuning", 21, 1 if stream_on else 0, ctypes.byref(old_key))
    try:
        name = O.conv_variant(g, e, False)
        L.call("hyres_conv_forward", ctypes.byref(g), x.data_ptr(), w2.data_ptr(), Ci, y.data_ptr(), ctypes.byref(e),
               None, 0, L.stream())
        torch.cuda.synchronize()
    finally:
        L.call("hyres_conv_tuning", 21, old_key.value, None)
    r = (x.double() @ w.double().reshape(Co, Ci).t()) * sc.double()[:, None] + b.double()
    ra = r
    if act == L.ACT_PRELU:
        ra = torch.where(r >= 0, r, 0.25 * r)
    elif act == L.ACT_RELU:
        ra = r.clamp_min(0)
    return name, max(rel_err(y.double().cpu(), ra.cpu()), rel_err(pre.double().cpu(), r.cpu())), y


@pytest.mark.parametrize("act", ["prelu", "none", "relu"])
def test_stream_b6_rowscale_matches_fp64(act):
    """conv1x1_stream_b6_kernel<2, 12, 16> (round 6, hyres_conv_tuning key 21): the fusion 1x1's ROWSCALE forward
    192 -> 64 with the pre-activation copy, on a ragged pixel count vs fp64 (2e-6 normwise, no worse than twice the
    implicit GEMM it replaces on the same call)."""
    from hyres_hip import _lib as L
    a = {"prelu": L.ACT_PRELU, "none": L.ACT_NONE, "relu": L.ACT_RELU}[act]
    name_s, err_s, y_s = _run_rowscale(a, True)
    name_t, err_t, y_t = _run_rowscale(a, False)
    # the two kernels sum K in different orders: equal outputs would mean the stream build never ran (the label is
    # the launcher's choice function, which does not see pointer alignment)
    assert not torch.equal(y_s, y_t)
    print(f"ROWSCALE 192->64 {act}: {name_s} {err_s:.2e}, {name_t} {err_t:.2e}")
    assert name_s == "conv1x1_stream_b6_kernel<2, 12, 16, true>", name_s
    assert not name_t.startswith("conv1x1_stream_b6"), name_t
    assert err_s < 2e-6 and err_s <= 2 * err_t + 1e-9, (err_s, err_t)
