"""Deferred split-K weight-gradient reduces (hyres_conv_wgrad_deferred + hyres_wgrad_reduce_jobs, ops.WgradBatch).

The weight gradient of every conv in loss.backward() (reference: src/utils/engine.py:63 through the convs of
models/checkerboard.py:35-88 and models/layers/*.py) is a GEMM over the batch's pixels, split over pixel ranges
into partial slabs. The deferred form launches the GEMMs per layer and reduces many layers' slabs in one launch;
it must give exactly the per-layer path's bits (same plan, same per-output summation order), and a whole
training step must be bit-identical with and without deferral and from run to run (determinism).
"""
import ctypes

import pytest
import torch

from helpers import build_model, load_npz

pytestmark = pytest.mark.gpu

# (B, H, W, Ci, Co, K, stride, pad, dil, bias, f16): the halo 3x3 (fp32 / AMP), dilated 3x3, 1x1 with a bias
# (wgrad1x1, two groups), a 5x5 stride-2, the 3-channel image layer (swapped, colsum bias), a thin layer
# (Co = 3) and a small 32^2 grid with many splits
CASES = [
    (4, 64, 64, 64, 64, 3, 1, 1, 1, True, False),
    (4, 64, 64, 64, 64, 3, 1, 1, 1, True, True),
    (2, 64, 64, 64, 64, 3, 1, 2, 2, False, False),
    (4, 64, 64, 128, 64, 1, 1, 0, 1, True, False),
    (2, 64, 64, 64, 128, 5, 2, 2, 1, True, False),
    (2, 64, 64, 3, 64, 5, 2, 2, 1, True, False),
    (2, 64, 64, 64, 3, 3, 1, 1, 1, True, False),
    (16, 16, 16, 96, 96, 3, 1, 1, 1, True, False),
]


def _desc(L, B, H, W, Ci, Co, K, stride, pad, dil, f16):
    d = L.WgradDesc()
    L.call("hyres_wgrad_desc_conv2d", ctypes.byref(d), B, H, W, Ci, Ci, Co, Co, K, K, stride, pad, dil)
    d.sm = Ci * K * K
    d.accumulate = 1
    d.f16_operands = int(f16)
    return d


def _run(L, lib, case, deferred, seed=0):
    B, H, W, Ci, Co, K, stride, pad, dil, bias, f16 = case
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(seed)
    Ho = (H + 2 * pad - dil * (K - 1) - 1) // stride + 1
    Wo = (W + 2 * pad - dil * (K - 1) - 1) // stride + 1
    x = torch.randn(B, H, W, Ci, generator=g).to(dev)
    gy = torch.randn(B, Ho, Wo, Co, generator=g).to(dev)
    dw = (0.1 * torch.randn(Co, Ci, K, K, generator=g)).to(dev)  # accumulate onto a nonzero gradient
    db = (0.1 * torch.randn(Co, generator=g)).to(dev) if bias else None
    d = _desc(L, B, H, W, Ci, Co, K, stride, pad, dil, f16)
    nbytes = int(lib.hyres_wgrad_workspace_bytes(ctypes.byref(d)))
    ws = torch.full((max(nbytes, 16),), 0x7F, dtype=torch.uint8, device=dev)
    st = L.stream()
    if deferred:
        jobs = (L.WgradJob * 2)()
        nj = ctypes.c_int(0)
        L.call("hyres_conv_wgrad_deferred", ctypes.byref(d), gy.data_ptr(), x.data_ptr(), dw.data_ptr(),
               None if db is None else db.data_ptr(), ws.data_ptr(), ws.numel(), jobs, ctypes.byref(nj), st)
        assert 1 <= nj.value <= 2
        L.call("hyres_wgrad_reduce_jobs", jobs, nj.value, st)
    else:
        L.call("hyres_conv_wgrad", ctypes.byref(d), gy.data_ptr(), x.data_ptr(), dw.data_ptr(),
               None if db is None else db.data_ptr(), ws.data_ptr(), ws.numel(), st)
    torch.cuda.synchronize()
    return dw, db, (x, gy)


@pytest.mark.parametrize("case", CASES)
def test_deferred_reduce_bit_identical(case):
    import hyres_hip._lib as L
    lib = L.load()
    dw0, db0, (x, gy) = _run(L, lib, case, deferred=False)
    dw1, db1, _ = _run(L, lib, case, deferred=True)
    assert torch.equal(dw0, dw1)
    if db0 is not None:
        assert torch.equal(db0, db1)
    # and it is the gradient: fp64 check of the accumulated result
    B, H, W, Ci, Co, K, stride, pad, dil, bias, f16 = case
    g = torch.Generator(device="cpu").manual_seed(0)
    torch.randn(B, H, W, Ci, generator=g)
    Ho = (H + 2 * pad - dil * (K - 1) - 1) // stride + 1
    Wo = (W + 2 * pad - dil * (K - 1) - 1) // stride + 1
    torch.randn(B, Ho, Wo, Co, generator=g)
    dw_init = (0.1 * torch.randn(Co, Ci, K, K, generator=g)).double()
    xd, gd = x.double().permute(0, 3, 1, 2).cpu(), gy.double().permute(0, 3, 1, 2).cpu()
    if f16:
        xd, gd = xd.half().double(), gd.half().double()
    ref = dw_init + torch.nn.grad.conv2d_weight(xd, (Co, Ci, K, K), gd, stride=stride, padding=pad, dilation=dil)
    err = float((dw1.double().cpu() - ref).abs().max() / ref.abs().max())
    assert err < 1e-5, err


def test_reduce_jobs_batch_of_layers():
    """Many layers' jobs in one hyres_wgrad_reduce_jobs call (more than HYRES_WGRAD_MAX_JOBS: two launches)."""
    import hyres_hip._lib as L
    lib = L.load()
    dev = torch.device("cuda:0")
    st = L.stream()
    refs, outs, keep, jobs = [], [], [], []
    for i in range(30):  # 30 layers x 2 jobs (weight + bias) = 60 > 48
        case = CASES[i % len(CASES)]
        if case[-1] or not case[-2]:
            case = CASES[3]
        B, H, W, Ci, Co, K, stride, pad, dil, bias, f16 = case
        dw0, db0, (x, gy) = _run(L, lib, case, deferred=False, seed=i)
        refs.append((dw0, db0))
        g = torch.Generator(device="cpu").manual_seed(i)
        torch.randn(B, H, W, Ci, generator=g)
        Ho = (H + 2 * pad - dil * (K - 1) - 1) // stride + 1
        Wo = (W + 2 * pad - dil * (K - 1) - 1) // stride + 1
        torch.randn(B, Ho, Wo, Co, generator=g)
        dw = (0.1 * torch.randn(Co, Ci, K, K, generator=g)).to(dev)
        db = (0.1 * torch.randn(Co, generator=g)).to(dev)
        d = _desc(L, B, H, W, Ci, Co, K, stride, pad, dil, f16)
        nbytes = int(lib.hyres_wgrad_workspace_bytes(ctypes.byref(d)))
        ws = torch.empty((max(nbytes, 16),), dtype=torch.uint8, device=dev)
        j2 = (L.WgradJob * 2)()
        nj = ctypes.c_int(0)
        L.call("hyres_conv_wgrad_deferred", ctypes.byref(d), gy.data_ptr(), x.data_ptr(), dw.data_ptr(),
               db.data_ptr(), ws.data_ptr(), ws.numel(), j2, ctypes.byref(nj), st)
        jobs.extend(j2[k] for k in range(nj.value))
        keep.extend([ws, x, gy])
        outs.append((dw, db))
    arr = (L.WgradJob * len(jobs))(*jobs)
    L.call("hyres_wgrad_reduce_jobs", arr, len(jobs), st)
    torch.cuda.synchronize()
    for (a, b), (c, e) in zip(refs, outs):
        assert torch.equal(a, c)
        if b is not None:
            assert torch.equal(b, e)


NQ_KEYS = {"z": "noise_z", "y_anchor": "noise_y_anchor", "y_non_anchor": "noise_y_non_anchor", "y": "noise_y"}


def _train_grads(defer, amp=False):
    """One noisequant train step on the reference fixture batch with its recorded noise injected."""
    from hyres_hip import ops
    from hyres_hip.loss import RateDistortionLoss
    g = load_npz("hyres_train_nq_b2_64.npz")
    dev = torch.device("cuda:0")
    old = ops.WgradBatch.enabled
    ops.WgradBatch.enabled = defer
    try:
        net, _ = build_model()
        net = net.to(dev).train()
        net.residual_model.noise.injected = {k: g[src].permute(0, 2, 3, 1).contiguous().to(dev)
                                             for k, src in NQ_KEYS.items()}
        x = g["x"].to(dev)
        with torch.autocast("cuda", dtype=torch.float16, enabled=amp):
            out = net(g["x"], noisequant=True, jpeg=(g["jpeg_decoded"], float(g["jpeg_bpp"])))
            crit = RateDistortionLoss(lmbda=0.045, alpha=0)(out, x)
        crit["loss"].backward()
        torch.cuda.synchronize()
        assert ops.WgradBatch.pending() == 0
        return {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.grad is not None}
    finally:
        ops.WgradBatch.enabled = old


@pytest.mark.parametrize("amp", [False, True])
def test_train_step_gradients_bit_identical_deferred_and_deterministic(amp):
    g_off = _train_grads(False, amp)
    g_on = _train_grads(True, amp)
    g_on2 = _train_grads(True, amp)
    assert g_off.keys() == g_on.keys() and len(g_on) > 100
    for n in g_off:
        assert torch.equal(g_off[n], g_on[n]), n
        assert torch.equal(g_on[n], g_on2[n]), n
