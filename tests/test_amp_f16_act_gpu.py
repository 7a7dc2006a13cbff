"""AMP training with fp16 SAVED activations (``ops.AMP_F16_ACT``): inside an ``f16_region`` the forward outputs
that backward reads are stored as fp16 in HBM — as torch autocast's conv outputs are fp16 tensors
(/root/reference/src/utils/engine.py:32, train.sh:19 ``--mixed-precision``) — and (``ops.AMP_F16_GRAD``, round 4)
their gradients are fp16 as well, as autograd gives an fp16 tensor an fp16 gradient.

Why exact comparisons are possible: every kernel computes in fp32 from its operands; the fp16-storage
variants only change how a saved activation is read (8-byte loads of 4 halves, converted exactly) or how
an output is written (rounded once). So on fp16-representable inputs
  * each fp16-saved-activation backward entry point equals its fp32 twin BIT FOR BIT;
  * a conv / deconv / GDN layer's weight and input gradients equal those of the fp32-storage layer bit for
    bit when no activation mask is involved (the f16 MFMA kernels round their operands to fp16 anyway; the
    fp32 weight-gradient kernels read an exact fp32 copy of the fp16 operand);
  * a ResidualUnit chain matches torch (float64) with the same fp16 rounding points to 1e-4.
The whole model under autocast is pinned to the reference's own autocast run in
test_parity_gpu.py::test_amp_matches_reference_autocast_fixture (which now runs with fp16 activations)."""
import pytest
import torch
import torch.nn.functional as F

from helpers import rel_err

pytestmark = pytest.mark.gpu


def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


def _rand(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(shape, generator=g) * 2 - 1) * scale


def _h(t):
    """fp16-representable fp32 copy."""
    return t.half().float()


# ------------------------------------------------------------------------------------------ elementwise
def test_f16_saved_activation_backward_entry_points_bitwise():
    """relu / PReLU / attention gate / GDN dnorm / SE / spatial-attention backward with fp16 saved operands
    equal the fp32 entry points on the same (fp16-representable) values, bit for bit — except where a sum of
products feeds the result (the PReLU slope gradient, the spatial-attention logit sums): there the two
instantiations contract their multiply-adds differently (v_fma_mix on the fp16 operand), measured 1 ulp,
checked to 1e-6."""
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    D = dev()
    B, H, W, C = 2, 16, 24, 64
    P = B * H * W
    y = _h(_rand((P, C), 1)).to(D)
    g = _rand((P, C), 2).to(D)
    s = L.stream()

    def pair(name, args16, args32, outs, tol=None):
        res = []
        for fn, args in ((name + "_f16", args16), (name, args32)):
            for o in outs:
                o.zero_()
            L.call(fn, *args)
            res.append([o.clone() for o in outs])
        torch.cuda.synchronize()
        for k, (a, b) in enumerate(zip(*res)):
            if tol is not None and tol[k] > 0:  # a reduction: FMA contraction may differ between the two builds
                assert rel_err(a.cpu(), b.cpu()) <= tol[k], (name, k)
                continue
            if not torch.equal(a, b):
                bad = (a != b).nonzero()
                print(name, k, "mismatches", bad.shape[0], "first", bad[:4].tolist(), a[tuple(bad[0])].item(),
                      b[tuple(bad[0])].item())
            assert torch.equal(a, b), (name, k)

    gx = torch.empty(P, C, device=D)
    yh = y.half()
    pair("hyres_relu_bwd_2d", (yh.data_ptr(), C, g.data_ptr(), C, gx.data_ptr(), C, P, C, 0, s),
         (y.data_ptr(), C, g.data_ptr(), C, gx.data_ptr(), C, P, C, s), [gx])
    slope = torch.tensor([0.25], device=D)
    dslope = torch.zeros(1, device=D)
    ws = torch.empty(int(L.load().hyres_reduce_workspace_bytes(P * C)), dtype=torch.uint8, device=D)
    pair("hyres_prelu_bwd", (yh.data_ptr(), C, g.data_ptr(), C, gx.data_ptr(), C, P, C, slope.data_ptr(),
                             dslope.data_ptr(), ws.data_ptr(), ws.numel(), 0, s),
         (y.data_ptr(), C, g.data_ptr(), C, gx.data_ptr(), C, P, C, slope.data_ptr(), dslope.data_ptr(),
          ws.data_ptr(), ws.numel(), s), [gx, dslope], tol=[0, 1e-6])
    b = _h(_rand((P, C), 3)).to(D)
    bh = b.half()
    ga, gb = torch.empty(P, C, device=D), torch.empty(P, C, device=D)
    pair("hyres_attn_gate_bwd", (yh.data_ptr(), bh.data_ptr(), g.data_ptr(), ga.data_ptr(), gb.data_ptr(), P * C, 0, s),
         (y.data_ptr(), b.data_ptr(), g.data_ptr(), ga.data_ptr(), gb.data_ptr(), P * C, s), [ga, gb])
    nrm = _h(_rand((P, C), 4).abs() + 0.5).to(D)
    nh = nrm.half()
    dn = torch.empty(P, C, device=D)
    for inv in (0, 1):
        pair("hyres_gdn_dnorm", (g.data_ptr(), yh.data_ptr(), nh.data_ptr(), dn.data_ptr(), P, C, inv, 0, s),
             (g.data_ptr(), y.data_ptr(), nrm.data_ptr(), dn.data_ptr(), P, C, inv, s), [dn])
    # SE / spatial attention: run the fp32 forward on the fp16-representable x for the saved state, then both
    # backward flavours
    Cr = 4
    w1 = _rand((Cr, C), 5, 0.2).to(D)
    w2 = _rand((C, Cr), 6, 0.2).to(D)
    pooled, hidden, sgate = (torch.empty(B, C, device=D), torch.empty(B, Cr, device=D), torch.empty(B, C, device=D))
    yse = torch.empty(P, C, device=D)
    wsb = int(L.load().hyres_se_workspace_bytes(B, H * W, C)) + B * C * 4
    ws = torch.empty(wsb, dtype=torch.uint8, device=D)
    L.call("hyres_se_fwd", y.data_ptr(), w1.data_ptr(), w2.data_ptr(), yse.data_ptr(), pooled.data_ptr(),
           hidden.data_ptr(), sgate.data_ptr(), B, H * W, C, Cr, ws.data_ptr(), ws.numel(), s)
    gw1, gw2 = torch.zeros(Cr, C, device=D), torch.zeros(C, Cr, device=D)
    pair("hyres_se_bwd", (yh.data_ptr(), g.data_ptr(), w1.data_ptr(), w2.data_ptr(), pooled.data_ptr(),
                          hidden.data_ptr(), sgate.data_ptr(), gx.data_ptr(), gw1.data_ptr(), gw2.data_ptr(), B, H * W,
                          C, Cr, ws.data_ptr(), ws.numel(), 0, s),
         (y.data_ptr(), g.data_ptr(), w1.data_ptr(), w2.data_ptr(), pooled.data_ptr(), hidden.data_ptr(),
          sgate.data_ptr(), gx.data_ptr(), gw1.data_ptr(), gw2.data_ptr(), B, H * W, C, Cr, ws.data_ptr(),
          ws.numel(), s), [gx, gw1, gw2])
    wsa = _rand((1, 2, 7, 7), 7, 0.1).to(D)
    pooled2 = torch.empty(P, 2, device=D)
    amax = torch.empty(P, dtype=torch.int32, device=D)
    attn = torch.empty(P, device=D)
    ysa = torch.empty(P, C, device=D)
    L.call("hyres_spatial_attn_fwd", y.data_ptr(), wsa.data_ptr(), pooled2.data_ptr(), amax.data_ptr(),
           attn.data_ptr(), ysa.data_ptr(), B, H, W, C, s)
    gw = torch.zeros(1, 2, 7, 7, device=D)
    wsb = int(L.load().hyres_spatial_attn_workspace_bytes(B, H, W))
    ws = torch.empty(wsb, dtype=torch.uint8, device=D)
    pair("hyres_spatial_attn_bwd", (yh.data_ptr(), wsa.data_ptr(), pooled2.data_ptr(), amax.data_ptr(),
                                    attn.data_ptr(), g.data_ptr(), gx.data_ptr(), gw.data_ptr(), B, H, W, C,
                                    ws.data_ptr(), ws.numel(), 0, s),
         (y.data_ptr(), wsa.data_ptr(), pooled2.data_ptr(), amax.data_ptr(), attn.data_ptr(), g.data_ptr(),
          gx.data_ptr(), gw.data_ptr(), B, H, W, C, ws.data_ptr(), ws.numel(), s), [gx, gw], tol=[1e-6, 1e-6])


def test_f16_gradient_backward_entry_points_match_rounded_fp32():
    """g16 = 1 (AMP fp16 activation gradients, autocast's own semantics): the same entry points with the incoming
    gradient and the produced gradients fp16. Every kernel computes in fp32 from exactly converted operands and
    rounds its output once, so on fp16-representable inputs each fp16 gradient equals the fp32 entry point's
    result rounded to fp16, BIT FOR BIT (weight / slope gradients stay fp32: 1e-6 where FMA contraction may
    differ). Also the fp16 add2d / accumulate / colsum / bilinear-backward entry points against fp32."""
    from hyres_hip import _lib as L
    D = dev()
    B, H, W, C = 2, 16, 24, 64
    P = B * H * W
    s = L.stream()
    y = _h(_rand((P, C), 1)).to(D)
    yh = y.half()
    g = _h(_rand((P, C), 2)).to(D)
    gh = g.half()

    def check(got16, want32, what):
        # bit for bit, except that the compiler may fuse a kernel's last fp32 multiply with the fp16 store
        # (v_fma_mixlo_f16: ONE rounding of the exact product, where fp32-then-fp16 rounds twice) — that differs by
        # one fp16 ulp at double-rounding ties only: a handful of elements, never more than 1 ulp
        want = want32.half()
        if not torch.equal(got16, want):
            bad = (got16 != want).nonzero()
            m = got16 != want  # (+0 / -0 compare equal)
            ulps = (got16[m].view(torch.int16).int() - want[m].view(torch.int16).int()).abs().max().item()
            print(what, "mismatches", bad.shape[0], "max ulps", ulps, got16[tuple(bad[0])].item(),
                  want[tuple(bad[0])].item())
            assert ulps <= 1 and bad.shape[0] <= max(4, got16.numel() // 4096), what

    gx32, gx16 = torch.empty(P, C, device=D), torch.empty(P, C, device=D, dtype=torch.float16)
    L.call("hyres_relu_bwd_2d", y.data_ptr(), C, g.data_ptr(), C, gx32.data_ptr(), C, P, C, s)
    L.call("hyres_relu_bwd_2d_f16", yh.data_ptr(), C, gh.data_ptr(), C, gx16.data_ptr(), C, P, C, 1, s)
    check(gx16, gx32, "relu")
    slope = torch.tensor([0.25], device=D)
    d32, d16 = torch.zeros(1, device=D), torch.zeros(1, device=D)
    ws = torch.empty(int(L.load().hyres_reduce_workspace_bytes(P * C)), dtype=torch.uint8, device=D)
    L.call("hyres_prelu_bwd", y.data_ptr(), C, g.data_ptr(), C, gx32.data_ptr(), C, P, C, slope.data_ptr(),
           d32.data_ptr(), ws.data_ptr(), ws.numel(), s)
    L.call("hyres_prelu_bwd_f16", yh.data_ptr(), C, gh.data_ptr(), C, gx16.data_ptr(), C, P, C, slope.data_ptr(),
           d16.data_ptr(), ws.data_ptr(), ws.numel(), 1, s)
    check(gx16, gx32, "prelu")
    assert rel_err(d16.cpu(), d32.cpu()) <= 1e-6
    b = _h(_rand((P, C), 3)).to(D)
    bh = b.half()
    ga32, gb32 = torch.empty(P, C, device=D), torch.empty(P, C, device=D)
    ga16, gb16 = torch.empty_like(gx16), torch.empty_like(gx16)
    L.call("hyres_attn_gate_bwd", y.data_ptr(), b.data_ptr(), g.data_ptr(), ga32.data_ptr(), gb32.data_ptr(), P * C, s)
    L.call("hyres_attn_gate_bwd_f16", yh.data_ptr(), bh.data_ptr(), gh.data_ptr(), ga16.data_ptr(), gb16.data_ptr(),
           P * C, 1, s)
    check(ga16, ga32, "gate a")
    check(gb16, gb32, "gate b")
    nrm = _h(_rand((P, C), 4).abs() + 0.5).to(D)
    nrm16 = nrm.half()  # held for the call (a temporary's block returns to the allocator before the kernel runs)
    for inv in (0, 1):
        L.call("hyres_gdn_dnorm", g.data_ptr(), y.data_ptr(), nrm.data_ptr(), gx32.data_ptr(), P, C, inv, s)
        L.call("hyres_gdn_dnorm_f16", gh.data_ptr(), yh.data_ptr(), nrm16.data_ptr(), gx16.data_ptr(), P, C, inv,
               1, s)
        check(gx16, gx32, f"gdn dnorm inv={inv}")
    # add2d with every storage combination, accumulate on and off
    for io in (1, 2, 3):
        for acc in (0, 1):
            base = _h(_rand((P, C), 5)).to(D)
            dst32 = base.clone()
            L.call("hyres_add2d", g.data_ptr(), C, dst32.data_ptr(), C, P, C, acc, s)
            src = gh if io & 1 else g
            dst = base.half() if io & 2 else base.clone()
            L.call("hyres_add2d_f16", src.data_ptr(), C, dst.data_ptr(), C, P, C, acc, io, s)
            if io & 2:
                check(dst, dst32, f"add2d io={io} acc={acc}")
            else:
                assert torch.equal(dst, dst32), (io, acc)
    acc16 = y.half()
    L.call("hyres_accumulate_f16", gh.data_ptr(), acc16.data_ptr(), P * C, s)
    check(acc16, y + g, "accumulate")
    # bias column sums over a fp16 gradient: the same sums as over its fp32 copy, bit for bit
    c32, c16 = torch.zeros(C, device=D), torch.zeros(C, device=D)
    wsc = torch.empty(int(L.load().hyres_colsum_workspace_bytes(P, C)), dtype=torch.uint8, device=D)
    L.call("hyres_colsum", g.data_ptr(), P, C, C, c32.data_ptr(), 0, wsc.data_ptr(), wsc.numel(), s)
    L.call("hyres_colsum_f16", gh.data_ptr(), P, C, C, c16.data_ptr(), 0, wsc.data_ptr(), wsc.numel(), s)
    torch.cuda.synchronize()
    assert torch.equal(c16, c32)
    # bilinear backward (general gather and the exact x1/2 down-sampling kernel), accumulate on
    for (Hi, Wi, Ho, Wo, sc) in ((H, W, 2 * H, 2 * W, 0.5), (H, W, H // 2, W // 2, 2.0)):
        gy = _h(_rand((B * Ho * Wo, C), 6)).to(D)
        base = _h(_rand((P, C), 7)).to(D)
        o32, o16, gy16 = base.clone(), base.half(), gy.half()
        L.call("hyres_bilinear_bwd", gy.data_ptr(), C, o32.data_ptr(), C, B, Hi, Wi, Ho, Wo, C, sc, sc, 1, s)
        L.call("hyres_bilinear_bwd_f16", gy16.data_ptr(), C, o16.data_ptr(), C, B, Hi, Wi, Ho, Wo, C, sc, sc, 1, s)
        check(o16, o32, f"bilinear bwd {Ho}x{Wo}")
    # SE / spatial attention backward with fp16 gy / gx
    Cr = 4
    w1 = _rand((Cr, C), 5, 0.2).to(D)
    w2 = _rand((C, Cr), 6, 0.2).to(D)
    pooled, hidden, sgate = (torch.empty(B, C, device=D), torch.empty(B, Cr, device=D), torch.empty(B, C, device=D))
    yse = torch.empty(P, C, device=D)
    wsb = int(L.load().hyres_se_workspace_bytes(B, H * W, C)) + B * C * 4
    ws = torch.empty(wsb, dtype=torch.uint8, device=D)
    L.call("hyres_se_fwd", y.data_ptr(), w1.data_ptr(), w2.data_ptr(), yse.data_ptr(), pooled.data_ptr(),
           hidden.data_ptr(), sgate.data_ptr(), B, H * W, C, Cr, ws.data_ptr(), ws.numel(), s)
    gws = [torch.zeros(Cr, C, device=D), torch.zeros(C, Cr, device=D), torch.zeros(Cr, C, device=D),
           torch.zeros(C, Cr, device=D)]
    L.call("hyres_se_bwd", y.data_ptr(), g.data_ptr(), w1.data_ptr(), w2.data_ptr(), pooled.data_ptr(),
           hidden.data_ptr(), sgate.data_ptr(), gx32.data_ptr(), gws[0].data_ptr(), gws[1].data_ptr(), B, H * W, C, Cr,
           ws.data_ptr(), ws.numel(), s)
    L.call("hyres_se_bwd_f16", yh.data_ptr(), gh.data_ptr(), w1.data_ptr(), w2.data_ptr(), pooled.data_ptr(),
           hidden.data_ptr(), sgate.data_ptr(), gx16.data_ptr(), gws[2].data_ptr(), gws[3].data_ptr(), B, H * W, C, Cr,
           ws.data_ptr(), ws.numel(), 1, s)
    check(gx16, gx32, "se gx")
    assert rel_err(gws[2].cpu(), gws[0].cpu()) <= 1e-6 and rel_err(gws[3].cpu(), gws[1].cpu()) <= 1e-6
    wsa = _rand((1, 2, 7, 7), 7, 0.1).to(D)
    pooled2 = torch.empty(P, 2, device=D)
    amax = torch.empty(P, dtype=torch.int32, device=D)
    attn = torch.empty(P, device=D)
    ysa = torch.empty(P, C, device=D)
    L.call("hyres_spatial_attn_fwd", y.data_ptr(), wsa.data_ptr(), pooled2.data_ptr(), amax.data_ptr(),
           attn.data_ptr(), ysa.data_ptr(), B, H, W, C, s)
    gw32, gw16 = torch.zeros(1, 2, 7, 7, device=D), torch.zeros(1, 2, 7, 7, device=D)
    wsb = int(L.load().hyres_spatial_attn_workspace_bytes(B, H, W))
    ws = torch.empty(wsb, dtype=torch.uint8, device=D)
    L.call("hyres_spatial_attn_bwd", y.data_ptr(), wsa.data_ptr(), pooled2.data_ptr(), amax.data_ptr(),
           attn.data_ptr(), g.data_ptr(), gx32.data_ptr(), gw32.data_ptr(), B, H, W, C, ws.data_ptr(), ws.numel(), s)
    L.call("hyres_spatial_attn_bwd_f16", yh.data_ptr(), wsa.data_ptr(), pooled2.data_ptr(), amax.data_ptr(),
           attn.data_ptr(), gh.data_ptr(), gx16.data_ptr(), gw16.data_ptr(), B, H, W, C, ws.data_ptr(), ws.numel(), 1,
           s)
    torch.cuda.synchronize()
    # the logit sums may contract differently (1 ulp): gx within one fp16 ulp of the rounded fp32 result
    assert (gx16.float() - gx32.half().float()).abs().max() <= 1e-3 * gx32.abs().max()
    assert rel_err(gw16.cpu(), gw32.cpu()) <= 1e-6


# ------------------------------------------------------------------------------------------ conv layers
LAYER_CASES = [
    # kind, B, Ci, Co, H, W, K, stride, pad, dil
    ("conv", 2, 64, 64, 32, 64, 3, 1, 1, 1),      # f16 halo weight gradient (Q = x fp16), 3x3 dgrad
    ("conv", 2, 64, 64, 20, 64, 3, 1, 2, 2),      # dilated 3x3 (MultiScaleRefine)
    ("conv", 4, 64, 128, 64, 64, 1, 1, 0, 1),     # 1x1: f16 ONE weight-gradient path
    ("conv", 2, 128, 128, 32, 32, 5, 2, 2, 1),    # 5x5 stride 2 (g_a), Q stride 2
    ("conv", 2, 64, 96, 12, 20, 3, 1, 1, 1),      # generic f16 weight gradient (rows not a multiple of 32)
    ("conv", 2, 64, 3, 16, 64, 3, 1, 1, 1),       # Co = 3: swapped thin weight gradient with a fp16 P
    ("deconv", 2, 128, 128, 16, 32, 5, 2, 2, 1),  # P = x fp16 (g_s)
    ("deconv", 2, 128, 3, 16, 16, 5, 2, 2, 1),    # thin weight gradient with a fp16 P (g_s's last deconv)
]


@pytest.mark.parametrize("wgrad_f16", [1, 0])
@pytest.mark.parametrize("case", LAYER_CASES)
def test_layer_with_fp16_input_matches_fp32_storage(case, wgrad_f16, monkeypatch):
    """One conv / deconv recorded on the tape under autocast inside an f16_region with its input stored fp16,
    against the same layer on an fp32 node holding the same values (AMP_F16_ACT off): weight, bias and
    input gradients bit-identical (no mask: act none); the fp16 output within fp16 rounding of the fp32 one.
    wgrad_f16 = 0 (HYRES_AMP_WGRAD_F16=0): the fp32 weight-gradient kernels on the converted operand."""
    from hyres_hip import ops as O
    kind, B, Ci, Co, H, W, K, s, p, d = case
    D = dev()
    x = _h(_rand((B, Ci, H, W), 11)).to(D)
    if kind == "conv":
        w = _rand((Co, Ci, K, K), 12, 1.0 / (Ci * K * K) ** 0.5).to(D)
    else:
        w = _rand((Ci, Co, K, K), 12, 1.0 / (Ci * K * K / 4) ** 0.5).to(D)
    b = _rand((Co,), 13, 0.1).to(D)
    monkeypatch.setattr(O, "AMP_WGRAD_F16", wgrad_f16)
    res = {}
    for f16_act in (True, False):
        monkeypatch.setattr(O, "AMP_F16_ACT", f16_act)
        wd, bd = torch.nn.Parameter(w.clone()), torch.nn.Parameter(b.clone())
        tape = O.Tape()
        xn = O.to_nhwc(x, rg=True)
        if f16_act:
            xn = O.Node(xn.v.half(), rg=True)
        with torch.autocast("cuda", dtype=torch.float16), O.f16_region():
            if kind == "conv":
                yn = O.conv2d(tape, xn, wd, bd, stride=s, pad=p, dil=d)
            else:
                yn = O.deconv2d(tape, xn, wd, bd)
        assert yn.half == (f16_act and Co > 4)
        gy = _h(_rand((yn.B, yn.C, yn.H, yn.W), 14)).to(D)  # fp16-representable: the fp16 gradient holds it exactly
        y = O.to_nchw(yn)
        yn.set_grad(O.nchw_grad_to_nhwc(gy))
        tape.backward()
        torch.cuda.synchronize()
        res[f16_act] = (y, O.to_nchw_grad(xn), wd.grad.clone(), bd.grad.clone())
    (y16, gx16, gw16, gb16), (y32, gx32, gw32, gb32) = res[True], res[False]
    print(case, "forward fp16-stored vs fp32:", rel_err(y16.cpu(), y32.cpu()),
          "vs fp32 rounded:", rel_err(y16.cpu(), y32.half().float().cpu()))
    assert rel_err(y16.cpu(), y32.cpu()) < 1e-3  # one fp16 rounding of the same fp32 value (+ summation order)
    # fp16 activation gradients (O.AMP_F16_GRAD): x's gradient is the fp32 layer's, rounded once to fp16
    assert torch.equal(gx16, gx32.half().float() if O.AMP_F16_GRAD else gx32)
    assert torch.equal(gw16, gw32)
    assert torch.equal(gb16, gb32)


def test_gdn_with_fp16_activations_matches_fp32_storage(monkeypatch):
    """GDN / IGDN in AMP training with fp16 x, y and saved norm: the norm gradient (gdn_dnorm_f16), the gamma
    weight gradient (square_q with a fp16 Q) and the input gradient (GDN-backward epilogue reading fp16 x and
    norm through HYRES_IO_AUX16) against the fp32-storage layer fed the fp16-rounded y and norm: 1e-5."""
    from hyres_hip import ops as O
    D = dev()
    B, C, H, W = 2, 128, 16, 32
    x = _h(_rand((B, C, H, W), 21)).to(D)
    beta = (torch.rand(C, generator=torch.Generator().manual_seed(22)) + 0.5).to(D)
    gamma = (0.1 * torch.eye(C) + 0.01 * torch.rand(C, C, generator=torch.Generator().manual_seed(23))).to(D)
    for inverse in (False, True):
        res = {}
        for f16_act in (True, False):
            monkeypatch.setattr(O, "AMP_F16_ACT", f16_act)
            bp, gp = torch.nn.Parameter(beta.clone()), torch.nn.Parameter(gamma.clone())
            tape = O.Tape()
            xn = O.to_nhwc(x, rg=True)
            if f16_act:
                xn = O.Node(xn.v.half(), rg=True)
            with torch.autocast("cuda", dtype=torch.float16), O.f16_region():
                yn = O.gdn(tape, xn, bp, gp, inverse)
            gy = _rand((B, C, H, W), 24).to(D)
            y = O.to_nchw(yn)
            yn.set_grad(O.nchw_grad_to_nhwc(gy))
            tape.backward()
            torch.cuda.synchronize()
            res[f16_act] = (y, O.to_nchw_grad(xn), bp.grad.clone(), gp.grad.clone())
        (y16, gx16, gb16, gg16), (y32, gx32, gb32, gg32) = res[True], res[False]
        assert rel_err(y16.cpu(), y32.cpu()) < 1e-3
        # the fp16 path's backward reads y and the norm rounded to fp16: bounded by that rounding
        for a, r in ((gx16, gx32), (gb16, gb32), (gg16, gg32)):
            assert rel_err(a.cpu(), r.cpu()) < 2e-3, (inverse, rel_err(a.cpu(), r.cpu()))


def test_residual_unit_chain_fp16_activations_vs_torch():
    """AttentionBlock's ResidualUnit (models/layers/attention.py:11-30): relu(x + 1x1(relu(3x3(relu(1x1(x)))))),
    x fp16, under autocast inside an f16_region with fp16 saved activations. Torch (float64) with the same
    rounding points: fp16 operands for every GEMM (forward, input and weight gradients), each stored
    activation rounded to fp16, gradients fp32. The input-gradient convs apply the ReLU masks from the fp16
    activations (HYRES_IO_AUX16). 1e-4 relative (summation order moves a few fp16 roundings by one ulp)."""
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    D = dev()
    B, N, H, W = 2, 128, 32, 64
    x = _h(_rand((B, N, H, W), 31))
    ws = [_rand((N // 2, N, 1, 1), 32, N ** -0.5), _rand((N // 2, N // 2, 3, 3), 33, (N / 2 * 9) ** -0.5),
          _rand((N, N // 2, 1, 1), 34, (N / 2) ** -0.5)]
    bs = [_rand((c,), 35 + i, 0.1) for i, c in enumerate((N // 2, N // 2, N))]
    gy = _rand((B, N, H, W), 38)

    # torch reference (float64), fp16 rounding where the HIP path rounds
    def r16(t):
        return t.half().double()
    xd = x.double().requires_grad_()
    wd = [w.double().requires_grad_() for w in ws]
    bd = [b.double().requires_grad_() for b in bs]

    g16 = O.AMP_F16_GRAD

    class Round(torch.autograd.Function):
        """fp16 storage of a forward output; its gradient is stored fp16 too (O.AMP_F16_GRAD: autocast's fp16
        activation gradients), i.e. rounded where the HIP path stores it."""
        @staticmethod
        def forward(ctx, t):
            return r16(t)

        @staticmethod
        def backward(ctx, g):
            return r16(g) if g16 else g

    class Conv16(torch.autograd.Function):
        """f16-MFMA conv: fp16 operands in every GEMM (forward: x, w; backward: the incoming gradient and w /
        x), fp32-or-better accumulation, the bias gradient from the unrounded gradient."""
        @staticmethod
        def forward(ctx, t, w, b, pad):
            th, wh = r16(t), r16(w)
            ctx.save_for_backward(th, wh)
            ctx.pad = pad
            return F.conv2d(th, wh, b, padding=pad)

        @staticmethod
        def backward(ctx, g):
            th, wh = ctx.saved_tensors
            gh = r16(g)
            gx = torch.nn.grad.conv2d_input(th.shape, wh, gh, padding=ctx.pad)
            gw = torch.nn.grad.conv2d_weight(th, wh.shape, gh, padding=ctx.pad)
            return gx, gw, g.sum((0, 2, 3)), None

    def conv(t, i, pad):
        return Conv16.apply(t, wd[i], bd[i], pad)

    t1 = Round.apply(F.relu(conv(xd, 0, 0)))
    t2 = Round.apply(F.relu(conv(t1, 1, 1)))
    y = Round.apply(F.relu(conv(t2, 2, 0) + xd))
    y.backward(gy.double())

    Dv = D
    wp = [torch.nn.Parameter(w.to(Dv)) for w in ws]
    bp = [torch.nn.Parameter(b.to(Dv)) for b in bs]
    tape = O.Tape()
    xn = O.to_nhwc(x.to(Dv), rg=True)
    xn = O.Node(xn.v.half(), rg=True)
    with torch.autocast("cuda", dtype=torch.float16), O.f16_region():
        a1 = O.conv2d(tape, xn, wp[0], bp[0], act=L.ACT_RELU)
        a2 = O.conv2d(tape, a1, wp[1], bp[1], pad=1, act=L.ACT_RELU)
        yn = O.conv2d(tape, a2, wp[2], bp[2], act=L.ACT_RELU, res=xn)
    assert a1.half and a2.half and yn.half
    yh = O.to_nchw(yn)
    yn.set_grad(O.nchw_grad_to_nhwc(gy.to(Dv)))
    tape.backward()
    torch.cuda.synchronize()
    print("chain a1", rel_err(O.to_nchw(a1).cpu(), t1.detach().float()), "a2",
          rel_err(O.to_nchw(a2).cpu(), t2.detach().float()), "y", rel_err(yh.cpu(), y.detach().float()))
    assert rel_err(yh.cpu(), y.detach().float()) < 2e-3  # max-norm: one fp16 ulp of the largest |y|
    # x's gradient (conv path + residual path, summed in fp32) is stored fp16 with fp16 gradients: one rounding
    assert rel_err(O.to_nchw_grad(xn).cpu(), xd.grad.float()) < (1e-3 if g16 else 1e-4)
    for i in range(3):
        assert rel_err(wp[i].grad.cpu(), wd[i].grad.float()) < 1e-4, i
        assert rel_err(bp[i].grad.cpu(), bd[i].grad.float()) < 1e-4, i


@pytest.mark.parametrize("acc", [0, 1])
def test_stream_hf_sa_bwd_epilogue(acc):
    """conv1x1_stream_hf_kernel's SA_BWD build (round 6): MultiScaleRefine's fusion input-gradient 64 -> 192 under AMP
    with SpatialAttention's mean / max backward in the epilogue — y = fp16((W^T gs + d mean / C) + [c == argmax] d max
    (+ old y)), fp16 gs and W on the f16 MFMA. vs float64 torch on the same fp16 operands: one fp16 rounding (1e-3
    max-norm); the launcher's own label names the kernel."""
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    D = dev()
    B, H, W = 2, 96, 96
    P = B * H * W
    gs = _h(_rand((P, 64), 61)).half().to(D)
    w = _rand((192, 64), 62, 0.125).to(D)
    gm = _rand((P, 2), 63).to(D)
    am = torch.randint(0, 192, (P,), generator=torch.Generator().manual_seed(64), dtype=torch.int32).to(D)
    old = _h(_rand((P, 192), 65)).half().to(D)
    y = old.clone() if acc else torch.empty(P, 192, device=D, dtype=torch.float16)
    g = O._geom("hyres_geom_conv2d", B, H, W, 64, 64, 192, 192, 1, 1, 1, 0, 1)
    e = L.Epilogue()
    e.kind = L.EPI_SA_BWD
    e.aux0, e.ld0 = gm.data_ptr(), 2
    e.aux2 = am.data_ptr()
    e.f16_operands = 1
    e.io_f16 = L.IO_X16 | L.IO_Y16
    e.accumulate = acc
    assert O.conv_variant(g, e, False) == f"conv1x1_stream_hf_kernel<6, 4, {8 | 4 * acc}>"
    O._launch_conv(g, gs.data_ptr(), w, 64, y.data_ptr(), e)
    torch.cuda.synchronize()
    gmd = gm.double().cpu()
    ref = gs.double().cpu() @ w.half().double().cpu().T + gmd[:, :1]
    ref += torch.nn.functional.one_hot(am.long().cpu(), 192).double() * gmd[:, 1:]
    if acc:
        ref += old.double().cpu()
    assert rel_err(y.float().cpu(), ref) < 1e-3


def _amp_head(fold, m, multi, gy, D):
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    from hyres_hip import refine_ops as R
    for p in m.parameters():
        p.grad = None
    tape = O.Tape()
    xn = O.Node(O.to_nhwc(multi.to(D), rg=True).v.half(), rg=True)
    with torch.autocast("cuda", dtype=torch.float16), O.f16_region():
        assert R.sa_fold_amp_ok(tape, xn, 64)
        if fold:
            hn = R.sa_fold_fusion(tape, xn, m.spatial_att.conv.weight, m.fusion[0].weight, m.fusion[0].bias,
                                  m.fusion[1].weight)
        else:
            hn = m.fusion[0].hip(tape, m.spatial_att.hip_mul(tape, xn), act=L.ACT_PRELU, slope=m.fusion[1].weight)
        assert hn.half
        yn = m.fusion[2].hip(tape, hn)
    yn.set_grad(O.nchw_grad_to_nhwc(gy.to(D)))
    tape.backward()
    torch.cuda.synchronize()
    assert xn.grad().dtype == torch.float16
    out = {"y": O.to_nchw(yn).float().cpu(), "dmulti": O.to_nchw_grad(xn).float().cpu()}
    for k, p in m.named_parameters():
        if k.startswith(("fusion", "spatial_att")):
            out[k] = p.grad.cpu()
    return out


def test_refine_fusion_head_sa_fold_amp():
    """MultiScaleRefine's head (enhancement.py:105-109) in AMP training with fp16 activations and gradients: the
    SpatialAttention multiply folded into the fusion 1x1 (refine_ops.sa_fold_fusion's round-6 AMP build: ROWSCALE
    forward on fp16 operands, hyres_sa_fold_bwd_f16, the SA_BWD epilogue on conv1x1_stream_hf_kernel) and unfused
    (spatial_attention_mul + Sequential), each vs float64 torch without fp16 rounding: output, d multi and every
    parameter gradient within the AMP rounding (2e-2 max-norm; the slope, one cancelled sum, 5e-2; d multi 6e-2: the
    unfused chain measures 4.8e-2 on it here, the fold 4.7e-2 — fp16 gradients through the 7x7 map), and the fold
    no less accurate than the unfused chain on any of them (1.5x + 1e-3). One channel per pixel holds the unique
    maximum (1.0): fp16 ties at the max would move the max-pool's gradient between channels in either path."""
    import models.layers.enhancement as EH
    D = dev()
    B, C, H, W = 2, 192, 96, 96
    torch.manual_seed(11)
    m = EH.MultiScaleRefine(3, 64)
    multi = _h(_rand((B, C, H, W), 41, 0.9))
    top = torch.randint(0, C, (B, 1, H, W), generator=torch.Generator().manual_seed(43))
    multi.scatter_(1, top, 1.0)
    gy = _rand((B, 3, H, W), 42)
    sd = {k: v.detach().double().clone().requires_grad_(True) for k, v in m.state_dict().items()
          if k.startswith(("fusion", "spatial_att"))}
    sd["fusion.0.bias"].data.add_(0.05)
    xr = multi.double().requires_grad_(True)
    a = torch.sigmoid(F.conv2d(torch.cat([xr.mean(1, keepdim=True), xr.max(1, keepdim=True)[0]], 1),
                               sd["spatial_att.conv.weight"], None, padding=3))
    h = F.prelu(F.conv2d(xr * a, sd["fusion.0.weight"], sd["fusion.0.bias"]), sd["fusion.1.weight"])
    yr = F.conv2d(h, sd["fusion.2.weight"], sd["fusion.2.bias"], padding=1)
    yr.backward(gy.double())
    ref = {"y": yr.detach(), "dmulti": xr.grad}
    ref.update({k: v.grad for k, v in sd.items()})
    m = m.to(D)
    with torch.no_grad():
        for k, v in m.named_parameters():
            if k in sd:
                v.copy_(sd[k].detach().float())
    errs = {}
    for fold in (True, False):
        got = _amp_head(fold, m, multi, gy, D)
        errs[fold] = {k: rel_err(got[k], ref[k]) for k in ref}
        print("fold" if fold else "unfused", {k: f"{v:.1e}" for k, v in errs[fold].items()})
    for fold in (True, False):
        bad = {k: v for k, v in errs[fold].items() if v > {"fusion.1.weight": 5e-2, "dmulti": 6e-2}.get(k, 2e-2)}
        assert not bad, (fold, errs[fold])
    worse = {k: (errs[True][k], errs[False][k]) for k in ref if errs[True][k] > 1.5 * errs[False][k] + 1e-3}
    assert not worse, worse


@pytest.mark.parametrize("g16", [1, 0])
def test_sa_fold_bwd_f16_matches_fp32_kernel(g16):
    """hyres_sa_fold_bwd_f16 (fp16 pre-activation; fp16 or fp32 gy / gs) vs hyres_sa_fold_bwd on the same fp16-
    representable values: gs within one fp16 rounding of the fp32 kernel's (1 ulp), glogit / d bias / d slope to fp32
    summation order (1e-5). A ragged pixel count, both PReLU sides, accumulation into existing d bias / d slope."""
    from hyres_hip import _lib as L
    D = dev()
    P, C = 2 * 37 * 41, 64
    pre = _h(_rand((P, C), 71)).to(D)
    gy = _h(_rand((P, C), 72)).to(D)
    attn = torch.rand(P, generator=torch.Generator().manual_seed(73)).to(D)
    bias = _rand((C,), 74, 0.1).to(D)
    slope = torch.full((1,), 0.25, device=D)
    ws = torch.empty(L.load().hyres_sa_fold_workspace_bytes(P, C) // 4 + 1, device=D)
    gdt = torch.float16 if g16 else torch.float32
    pre16, gyc = pre.half(), gy.to(gdt)  # held: a temporary's pointer would be recycled before the call
    outs = {}
    for name, f16 in (("f32", False), ("f16", True)):
        gs = torch.empty(P, C, device=D, dtype=gdt if f16 else torch.float32)
        gl = torch.empty(P, device=D)
        db = torch.full((C,), 0.5, device=D)
        ds = torch.full((1,), 0.5, device=D)
        if f16:
            L.call("hyres_sa_fold_bwd_f16", pre16.data_ptr(), C, gyc.data_ptr(), C, attn.data_ptr(),
                   bias.data_ptr(), slope.data_ptr(), gs.data_ptr(), gl.data_ptr(), db.data_ptr(), ds.data_ptr(), P, C,
                   ws.data_ptr(), ws.numel() * 4, g16, L.stream())
        else:
            L.call("hyres_sa_fold_bwd", pre.data_ptr(), C, gy.data_ptr(), C, attn.data_ptr(), bias.data_ptr(),
                   slope.data_ptr(), gs.data_ptr(), gl.data_ptr(), db.data_ptr(), ds.data_ptr(), P, C, ws.data_ptr(),
                   ws.numel() * 4, L.stream())
        torch.cuda.synchronize()
        outs[name] = (gs.clone(), gl.clone(), db.clone(), ds.clone())
    (gs32, gl32, db32, ds32), (gs16, gl16, db16, ds16) = outs["f32"], outs["f16"]
    assert bool((pre < 0).any()) and bool((pre > 0).any())
    if g16:
        a = gs16.view(-1) + 0
        b = gs32.half().view(-1) + 0
        assert int((a.view(torch.int16).int() - b.view(torch.int16).int()).abs().max()) <= 1
    else:
        assert rel_err(gs16.cpu(), gs32.cpu()) < 1e-6
    assert rel_err(gl16.cpu(), gl32.cpu()) < 1e-5
    assert rel_err(db16.cpu(), db32.cpu()) < 1e-5 and rel_err(ds16.cpu(), ds32.cpu()) < 1e-5


@pytest.mark.parametrize("act", ["prelu", "none"])
def test_stream_hf_rowscale_matches_tiles(act):
    """conv1x1_stream_hf_kernel's ROWSCALE build (round 6): the AMP fusion forward 192 -> 64 with SpatialAttention
    folded — y = act(attn[p] * (W x)[p] + b) and the fp16 pre-activation copy — against the tiled f16 kernel
    (hyres_conv_tuning key 17 = 0) on the same call: the same fp16 products, at most 1 fp16 ulp apart (the epilogue's
    multiply-add may contract differently); and vs float64 on the fp16 operands at 1e-3 (one fp16 rounding)."""
    import ctypes
    from hyres_hip import _lib as L
    from hyres_hip import ops as O
    D = dev()
    B, H, W = 2, 96, 96
    P, Ci, Co = B * H * W, 192, 64
    x = _h(_rand((P, Ci), 81)).half().to(D)
    w = _rand((Co, Ci), 82, Ci ** -0.5).to(D)
    b = _rand((Co,), 83, 0.1).to(D)
    sc = torch.rand(P, generator=torch.Generator().manual_seed(84)).to(D)
    slope = torch.full((1,), 0.25, device=D)
    g = O._geom("hyres_geom_conv2d", B, H, W, Ci, Ci, Co, Co, 1, 1, 1, 0, 1)
    res = {}
    for key in (1, 0):
        y = torch.empty(P, Co, device=D, dtype=torch.float16)
        pre = torch.empty(P, Co, device=D, dtype=torch.float16)
        e = L.Epilogue()
        e.kind = L.EPI_ROWSCALE
        e.act = L.ACT_PRELU if act == "prelu" else L.ACT_NONE
        e.bias = b.data_ptr()
        e.slope = slope.data_ptr()
        e.aux1, e.ld1 = sc.data_ptr(), 1
        e.out2, e.ldo2 = pre.data_ptr(), Co
        e.f16_operands = 1
        e.io_f16 = L.IO_X16 | L.IO_Y16
        old = ctypes.c_int(0)
        L.call("hyres_conv_tuning", 17, key, ctypes.byref(old))
        try:
            name = O.conv_variant(g, e, False)
            O._launch_conv(g, x.data_ptr(), w, Ci, y.data_ptr(), e)
            torch.cuda.synchronize()
        finally:
            L.call("hyres_conv_tuning", 17, old.value, None)
        res[key] = (name, y, pre)
    assert res[1][0] == "conv1x1_stream_hf_kernel<2, 12, 16>", res[1][0]
    assert not res[0][0].startswith("conv1x1_stream_hf"), res[0][0]
    for i in (1, 2):
        u = res[1][i].view(-1) + 0
        v = res[0][i].view(-1) + 0
        assert int((u.view(torch.int16).int() - v.view(torch.int16).int()).abs().max()) <= 1
    r = (x.double() @ w.half().double().t()) * sc.double()[:, None] + b.double()
    ra = torch.where(r >= 0, r, 0.25 * r) if act == "prelu" else r
    assert rel_err(res[1][2].double().cpu(), r.cpu()) < 1e-3 and rel_err(res[1][1].double().cpu(), ra.cpu()) < 1e-3
