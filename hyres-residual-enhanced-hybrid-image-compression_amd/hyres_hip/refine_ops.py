"""MultiScaleRefine building blocks and the ResidualJPEGCompression glue on HIP.

Reference anchors: models/layers/enhancement.py:7-112 (SpatialAttention, SEBlock, MultiScaleRefine),
models/hyres.py:48,62,65-67 (residual, x_hat_initial, refine + clamp)."""
from __future__ import annotations

from typing import Optional

import ctypes

import torch

from . import _lib as L
from . import ops as O
from .ops import Node, Tape, _empty, accumulate, param_grad, _ws


def bilinear(tape: Optional[Tape], x: Node, Ho: int, Wo: int, scale_h: float, scale_w: float,
             out: Optional[Node] = None) -> Node:
    """F.interpolate(mode='bilinear', align_corners=False).  ``scale_*`` is torch's source-index scale:
    1/scale_factor when a scale_factor is given (enhancement.py:96,101), in/out for ``size=``
    (enhancement.py:98,103)."""
    y = out if out is not None else Node.new(x.B, Ho, Wo, x.C, x.device, dtype=x.v.dtype)
    if x.half:  # fp16 activations (autocast; the backward below only reads gradients)
        assert y.half
        L.call("hyres_bilinear_fwd_f16", x.ptr(), x.ld, y.ptr(), y.ld, x.B, x.H, x.W, Ho, Wo, x.C, float(scale_h),
               float(scale_w), L.stream())
    else:
        L.call("hyres_bilinear_fwd", x.ptr(), x.ld, y.ptr(), y.ld, x.B, x.H, x.W, Ho, Wo, x.C, float(scale_h),
               float(scale_w), 0, L.stream())
    if tape is None:
        return y

    def bwd():
        g = y.grad()
        if g is None or not x.rg:
            return
        tgt, acc = x.grad_target()
        assert g.dtype == tgt.dtype
        if (O.FOLD_PRELU and acc == 0 and x.prelu is not None and x.parent is None and Ho > x.H and Wo > x.W
                and x.C % 4 == 0 and x.prelu[0].is_contiguous() and not O.Trace.traced(x)):
            # round 6: MultiScaleRefine's scales 2 / 3 end in conv + PReLU, whose output only this up-sample reads
            # (enhancement.py:89-103): the PReLU backward rides on the up-sample's backward (its one gradient writer)
            pre, slope = x.prelu
            dslope = param_grad(slope) if slope.requires_grad else _empty((1,), x.device)
            ws = _ws(L.load().hyres_bilinear_bwd_prelu_workspace_bytes(x.B, x.H, x.W, x.C), x.device, slot=1)
            io = (1 if g.dtype == torch.float16 else 0) | (2 if pre.dtype == torch.float16 else 0)
            L.call("hyres_bilinear_bwd_prelu", g.data_ptr(), y.grad_ld(), tgt.data_ptr(), x.grad_ld(), x.B, x.H, x.W,
                   Ho, Wo, x.C, float(scale_h), float(scale_w), pre.data_ptr(), x.C, slope.data_ptr(),
                   dslope.data_ptr(), ws.data_ptr(), ws.numel(), io, L.stream())
            x.pmasked = True
            return
        fn = "hyres_bilinear_bwd_f16" if g.dtype == torch.float16 else "hyres_bilinear_bwd"  # AMP fp16 gradients
        L.call(fn, g.data_ptr(), y.grad_ld(), tgt.data_ptr(), x.grad_ld(), x.B, x.H, x.W, Ho, Wo,
               x.C, float(scale_h), float(scale_w), acc, L.stream())

    tape.push(bwd)
    return y


def se_block(tape: Optional[Tape], x: Node, w1: torch.Tensor, w2: torch.Tensor) -> Node:
    """SEBlock (enhancement.py:25-40): y = x * sigmoid(W2 relu(W1 avgpool(x)))."""
    assert x.contiguous
    B, HW, C = x.B, x.H * x.W, x.C
    Cr = w1.shape[0]
    dev = x.device
    y = Node.new(x.B, x.H, x.W, C, dev, dtype=x.v.dtype)
    pooled = _empty((B, C), dev)
    hidden = _empty((B, Cr), dev)
    sgate = _empty((B, C), dev)
    wsb = L.load().hyres_se_workspace_bytes(B, HW, C)
    ws = _ws(wsb + B * C * 4, dev, slot=1)
    fn = "hyres_se_fwd_f16" if x.half else "hyres_se_fwd"
    L.call(fn, x.ptr(), w1.data_ptr(), w2.data_ptr(), y.ptr(), pooled.data_ptr(), hidden.data_ptr(),
           sgate.data_ptr(), B, HW, C, Cr, ws.data_ptr(), ws.numel(), L.stream())
    if tape is None:
        return y

    def bwd():
        g = y.grad()
        if g is None:
            return
        assert y.grad_ld() == C
        gw1 = param_grad(w1)
        gw2 = param_grad(w2)
        tgt, acc = x.grad_target()
        assert g.dtype == tgt.dtype
        gx = tgt if acc == 0 else _empty((x.B, x.H, x.W, C), dev, tgt.dtype)
        if (O.FOLD_PRELU and acc == 0 and x.prelu is not None and x.parent is None and not O.Trace.traced(x)
                and x.prelu[0].dtype == x.v.dtype and x.prelu[0].is_contiguous() and C % 4 == 0):
            # the producing PReLU's backward folded in (conv_in's act_in, enhancement.py:107-110): the SE block is
            # the only reader of PReLU(conv_in(x)), so its input-gradient is the PReLU output's whole gradient
            pre, slope = x.prelu
            dslope = param_grad(slope) if slope.requires_grad else _empty((1,), dev)
            ws2 = _ws(wsb + B * C * 4 + 2048 * 4, dev, slot=1)
            if x.half:  # AMP (round 6): fp16 pre-activation, fp16 or fp32 gradients
                L.call("hyres_se_bwd_prelu_f16", x.ptr(), g.data_ptr(), w1.data_ptr(), w2.data_ptr(), pooled.data_ptr(),
                       hidden.data_ptr(), sgate.data_ptr(), gx.data_ptr(), gw1.data_ptr(), gw2.data_ptr(), B, HW, C, Cr,
                       pre.data_ptr(), slope.data_ptr(), dslope.data_ptr(), ws2.data_ptr(), ws2.numel(),
                       int(g.dtype == torch.float16), L.stream())
            else:
                assert g.dtype == torch.float32
                L.call("hyres_se_bwd_prelu", x.ptr(), g.data_ptr(), w1.data_ptr(), w2.data_ptr(), pooled.data_ptr(),
                       hidden.data_ptr(), sgate.data_ptr(), gx.data_ptr(), gw1.data_ptr(), gw2.data_ptr(), B, HW, C,
                       Cr, pre.data_ptr(), slope.data_ptr(), dslope.data_ptr(), ws2.data_ptr(), ws2.numel(),
                       L.stream())
            x.pmasked = True
            return
        ws2 = _ws(wsb + B * C * 4, dev, slot=1)
        if x.half:
            L.call("hyres_se_bwd_f16", x.ptr(), g.data_ptr(), w1.data_ptr(), w2.data_ptr(), pooled.data_ptr(),
                   hidden.data_ptr(), sgate.data_ptr(), gx.data_ptr(), gw1.data_ptr(), gw2.data_ptr(), B, HW, C, Cr,
                   ws2.data_ptr(), ws2.numel(), int(g.dtype == torch.float16), L.stream())
        else:
            L.call("hyres_se_bwd", x.ptr(), g.data_ptr(), w1.data_ptr(), w2.data_ptr(), pooled.data_ptr(),
                   hidden.data_ptr(), sgate.data_ptr(), gx.data_ptr(), gw1.data_ptr(), gw2.data_ptr(), B, HW, C, Cr,
                   ws2.data_ptr(), ws2.numel(), L.stream())
        if acc:
            accumulate(gx, tgt)

    tape.push(bwd)
    return y


def spatial_attention_map(x: Node, w: torch.Tensor, keep: bool = False):
    """SpatialAttention(x) alone (enhancement.py:7-21): the [B, H, W] sigmoid map, fp32 — its multiply is folded
    into the next 1x1 conv's epilogue (ops.conv2d ``rowscale``; training: ``sa_fold_fusion``). ``keep``: also return
    the pooled [B, H, W, 2] map and the channel argmax the backward needs."""
    assert x.contiguous
    B, H, W, C = x.B, x.H, x.W, x.C
    dev = x.device
    pooled2 = _empty((B, H, W, 2), dev)
    argmax = torch.empty((B, H, W), dtype=torch.int32, device=dev)
    attn = _empty((B, H, W), dev)
    fn = "hyres_spatial_attn_fwd_f16" if x.half else "hyres_spatial_attn_fwd"
    L.call(fn, x.ptr(), w.data_ptr(), pooled2.data_ptr(), argmax.data_ptr(), attn.data_ptr(), None, B, H, W, C,
           L.stream())
    return (attn, pooled2, argmax) if keep else attn


def sa_fold_fusion(tape: Optional[Tape], multi: Node, w_sa: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor,
                   slope: torch.Tensor) -> Node:
    """PReLU(fusion[0](multi * SpatialAttention(multi))) of MultiScaleRefine (enhancement.py:105-109) in training,
    with the attention multiply never materialised (fp32 activations).

    Forward: the attention map, then ONE 1x1 conv whose epilogue forms attn[p] * (W multi)[p] + b (HYRES_EPI_ROWSCALE)
    and the PReLU, saving the pre-activation. Backward (hyres_sa_fold_bwd): gs = attn * PReLU'(gy) and the attention
    logit's gradient from the 64-channel pre-activation (no 192-channel pass); d W_sa and the pooled maps' gradients on
    the 2-channel map (hyres_spatial_attn_bwd_map); d W = gs x multi (weight gradient on the side stream, bias from the
    fold's own column sums); d multi = W^T gs with SpatialAttention's mean / max backward added in the input-gradient's
    epilogue (HYRES_EPI_SA_BWD). Replaces sa_mul, sa_bwd_logit, sa_bwd_x and the PReLU backward of the unfused chain
    (refine's 192-channel concat read and written three more times per step).

    Round 6, AMP training (``sa_fold_amp_ok``): fp16 ``multi``, output, pre-activation and gradients, fp16 operands on
    the f16 MFMA; backward hyres_sa_fold_bwd_f16, the input-gradient on conv1x1_stream_hf_kernel's SA_BWD build."""
    assert multi.contiguous and (not multi.half or sa_fold_amp_ok(tape, multi, weight.shape[0]))
    Co, Ci_w, KH, KW = weight.shape
    assert KH == 1 and KW == 1 and Ci_w == multi.C and slope.numel() == 1
    B, H, W, Ci = multi.B, multi.H, multi.W, multi.C
    dev = multi.device
    attn, pooled2, argmax = spatial_attention_map(multi, w_sa, keep=True)
    f16 = int(O.f16_convs())
    ydt = torch.float16 if Co > 4 and O.act_f16(tape, H, W) else torch.float32
    y = Node.new(B, H, W, Co, dev, dtype=ydt)
    pre = _empty((B, H, W, Co), dev, ydt)  # stored by the epilogue in y's dtype
    g = O._geom("hyres_geom_conv2d", B, H, W, Ci, multi.ld, Co, y.ld, 1, 1, 1, 0, 1)
    e = L.Epilogue()
    e.kind = L.EPI_ROWSCALE
    e.act = L.ACT_PRELU
    e.bias = bias.data_ptr()
    e.slope = slope.data_ptr()
    e.aux1, e.ld1 = attn.data_ptr(), 1
    e.out2, e.ldo2 = pre.data_ptr(), Co
    e.io_f16 = O._io_flags(multi, y, tape)
    e.f16_operands = f16
    O._launch_conv(g, multi.ptr(), weight, Ci_w, y.ptr(), e)
    O.Trace.act(y, L.ACT_PRELU, pre)
    if tape is None:
        return y

    def bwd():
        gy = y.grad()
        if gy is None:
            return
        assert gy.dtype == torch.float32 or pre.dtype == torch.float16
        P = y.P
        gs = _empty((B, H, W, Co), dev, gy.dtype)
        glogit = _empty((B, H, W), dev)
        ws = _ws(L.load().hyres_sa_fold_workspace_bytes(P, Co), dev, slot=1)
        dbias = param_grad(bias) if bias.requires_grad else _empty((Co,), dev)
        dslope = param_grad(slope) if slope.requires_grad else _empty((1,), dev)
        if pre.dtype == torch.float16:
            L.call("hyres_sa_fold_bwd_f16", pre.data_ptr(), Co, gy.data_ptr(), y.grad_ld(), attn.data_ptr(),
                   bias.data_ptr(), slope.data_ptr(), gs.data_ptr(), glogit.data_ptr(), dbias.data_ptr(),
                   dslope.data_ptr(), P, Co, ws.data_ptr(), ws.numel(), int(gy.dtype == torch.float16), L.stream())
        else:
            L.call("hyres_sa_fold_bwd", pre.data_ptr(), Co, gy.data_ptr(), y.grad_ld(), attn.data_ptr(),
                   bias.data_ptr(), slope.data_ptr(), gs.data_ptr(), glogit.data_ptr(), dbias.data_ptr(),
                   dslope.data_ptr(), P, Co, ws.data_ptr(), ws.numel(), L.stream())
        gp2 = _empty((B, H, W, 2), dev)
        gw_sa = param_grad(w_sa) if w_sa.requires_grad else _empty(w_sa.shape, dev)
        ws2 = _ws(L.load().hyres_spatial_attn_workspace_bytes(B, H, W), dev, slot=1)
        L.call("hyres_spatial_attn_bwd_map", glogit.data_ptr(), pooled2.data_ptr(), w_sa.data_ptr(), gp2.data_ptr(),
               gw_sa.data_ptr(), B, H, W, Ci, ws2.data_ptr(), ws2.numel(), L.stream())
        if weight.requires_grad:
            d = L.WgradDesc()
            L.call("hyres_wgrad_desc_conv2d", ctypes.byref(d), B, H, W, Ci, multi.ld, Co, Co, 1, 1, 1, 0, 1)
            d.sm = Ci_w
            d.accumulate = 1
            d.f16_operands = f16 * O.AMP_WGRAD_F16
            d.io_f16 = (1 if gs.dtype == torch.float16 else 0) | (2 if multi.half else 0)
            O._wgrad(d, gs.data_ptr(), multi.ptr(), param_grad(weight), dev, None, keep=(gs, multi.v), side=True)
        if multi.rg:
            ed = L.Epilogue()
            ed.kind = L.EPI_SA_BWD
            ed.aux0, ed.ld0 = gp2.data_ptr(), 2
            ed.aux2 = argmax.data_ptr()
            tgt, acc = multi.grad_target()
            gd = O._geom("hyres_geom_conv2d_dgrad", B, H, W, Ci, multi.grad_ld(), Co, Co, 1, 1, 1, 0, 1)
            w2d = O._prepped(weight, gd, L.WPREP_CONV_DGRAD, Ci_w, Co, 1, 1, 0)
            ed.accumulate = acc
            ed.f16_operands = f16
            ed.io_f16 = O._dgrad_io(gs, multi)
            sl = _prelu_slice0(multi, tgt.dtype) if acc == 0 else None
            if sl is not None:
                # round 6: multi[..., 0:64] is scale 1's PReLU output and this conv its one gradient writer: its
                # PReLU backward rides on the epilogue (HYRES_ACT_PRELU_MASK on the streaming SA_BWD kernels)
                pre1, slope1 = sl.prelu
                dslope1 = param_grad(slope1) if slope1.requires_grad else _empty((1,), dev)
                part = _empty((L.PRELU_PARTIALS,), dev)
                ed.act = L.ACT_PRELU_MASK
                ed.aux1, ed.ld1 = pre1.data_ptr(), sl.C
                ed.slope = slope1.data_ptr()
                ed.res = dslope1.data_ptr()
                ed.out2, ed.ldo2 = part.data_ptr(), L.PRELU_PARTIALS
                if ", 40" not in O.conv_variant(gd, ed, False):  # the streaming kernels' PReLU-mask form only
                    ed.act, ed.aux1, ed.ld1, ed.slope, ed.res, ed.out2, ed.ldo2 = L.ACT_NONE, None, 0, None, None, None, 0
                    sl = None
            O._launch_conv(gd, gs.data_ptr(), w2d, gd.ntaps * Co, tgt.data_ptr(), ed)
            if sl is not None:
                sl.pmasked = True

    tape.push(bwd)
    return y


def _prelu_slice0(multi: Node, gdt: torch.dtype) -> Optional[Node]:
    """The 64-channel slice at channel 0 of ``multi`` written by a conv with a fused PReLU (MultiScaleRefine's
    scale 1), when its PReLU backward may be folded into multi's gradient writer: folds on, not a trace point, the
    pre-activation contiguous and in the gradient's dtype (the SA_BWD kernels read it beside Y)."""
    if not O.FOLD_PRELU:
        return None
    for n in multi.prelu_slices or []:
        if (n.c0 == 0 and n.C == 64 and n.prelu is not None and not O.Trace.traced(n)
                and n.prelu[0].is_contiguous() and n.prelu[0].dtype == gdt):
            return n
    return None


def sa_fold_amp_ok(tape: Optional[Tape], multi: Node, Co: int) -> bool:
    """sa_fold_fusion under AMP training: fp16 ``multi`` with fp16 gradients, an fp16 fusion output, and the fusion's
    input-gradient (Co -> multi.C with HYRES_EPI_SA_BWD) routed to conv1x1_stream_hf_kernel — the one kernel with an
    fp16-Y SA_BWD epilogue (checked through the launcher's own choice, ops.conv_variant)."""
    if tape is None or not multi.half or not multi.ghalf or not multi.contiguous or not O.f16_convs():
        return False
    if not (Co > 4 and O.act_f16(tape, multi.H, multi.W)) or not O.AMP_F16_GRAD:
        return False
    gd = O._geom("hyres_geom_conv2d_dgrad", multi.B, multi.H, multi.W, multi.C, multi.C, Co, Co, 1, 1, 1, 0, 1)
    ed = L.Epilogue()
    ed.kind = L.EPI_SA_BWD
    ed.ld0 = 2
    ed.f16_operands = 1
    ed.io_f16 = L.IO_X16 | L.IO_Y16
    return O.conv_variant(gd, ed, False).startswith("conv1x1_stream_hf_kernel")


def spatial_attention_mul(tape: Optional[Tape], x: Node, w: torch.Tensor) -> Node:
    """multi * SpatialAttention(multi) (enhancement.py:7-21 and :105-106), fused."""
    assert x.contiguous
    B, H, W, C = x.B, x.H, x.W, x.C
    dev = x.device
    pooled2 = _empty((B, H, W, 2), dev)
    argmax = torch.empty((B, H, W), dtype=torch.int32, device=dev)
    attn = _empty((B, H, W), dev)
    y = Node.new(B, H, W, C, dev, dtype=x.v.dtype)
    fn = "hyres_spatial_attn_fwd_f16" if x.half else "hyres_spatial_attn_fwd"
    L.call(fn, x.ptr(), w.data_ptr(), pooled2.data_ptr(), argmax.data_ptr(), attn.data_ptr(), y.ptr(), B, H, W, C,
           L.stream())
    if tape is None:
        return y

    def bwd():
        g = y.grad()
        if g is None:
            return
        assert y.grad_ld() == C
        tgt, acc = x.grad_target()
        assert g.dtype == tgt.dtype
        gx = tgt if acc == 0 else _empty((B, H, W, C), dev, tgt.dtype)
        gw = param_grad(w) if w.requires_grad else _empty(w.shape, dev)
        wsb = L.load().hyres_spatial_attn_workspace_bytes(B, H, W)
        ws = _ws(wsb, dev, slot=1)
        if x.half:
            L.call("hyres_spatial_attn_bwd_f16", x.ptr(), w.data_ptr(), pooled2.data_ptr(), argmax.data_ptr(),
                   attn.data_ptr(), g.data_ptr(), gx.data_ptr(), gw.data_ptr(), B, H, W, C, ws.data_ptr(), ws.numel(),
                   int(g.dtype == torch.float16), L.stream())
        else:
            L.call("hyres_spatial_attn_bwd", x.ptr(), w.data_ptr(), pooled2.data_ptr(), argmax.data_ptr(),
                   attn.data_ptr(), g.data_ptr(), gx.data_ptr(), gw.data_ptr(), B, H, W, C, ws.data_ptr(), ws.numel(),
                   L.stream())
        if acc:
            accumulate(gx, tgt)

    tape.push(bwd)
    return y


def add(tape: Optional[Tape], a: Node, b: Node, alpha: float = 1.0) -> Node:
    """y = a + alpha*b (models/hyres.py:48 residual = x - jpeg; :62 x_hat_initial = jpeg + residual_hat)."""
    assert a.contiguous and b.contiguous
    y = Node.new(a.B, a.H, a.W, a.C, a.device, rg=a.rg or b.rg)
    L.call("hyres_axpby", a.ptr(), b.ptr(), float(alpha), y.ptr(), y.P * y.C, L.stream())
    if tape is None:
        return y

    def bwd():
        g = y.grad()
        if g is None:
            return
        if a.rg:
            a.set_grad(g)
        if b.rg:
            tgt, acc = b.grad_target()
            L.call("hyres_scale", g.data_ptr(), None, float(alpha), tgt.data_ptr(), y.P * y.C, acc, L.stream())

    tape.push(bwd)
    return y


def add_clamp01(tape: Optional[Tape], x0: Node, r: Node) -> Node:
    """x_hat = clamp(x0 + r, 0, 1)  (models/hyres.py:66-67)."""
    n = x0.P * x0.C
    pre = _empty(x0.v.shape, x0.device) if tape is not None else None
    y = Node.new(x0.B, x0.H, x0.W, x0.C, x0.device)
    if pre is not None:
        L.call("hyres_axpby", x0.ptr(), r.ptr(), 1.0, pre.data_ptr(), n, L.stream())
    L.call("hyres_add_clamp01", x0.ptr(), r.ptr(), y.ptr(), n, L.stream())
    if tape is None:
        return y

    def bwd():
        g = y.grad()
        if g is None:
            return
        gp = _empty(x0.v.shape, x0.device)
        L.call("hyres_add_clamp01_bwd", pre.data_ptr(), g.data_ptr(), gp.data_ptr(), 0, n, L.stream())
        for t in (x0, r):
            if t.rg:
                t.set_grad(gp)

    tape.push(bwd)
    return y
