"""Quantisation, checkerboard two-pass context split/merge and entropy-model likelihoods on HIP.

Reference anchors (reference repo paths):
  * LightWeightCheckerboard.forward split / quantise / combine   models/checkerboard.py:98-142
  * Quantizer                                                   models/utils/quantization.py:5-14
  * compressai 1.2.6 EntropyBottleneck / GaussianConditional     (restated in oracle/compressai_restated.py)
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from . import _lib as L
from .ops import Node, Tape, _empty, param_grad, _ws


_SALT = {"z": 0x5A17, "y_anchor": 0xA7C4, "y_non_anchor": 0x70A4, "y": 0x6C59}


class NoiseSource:
    """U(-0.5, 0.5) noise from the HIP counter-based RNG (replaces torch ``uniform_`` draws).

    Seeds are drawn from torch's CPU generator, so ``torch.manual_seed`` makes runs reproducible.
    Tests may inject explicit tensors (``inject``) keyed like the reference's draw order:
    EB(z) -> Quantizer(anchor) -> Quantizer(non-anchor) -> GC(y)."""

    def __init__(self):
        self.injected: Optional[Dict[str, torch.Tensor]] = None

    def draw(self, key: str, like: Node) -> torch.Tensor:
        if self.injected is not None and key in self.injected:
            t = self.injected[key]
            assert tuple(t.shape) == (like.B, like.H, like.W, like.C), (key, t.shape)
            return t.contiguous()
        out = _empty((like.B, like.H, like.W, like.C), like.device)
        if torch.cuda.is_current_stream_capturing():
            # inside a HIP graph capture a host seed would be baked into every replay: draw from the
            # device-resident seed instead (advanced on device after each draw)
            L.call("hyres_uniform_noise_dev", out.data_ptr(), out.numel(), self._device_seed(like.device).data_ptr(),
                   _SALT[key], L.stream())
            return out
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        L.call("hyres_uniform_noise", out.data_ptr(), out.numel(), seed, 0, L.stream())
        return out

    def _device_seed(self, device) -> torch.Tensor:
        seeds = self.__dict__.setdefault("_seeds", {})
        t = seeds.get(device.index)
        if t is None:  # initialised (outside any capture) from torch's CPU generator: manual_seed reproducible
            t = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).to(device)
            seeds[device.index] = t
        return t


def _eb_param_lists(eb):
    mats = [getattr(eb, f"_matrix{i}") for i in range(5)]
    biases = [getattr(eb, f"_bias{i}") for i in range(5)]
    factors = [getattr(eb, f"_factor{i}") for i in range(4)]
    return mats, biases, factors


def eb_pack(eb) -> torch.Tensor:
    mats, biases, factors = _eb_param_lists(eb)
    C = eb.channels
    packed = _empty((C, L.EB_REC), eb.quantiles.device)
    L.call("hyres_eb_pack", L.ptr_array(mats), L.ptr_array(biases), L.ptr_array(factors), eb.quantiles.data_ptr(),
           packed.data_ptr(), C, L.stream())
    return packed


def entropy_bottleneck(tape: Optional[Tape], eb, z: Node, training: bool, noisequant: bool,
                       noise: NoiseSource) -> Tuple[Node, Node]:
    """EntropyBottleneck(z) (+ the STE re-quantisation of models/checkerboard.py:98-101).

    Returns (z_hat fed to h_s, z_likelihoods)."""
    assert z.contiguous
    C = z.C
    P = z.P
    packed = eb_pack(eb)
    nz = noise.draw("z", z) if training else None
    z_q = _empty(z.v.shape, z.device)
    lik = Node.new(z.B, z.H, z.W, C, z.device)
    z_hat = None if noisequant else Node.new(z.B, z.H, z.W, C, z.device)
    L.call("hyres_eb_fwd", z.ptr(), packed.data_ptr(), L.ptr(nz), int(training), z_q.data_ptr(), lik.ptr(),
           None if z_hat is None else z_hat.ptr(), P, C, L.stream())
    if z_hat is None:
        z_hat = Node(z_q, rg=True)
    if tape is None:
        return z_hat, lik

    def bwd():
        g_lik = lik.grad()
        g_zh = z_hat.grad()
        if g_lik is None and g_zh is None:
            return
        mats, biases, factors = _eb_param_lists(eb)
        wsb = L.load().hyres_eb_workspace_bytes(P, C)
        ws = _ws(wsb, z.device, slot=3)
        tgt, acc = z.grad_target()
        gz = tgt if acc == 0 else _empty(z.v.shape, z.device)
        L.call("hyres_eb_bwd", z_q.data_ptr(), packed.data_ptr(), lik.ptr(), L.ptr(g_lik), L.ptr(g_zh),
               int(training), int(noisequant), gz.data_ptr(), ws.data_ptr(), P, C, L.stream())
        if acc:
            L.call("hyres_accumulate", gz.data_ptr(), tgt.data_ptr(), gz.numel(), L.stream())
        if any(p.requires_grad for p in mats + biases + factors):
            nb = (P + 1023) // 1024
            gm = [param_grad(p) for p in mats]
            gb = [param_grad(p) for p in biases]
            gf = [param_grad(p) for p in factors]
            gq = param_grad(eb.quantiles) if eb.quantiles.requires_grad else None
            L.call("hyres_eb_unpack_grad", ws.data_ptr(), nb, L.ptr_array(mats), L.ptr_array(factors),
                   L.ptr_array(gm), L.ptr_array(gb), L.ptr_array(gf), L.ptr(gq), C, 1, L.stream())

    tape.push(bwd)
    return z_hat, lik


class _AuxLoss(torch.autograd.Function):
    """EntropyBottleneck.loss() (compressai aux loss): sum |L(quantiles) - target|, MLP detached."""

    @staticmethod
    def forward(ctx, quantiles, eb):
        packed = eb_pack(eb)
        loss = _empty((1,), quantiles.device)
        gq = _empty(quantiles.shape, quantiles.device)
        L.call("hyres_eb_aux_loss", packed.data_ptr(), quantiles.data_ptr(), eb.target.data_ptr(), loss.data_ptr(),
               gq.data_ptr(), eb.channels, L.stream())
        ctx.save_for_backward(gq)
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        (gq,) = ctx.saved_tensors
        out = _empty(gq.shape, gq.device)
        g = g.contiguous().reshape(1)
        L.call("hyres_scale", gq.data_ptr(), g.data_ptr(), 1.0, out.data_ptr(), gq.numel(), 0, L.stream())
        return out, None


def eb_aux_loss(eb) -> torch.Tensor:
    return _AuxLoss.apply(eb.quantiles, eb)


def checkerboard_anchor(tape: Optional[Tape], y: Node, params_a: Node, noisequant: bool,
                        noise: NoiseSource) -> Node:
    """Anchor pass: y_anchor = y on (h+w) even; y_anchor_hat = STE(y_a - mu_a) + mu_a or y_a + U.

    models/checkerboard.py:106-122.  params_a = param_aggregation output [.., scales | means]."""
    B, H, W, C = y.B, y.H, y.W, y.C
    nq = noise.draw("y_anchor", y) if noisequant else None
    means = params_a.v[..., C:2 * C]
    ya_hat = Node.new(B, H, W, C, y.device)
    L.call("hyres_ckbd_anchor_fwd", y.ptr(), means.data_ptr(), params_a.ld, L.ptr(nq), ya_hat.ptr(), B, H, W, C,
           L.stream())
    if tape is None:
        return ya_hat

    def bwd():
        # STE / additive noise: d y_anchor_hat / d y = 1 at anchor positions, 0 for the means
        # (round(t) - t.detach() + t  +  mu has zero net mu-gradient). Only the context-model path is
        # left here: the y_hat path is handled by the non-anchor/GC backward, which writes y.grad.
        g = ya_hat.grad()
        if g is None or not y.rg:
            return
        tgt, acc = y.grad_target()
        assert acc == 1, "non-anchor/GC backward must have written y.grad first"
        L.call("hyres_ckbd_anchor_bwd", g.data_ptr(), tgt.data_ptr(), B, H, W, C, L.stream())

    tape.push(bwd)
    return ya_hat


def checkerboard_nonanchor_gc(tape: Optional[Tape], y: Node, ya_hat: Node, params_a: Node, params_na: Node,
                              training: bool, noisequant: bool, noise: NoiseSource):
    """Non-anchor pass + combine + GaussianConditional(y, scales, means): models/checkerboard.py:126-142.

    Returns (y_hat, y_likelihoods).  ``ya_hat`` keeps its own gradient for the context-model path; the
    y_hat gradient is routed to y by this op's backward."""
    B, H, W, C = y.B, y.H, y.W, y.C
    dev = y.device
    nq = noise.draw("y_non_anchor", y) if noisequant else None
    ngc = noise.draw("y", y) if training else None
    y_hat = Node.new(B, H, W, C, dev)
    scales = _empty((B, H, W, C), dev)
    means = _empty((B, H, W, C), dev)
    y_q = _empty((B, H, W, C), dev)
    lik = Node.new(B, H, W, C, dev)
    L.call("hyres_ckbd_nonanchor_gc_fwd", y.ptr(), ya_hat.ptr(), params_a.ptr(), params_a.ld, params_na.ptr(),
           params_na.ld, L.ptr(nq), L.ptr(ngc), y_hat.ptr(), scales.data_ptr(), means.data_ptr(), y_q.data_ptr(),
           lik.ptr(), B, H, W, C, L.stream())
    if tape is None:
        return y_hat, lik

    def bwd():
        g_yh = y_hat.grad()
        g_lik = lik.grad()
        if g_yh is None and g_lik is None:
            return
        if g_yh is None:
            from .ops import zeros
            g_yh = zeros((B, H, W, C), dev)
        # y_hat = y_a_hat + y_na_hat: the anchor half's gradient continues through ya_hat's STE
        # (same gradient for every position) -> accounted for in ckbd_gc_bwd's g_y; record nothing on
        # ya_hat here so that ya_hat.grad() afterwards only holds the context-model contribution.
        gy_t, acc = y.grad_target()
        assert acc == 0, "y.grad must be written first by the GC backward"
        gpa, _ = params_a.grad_target()
        gpn, _ = params_na.grad_target()
        assert gpa.stride(2) == params_a.grad_ld()
        L.call("hyres_ckbd_gc_bwd", y_q.data_ptr(), scales.data_ptr(), means.data_ptr(), L.ptr(g_lik),
               g_yh.data_ptr(), int(training), gy_t.data_ptr(), gpa.data_ptr(), params_a.grad_ld(), gpn.data_ptr(),
               params_na.grad_ld(), B, H, W, C, L.stream())

    tape.push(bwd)
    return y_hat, lik
