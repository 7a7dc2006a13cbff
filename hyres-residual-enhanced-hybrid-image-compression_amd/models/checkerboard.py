"""LightWeightCheckerboard residual codec (models/checkerboard.py:24-283) on MI355X.

Same module tree / state_dict keys as the reference; ``forward`` runs the whole codec as one HIP tape:
  g_a -> h_a -> EntropyBottleneck (+STE about the medians) -> h_s -> [anchor] param_aggregation ->
  anchor quantiser -> CheckboardMaskedConv2d -> [non-anchor] param_aggregation -> non-anchor quantiser +
  combine + GaussianConditional -> g_s.
``torch.cat([latent_params, zeros])`` / ``torch.cat([latent_params, ctx_params])`` are one NHWC buffer
[B,h,w,4M]: h_s writes channels [0,2M), the context model writes [2M,4M); the anchor pass reads only
the first 2M input channels of param_aggregation.0 (the zero half contributes nothing).
"""
from __future__ import annotations

import math
import time
from typing import Optional

import torch
import torch.nn as nn

from hyres_hip import _lib as L
from hyres_hip import entropy_coding as EC
from hyres_hip import entropy_ops as E
from hyres_hip import ops as O
from hyres_hip import runtime
from hyres_hip.layers import (CompressionModel, EntropyBottleneck, GaussianConditional, GDN, ReLU,
                              ResidualBottleneckBlock, Sequential, conv, deconv)
from hyres_hip.ops import Node

from .layers import AttentionBlock, CheckboardMaskedConv2d, conv1x1, conv3x3
from .utils.quantization import Quantizer

SCALES_MIN, SCALES_MAX, SCALES_LEVELS = 0.11, 256, 64


def get_scale_table(min=SCALES_MIN, max=SCALES_MAX, levels=SCALES_LEVELS):
    """models/checkerboard.py:20-21."""
    return torch.exp(torch.linspace(math.log(min), math.log(max), levels))


class LightWeightCheckerboard(CompressionModel):
    # True: obtain z_hat / y_anchor_hat inside compress by decoding the just-written strings, literally as
    # the reference does; False (default): dequantise the encoded symbols on the device (identical values)
    decode_in_compress = False

    def __init__(self, N=128, M=192):
        super().__init__()
        self.N, self.M = N, M
        self.entropy_bottleneck = EntropyBottleneck(N)
        self.gaussian_conditional = GaussianConditional(None)
        self.quantizer = Quantizer()
        self.noise = E.NoiseSource()

        self.g_a = Sequential(
            conv(3, N), GDN(N), ResidualBottleneckBlock(N, N), AttentionBlock(N),
            conv(N, N), GDN(N), ResidualBottleneckBlock(N, N), conv(N, M), AttentionBlock(M))
        self.g_s = Sequential(
            AttentionBlock(M), deconv(M, N), ResidualBottleneckBlock(N, N), GDN(N, inverse=True),
            deconv(N, N), AttentionBlock(N), ResidualBottleneckBlock(N, N), GDN(N, inverse=True),
            deconv(N, 3))
        self.h_a = Sequential(
            conv3x3(M, N), ReLU(inplace=True), conv(N, N), ReLU(inplace=True), conv(N, N))
        self.h_s = Sequential(
            deconv(N, N), ReLU(inplace=True), deconv(N, N * 3 // 2), ReLU(inplace=True),
            conv3x3(N * 3 // 2, 2 * M))
        self.context_prediction = CheckboardMaskedConv2d(M, 2 * M, kernel_size=5, padding=2, stride=1)
        self.param_aggregation = Sequential(
            conv1x1(4 * M, 640), ReLU(inplace=True), conv1x1(640, 512), ReLU(inplace=True), conv1x1(512, 2 * M))

    # ------------------------------------------------------------------ HIP graph
    def _g_a(self, tape, x: Node) -> Node:
        """g_a; under autocast inference its layers above the latent resolution keep fp16 activations in
        HBM (O.f16_region), conv(N, M) writes the latent y in fp32."""
        with O.f16_region():
            t = self.g_a[:7].hip(tape, x)
        return self.g_a[7:].hip(tape, t)

    def _g_s(self, tape, y_hat: Node) -> Node:
        """g_s; the latent AttentionBlock(M) in fp32, the rest in the fp16 region (autocast inference)."""
        t = self.g_s[:1].hip(tape, y_hat)
        with O.f16_region():
            return self.g_s[1:].hip(tape, t)

    def hip(self, tape, x: Node, training: bool, noisequant: bool):
        M = self.M
        T = O.Trace
        y = self._g_a(tape, x)
        O.GradReady.mark(tape, "hyper")  # backward: h_a/h_s/entropy/context/param_aggregation done
        z = self.h_a.hip(tape, y)
        z_hat, z_lik = self.entropy_bottleneck.hip(tape, z, training, noisequant, self.noise)
        lc = Node.new(y.B, y.H, y.W, 4 * M, y.device)
        latent = lc.slice(0, 2 * M)
        ctx = lc.slice(2 * M, 4 * M)
        self.h_s.hip(tape, z_hat, out=latent)
        params_a = self.param_aggregation.hip(tape, latent)
        ya_hat = E.checkerboard_anchor(tape, y, params_a, noisequant, self.noise)
        self.context_prediction.hip(tape, ya_hat, out=ctx)
        params_na = self.param_aggregation.hip(tape, lc)
        y_hat, y_lik = E.checkerboard_nonanchor_gc(tape, y, ya_hat, params_a, params_na, training, noisequant,
                                                   self.noise)
        O.GradReady.mark(tape, "g_s")
        x_hat = self._g_s(tape, y_hat)
        for name, n in (("y", y), ("z", z), ("z_hat", z_hat), ("latent_params", latent), ("y_anchor_hat", ya_hat),
                        ("ctx_params", ctx), ("y_hat", y_hat), ("residual_hat", x_hat)):
            T.add(name, n)
        return x_hat, y_lik, z_lik

    def forward(self, x, noisequant=False):
        training = self.training

        def build(tape, tensors):
            (xt,) = tensors
            xn = O.to_nhwc(xt, rg=xt.requires_grad)
            x_hat, y_lik, z_lik = self.hip(tape, xn, training, noisequant)
            return [xn], [x_hat, y_lik, z_lik]

        x_hat, y_lik, z_lik = runtime.run(build, [x], list(self.parameters()))
        return {"x_hat": x_hat, "likelihoods": {"y": y_lik, "z": z_lik}}

    def _split_tensor(self, x, mode):
        """models/checkerboard.py:149-157 (anchor = (h+w) even)."""
        h, w = x.shape[-2:]
        i = torch.arange(h, device=x.device).view(h, 1)
        j = torch.arange(w, device=x.device).view(1, w)
        anchor = ((i + j) % 2 == 0)
        keep = anchor if mode == "anchor" else ~anchor
        return x * keep.to(x.dtype)

    # ------------------------------------------------------------------ entropy coding (§8f f1)
    def _hyper(self, z_hat: Node, H: int, W: int):
        """h_s(z_hat) into cat-buffer [latent | ctx] and the anchor parameters (checkerboard.py:172-180)."""
        M = self.M
        lc = Node.new(z_hat.B, H, W, 4 * M, z_hat.device, rg=False)
        latent = lc.slice(0, 2 * M)
        self.h_s.hip(None, z_hat, out=latent)
        params_a = self.param_aggregation.hip(None, latent)  # cat([latent, 0]): zero half skipped
        return lc, params_a

    @torch.no_grad()
    def compress(self, x):
        """models/checkerboard.py:167-201: strings [[anchor, non_anchor], z] (one string per image each).
        The reference decodes its own anchor / z strings to obtain y_anchor_hat / z_hat; the symbols round
        trip exactly, so here they are dequantised on the device from the encoded symbols instead."""
        start_time = time.time()
        dev = next(self.parameters()).device
        M = self.M
        gc, eb = self.gaussian_conditional, self.entropy_bottleneck
        xn = O.to_nhwc(x.to(dev).float().contiguous(), rg=False)
        y = self._g_a(None, xn)
        z = self.h_a.hip(None, y)
        z_strings = EC.eb_compress(eb, z)
        z_hat = EC.eb_decompress(eb, z_strings, z.H, z.W, dev) if self.decode_in_compress else None
        if z_hat is None:
            z_hat = Node.new(z.B, z.H, z.W, z.C, dev, rg=False)
            sym = torch.empty(z.B * z.C * z.H * z.W, dtype=torch.int32, device=dev)
            L.call("hyres_eb_symbols", z.ptr(), z.ld, EC._medians(eb).data_ptr(), z.B, z.H, z.W, z.C, sym.data_ptr(),
                   None, 0, 0, L.stream())
            L.call("hyres_eb_symbols", None, 0, EC._medians(eb).data_ptr(), z.B, z.H, z.W, z.C, sym.data_ptr(),
                   z_hat.ptr(), z_hat.ld, 1, L.stream())
        lc, params_a = self._hyper(z_hat, y.H, y.W)
        anchor_strings = EC.gc_compress(gc, y, params_a, M, parity=0)
        ya_hat = Node.new(y.B, y.H, y.W, M, dev, rg=False)
        if self.decode_in_compress:
            EC.gc_decompress(gc, anchor_strings, params_a, M, ya_hat)
        else:
            sym, _ = EC._gc_indexes(gc, params_a, M, y, 0)
            L.call("hyres_gc_dequant", sym.data_ptr(), params_a.ptr(), params_a.ld, M, y.B, y.H, y.W, ya_hat.ptr(),
                   ya_hat.ld, 0, L.stream())
        self.context_prediction.hip(None, ya_hat, out=lc.slice(2 * M, 4 * M))
        params_na = self.param_aggregation.hip(None, lc)
        non_anchor_strings = EC.gc_compress(gc, y, params_na, M, parity=1)
        strings = EC.resolve([[anchor_strings, non_anchor_strings], z_strings])  # host rANS threads join
        return {
            "strings": strings,
            "shape": torch.Size([z.H, z.W]),
            "time": time.time() - start_time,
        }

    @torch.no_grad()
    def decompress(self, strings, shape):
        """models/checkerboard.py:203-240 (including its ``g_s(y_hat).clamp_(0, 1)``)."""
        start_time = time.time()
        dev = next(self.parameters()).device
        M = self.M
        gc, eb = self.gaussian_conditional, self.entropy_bottleneck
        h, w = int(shape[0]), int(shape[1])
        z_hat = EC.eb_decompress(eb, strings[1], h, w, dev)
        H, W = h * 4, w * 4
        lc, params_a = self._hyper(z_hat, H, W)
        y_hat = Node.new(z_hat.B, H, W, M, dev, rg=False)
        EC.gc_decompress(gc, strings[0][0], params_a, M, y_hat)          # y_anchor_hat
        self.context_prediction.hip(None, y_hat, out=lc.slice(2 * M, 4 * M))
        params_na = self.param_aggregation.hip(None, lc)
        EC.gc_decompress(gc, strings[0][1], params_na, M, y_hat, accumulate=True)  # + y_non_anchor_hat
        x_hat = O.to_nchw(self._g_s(None, y_hat)).clamp_(0, 1)
        return {"x_hat": x_hat, "time": time.time() - start_time}

    def inference(self, x):
        """models/checkerboard.py:242-259."""
        c = self.compress(x)
        d = self.decompress(c["strings"], c["shape"])
        return {"x_hat": d["x_hat"], "time": {"compression": c["time"], "decompression": d["time"],
                                             "total": c["time"] + d["time"]}}

    def update(self, scale_table=None, force=False, **kwargs):
        """models/checkerboard.py:261-267."""
        if scale_table is None:
            scale_table = get_scale_table()
        updated = self.gaussian_conditional.update_scale_table(scale_table, force=force)
        updated |= super().update(force=force)
        return updated

    def load_state_dict(self, state_dict, strict: bool = True, **kwargs):
        """models/checkerboard.py:269-276: resize the (possibly empty) entropy-coder buffers first."""
        for mod_name, mod in (("gaussian_conditional", self.gaussian_conditional),
                              ("entropy_bottleneck", self.entropy_bottleneck)):
            for b in ("_quantized_cdf", "_offset", "_cdf_length", "scale_table"):
                key = f"{mod_name}.{b}"
                if key in state_dict and hasattr(mod, b):
                    reg = getattr(mod, b)
                    if reg.numel() == 0:
                        reg.resize_(state_dict[key].size())
        out = super().load_state_dict(state_dict, strict=strict)
        O.bump_weight_epoch()
        return out

    @classmethod
    def from_state_dict(cls, state_dict):
        net = cls()
        net.load_state_dict(state_dict)
        return net
