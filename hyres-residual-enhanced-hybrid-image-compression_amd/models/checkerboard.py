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
from typing import Optional

import torch
import torch.nn as nn

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
    def hip(self, tape, x: Node, training: bool, noisequant: bool):
        M = self.M
        T = O.Trace
        y = self.g_a.hip(tape, x)
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
        x_hat = self.g_s.hip(tape, y_hat)
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

    def compress(self, x):
        raise NotImplementedError("rANS entropy coding (compress/decompress) is out of scope for this build: "
                                  "SURVEY.md §8f row f1")

    def decompress(self, strings, shape):
        raise NotImplementedError("rANS entropy coding (compress/decompress) is out of scope for this build: "
                                  "SURVEY.md §8f row f1")

    def update(self, scale_table=None, force=False, **kwargs):
        if scale_table is None:
            scale_table = get_scale_table()
        updated = self.gaussian_conditional.update_scale_table(scale_table, force=force)
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
