"""Quantizer (models/utils/quantization.py:4-14) on HIP.

Inside the codec the quantiser is fused into the checkerboard kernels; this standalone class keeps the
reference API for callers that use it directly: "noise" adds U(-.5,.5) from the HIP RNG, "ste" returns
round(x) - x.detach() + x (identity gradient), anything else rounds (half-to-even)."""
from __future__ import annotations

import torch

from hyres_hip import _lib as L
from hyres_hip.ops import _empty


class _QuantFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mode):
        L.require_device(x)
        x = x.contiguous()
        y = _empty(x.shape, x.device)
        L.call("hyres_quantize", x.data_ptr(), int(mode), y.data_ptr(), x.numel(), L.stream())
        ctx.mode = mode
        return y

    @staticmethod
    def backward(ctx, g):
        if ctx.mode == 0:  # STE: d/dx [round(x) - x.detach() + x] = 1
            return g, None
        return None, None  # round(): zero gradient


class Quantizer:
    def quantize(self, inputs, quantize_type="noise"):
        if quantize_type == "noise":
            noise = _empty(inputs.shape, inputs.device)
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
            L.call("hyres_uniform_noise", noise.data_ptr(), noise.numel(), seed, 0, L.stream())
            return inputs + noise
        elif quantize_type == "ste":
            return _QuantFn.apply(inputs, 0)
        else:
            return _QuantFn.apply(inputs, 1)
