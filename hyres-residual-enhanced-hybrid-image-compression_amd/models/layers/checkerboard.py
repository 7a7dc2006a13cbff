"""Masked convolutions (models/layers/checkerboard.py) on HIP."""
from __future__ import annotations

from typing import Any

import torch

from hyres_hip import _lib as L
from hyres_hip import ops as O
from hyres_hip.layers import Conv2d

__all__ = ["MaskedConv2d", "CheckboardMaskedConv2d"]


class _MaskedBase(Conv2d):
    def _apply_mask_inplace(self):
        # reference: ``self.weight.data *= self.mask`` on every forward (the parameter itself changes)
        w = self.weight
        L.call("hyres_mul", w.data_ptr(), self.mask.data_ptr(), w.data_ptr(), w.numel(), L.stream())

    def hip(self, tape, x, act=L.ACT_NONE, slope=None, res=None, out=None):
        self._apply_mask_inplace()
        return O.conv2d(tape, x, self.weight, self.bias, stride=self.stride[0], pad=self.padding[0],
                        dil=self.dilation[0], act=act, slope=slope, res=res, out=out, mask=self.mask)


class MaskedConv2d(_MaskedBase):
    """PixelCNN-style mask "A"/"B" (models/layers/checkerboard.py:8-23; unused by HyRES)."""

    def __init__(self, *args: Any, mask_type: str = "A", **kwargs: Any):
        super().__init__(*args, **kwargs)
        if mask_type not in ("A", "B"):
            raise ValueError(f'Invalid "mask_type" value "{mask_type}"')
        self.register_buffer("mask", torch.ones_like(self.weight.data))
        _, _, h, w = self.mask.size()
        self.mask[:, :, h // 2, w // 2 + (mask_type == "B"):] = 0
        self.mask[:, :, h // 2 + 1:] = 0


class CheckboardMaskedConv2d(_MaskedBase):
    """5x5 checkerboard context model: mask = 1 where (kh + kw) is odd (models/layers/checkerboard.py:26-50).

    Forward masks the weight in place (as the reference does) and runs the HIP conv; the weight
    gradient stays dense over all 25 taps, exactly like the reference's autograd."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.register_buffer("mask", torch.zeros_like(self.weight.data))
        self.mask[:, :, 0::2, 1::2] = 1
        self.mask[:, :, 1::2, 0::2] = 1
