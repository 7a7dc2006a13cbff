"""Deterministic synthetic weights for the HyRES architecture (no checkpoint ships with the reference).

The recipe is keyed on the parameter NAME (not on state_dict order), so any implementation with the
reference's key layout (``ResidualJPEGCompression.state_dict()``) gets bit-identical
weights: the reference model in ``tests/golden/make_golden.py``, the oracle and this package.

Per key (seed = crc32(key) ^ base_seed, CPU ``torch.Generator`` so values are platform-independent):
  * conv / linear ``weight`` (ndim >= 2) and their ``bias``: U(-g/sqrt(fan_in), g/sqrt(fan_in)) with
    PyTorch's fan_in convention (dim 1 x kernel area) and gain ``g`` (default sqrt(3): variance
    preserving, so latents are O(1) and the quantizer's rounding is actually exercised);
  * GDN ``beta``  : stored sqrt(1 + U(0, .5) + 2^-36)      (compressai init is sqrt(1 + 2^-36));
  * GDN ``gamma`` : stored sqrt(0.1*I + U(0, 0.02) + 2^-36);
  * EntropyBottleneck ``_matrix{i}`` default constant + U(-.1, .1); ``_bias{i}`` U(-.5, .5);
    ``_factor{i}`` U(-.5, .5); ``quantiles`` [-10, m, 10] with median m ~ U(-.5, .5);
  * PReLU ``weight`` : 0.25 + U(-.1, .1);
  * every buffer (masks, bounds, pedestals, targets, empty CDF tables) keeps its module default.
"""
from __future__ import annotations

import math
import zlib
from typing import Dict

import torch
from torch import Tensor

PEDESTAL = 2.0 ** -36


def _gen(key: str, base_seed: int) -> torch.Generator:
    g = torch.Generator(device="cpu")
    g.manual_seed((zlib.crc32(key.encode()) ^ int(base_seed)) & 0x7FFFFFFF)
    return g


def _u(shape, lo, hi, g) -> Tensor:
    return torch.rand(shape, generator=g, dtype=torch.float32) * (hi - lo) + lo


def synthetic_value(key: str, default: Tensor, base_seed: int = 1926, gain: float = math.sqrt(3.0),
                    conv_weights: Dict[str, Tensor] = None) -> Tensor:
    """Return the recipe value for ``key`` given the module's default tensor (shape/dtype)."""
    g = _gen(key, base_seed)
    name = key.rsplit(".", 1)[-1]
    shape = tuple(default.shape)
    if not default.is_floating_point():
        return default.clone()
    if "entropy_bottleneck" in key:
        if name.startswith("_matrix"):
            return default + _u(shape, -0.1, 0.1, g)
        if name.startswith("_bias") or name.startswith("_factor"):
            return _u(shape, -0.5, 0.5, g)
        if name == "quantiles":
            q = default.clone()
            q[:, :, 1] = _u((shape[0], 1), -0.5, 0.5, g)
            return q
        return default.clone()
    if name == "beta" and default.dim() == 1:
        return torch.sqrt(1.0 + _u(shape, 0.0, 0.5, g) + PEDESTAL)
    if name == "gamma" and default.dim() == 2:
        c = shape[0]
        return torch.sqrt(0.1 * torch.eye(c) + _u(shape, 0.0, 0.02, g) + PEDESTAL)
    if name == "weight" and default.dim() == 1 and (".act_in" in key or default.numel() == 1):
        return 0.25 + _u(shape, -0.1, 0.1, g)  # PReLU slope
    if name == "weight" and default.dim() >= 2:
        fan_in = shape[1] * (int(torch.tensor(shape[2:]).prod()) if len(shape) > 2 else 1)
        b = gain / math.sqrt(fan_in)
        return _u(shape, -b, b, g)
    if name == "bias" and conv_weights is not None:
        w = conv_weights.get(key[: -len("bias")] + "weight")
        if w is not None:
            fan_in = w.shape[1] * (int(torch.tensor(w.shape[2:]).prod()) if w.dim() > 2 else 1)
            b = gain / math.sqrt(fan_in)
            return _u(shape, -b, b, g)
    return default.clone()


def synthetic_state_dict(template: Dict[str, Tensor], base_seed: int = 1926,
                         gain: float = math.sqrt(3.0)) -> Dict[str, Tensor]:
    """Fill every key of ``template`` (a state_dict) with its recipe value (CPU fp32)."""
    tmpl = {k: v.detach().cpu() for k, v in template.items()}
    out = {}
    for k, v in tmpl.items():
        out[k] = synthetic_value(k, v, base_seed, gain, conv_weights=tmpl)
    return out
