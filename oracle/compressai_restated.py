"""TEST INFRASTRUCTURE ONLY — restatement of the compressai 1.2.6 surface used by HyRES.

compressai (pinned ``compressai~=1.2.6`` at /root/reference/requirements.txt:11) is a third-party
dependency that is NOT vendored under /root/reference and is not installed in this image.  This
module restates, from the published 1.2.6 algorithm, exactly the classes/functions the reference
imports (/root/reference/models/checkerboard.py:6-11, models/hyres.py:2):

  * ``compressai.ops.LowerBound`` / ``LowerBoundFunction``  (bound_ops.py: max(x, b); backward passes
    the gradient where ``x >= b`` or ``grad < 0``)
  * ``compressai.ops.NonNegativeParametrizer`` (parametrizers.py: out = LowerBound(x)^2 - pedestal,
    pedestal = reparam_offset^2 = 2^-36, bound = sqrt(minimum + pedestal))
  * ``compressai.ops.quantize_ste``  ((round(x) - x).detach() + x)
  * ``compressai.layers.GDN``   (norm = conv1x1(x^2, gamma') + beta'; x*rsqrt(norm) / x*sqrt(norm))
  * ``compressai.models.sensetime.ResidualBottleneckBlock`` (1x1 -> ReLU -> 3x3 -> ReLU -> 1x1 + id)
  * ``compressai.models.utils.conv / deconv / update_registered_buffers``
  * ``compressai.entropy_models.EntropyBottleneck`` (factorized prior, filters (3,3,3,3),
    likelihood = sigmoid(upper) - sigmoid(lower), medians = quantiles[:, :, 1:2])
  * ``compressai.entropy_models.GaussianConditional`` (0.5*erfc(-(v)/sqrt2) differences,
    scale LowerBound 0.11, likelihood LowerBound 1e-9)
  * ``compressai.models.base.CompressionModel`` (aux_loss = sum of EB losses)

Only the forward/backward semantics used on the hot path are restated; the rANS ``compress`` /
``update`` machinery (C++ in compressai) is out of scope.

This module is imported by ``oracle/`` and by ``tests/golden/make_golden.py`` (which places it in
``sys.modules`` as ``compressai.*`` so that the reference's own model files execute unchanged).
The shipped HIP product path never imports anything under ``oracle/``.
"""
from __future__ import annotations

import math
import types
from typing import Any, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch import Tensor


# --------------------------------------------------------------------------------------------
# ops
# --------------------------------------------------------------------------------------------
class LowerBoundFunction(torch.autograd.Function):
    """compressai/ops/bound_ops.py: forward max(x, bound); backward passes where x>=bound or g<0."""

    @staticmethod
    def forward(ctx, x, bound):
        ctx.save_for_backward(x, bound)
        return torch.max(x, bound)

    @staticmethod
    def backward(ctx, grad_output):
        x, bound = ctx.saved_tensors
        pass_through_if = (x >= bound) | (grad_output < 0)
        return pass_through_if * grad_output, None


class LowerBound(nn.Module):
    bound: Tensor

    def __init__(self, bound: float):
        super().__init__()
        self.register_buffer("bound", torch.Tensor([float(bound)]))

    def forward(self, x):
        return LowerBoundFunction.apply(x, self.bound)


class NonNegativeParametrizer(nn.Module):
    pedestal: Tensor

    def __init__(self, minimum: float = 0, reparam_offset: float = 2 ** -18):
        super().__init__()
        self.minimum = float(minimum)
        self.reparam_offset = float(reparam_offset)
        pedestal = self.reparam_offset ** 2
        self.register_buffer("pedestal", torch.Tensor([pedestal]))
        bound = (self.minimum + self.reparam_offset ** 2) ** 0.5
        self.lower_bound = LowerBound(bound)

    def init(self, x: Tensor) -> Tensor:
        return torch.sqrt(torch.max(x + self.pedestal, self.pedestal))

    def forward(self, x: Tensor) -> Tensor:
        out = self.lower_bound(x)
        out = out ** 2 - self.pedestal
        return out


def quantize_ste(x: Tensor) -> Tensor:
    return (torch.round(x) - x).detach() + x


# --------------------------------------------------------------------------------------------
# layers
# --------------------------------------------------------------------------------------------
def conv1x1(in_ch: int, out_ch: int, stride: int = 1) -> nn.Module:
    return nn.Conv2d(in_ch, out_ch, kernel_size=1, stride=stride)


def conv3x3(in_ch: int, out_ch: int, stride: int = 1) -> nn.Module:
    return nn.Conv2d(in_ch, out_ch, kernel_size=3, stride=stride, padding=1)


class GDN(nn.Module):
    def __init__(self, in_channels: int, inverse: bool = False, beta_min: float = 1e-6,
                 gamma_init: float = 0.1):
        super().__init__()
        self.inverse = bool(inverse)
        self.beta_reparam = NonNegativeParametrizer(minimum=float(beta_min))
        beta = self.beta_reparam.init(torch.ones(in_channels))
        self.beta = nn.Parameter(beta)
        self.gamma_reparam = NonNegativeParametrizer()
        gamma = self.gamma_reparam.init(float(gamma_init) * torch.eye(in_channels))
        self.gamma = nn.Parameter(gamma)

    def forward(self, x: Tensor) -> Tensor:
        _, C, _, _ = x.size()
        beta = self.beta_reparam(self.beta)
        gamma = self.gamma_reparam(self.gamma).reshape(C, C, 1, 1)
        norm = F.conv2d(x ** 2, gamma, beta)
        norm = torch.sqrt(norm) if self.inverse else torch.rsqrt(norm)
        return x * norm


class ResidualBottleneckBlock(nn.Module):
    def __init__(self, in_ch: int, out_ch: int):
        super().__init__()
        mid_ch = min(in_ch, out_ch) // 2
        self.conv1 = conv1x1(in_ch, mid_ch)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(mid_ch, mid_ch)
        self.conv3 = conv1x1(mid_ch, out_ch)
        self.skip = conv1x1(in_ch, out_ch) if in_ch != out_ch else nn.Identity()

    def forward(self, x: Tensor) -> Tensor:
        identity = self.skip(x)
        out = self.conv1(x)
        out = self.relu(out)
        out = self.conv2(out)
        out = self.relu(out)
        out = self.conv3(out)
        return out + identity


def conv(in_channels, out_channels, kernel_size=5, stride=2):
    return nn.Conv2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                     padding=kernel_size // 2)


def deconv(in_channels, out_channels, kernel_size=5, stride=2):
    return nn.ConvTranspose2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                              output_padding=stride - 1, padding=kernel_size // 2)


def update_registered_buffers(module, module_name, buffer_names, state_dict, policy="resize_if_empty",
                              dtype=torch.int):
    """compressai/models/utils.py: resize registered (possibly empty) buffers to the loaded shape."""
    valid = {n for n, _ in module.named_buffers()}
    for buffer_name in buffer_names:
        if buffer_name not in valid:
            raise ValueError(f'Invalid buffer name "{buffer_name}"')
    for buffer_name in buffer_names:
        key = f"{module_name}.{buffer_name}"
        if key not in state_dict:
            continue
        registered = getattr(module, buffer_name)
        if policy in ("resize_if_empty", "resize"):
            if policy == "resize" or registered.numel() == 0:
                registered.resize_(state_dict[key].size())
        elif policy == "register":
            module.register_buffer(buffer_name, torch.empty_like(state_dict[key], dtype=dtype).fill_(0))


# --------------------------------------------------------------------------------------------
# entropy models
# --------------------------------------------------------------------------------------------
class EntropyModel(nn.Module):
    def __init__(self, likelihood_bound: float = 1e-9, entropy_coder=None, entropy_coder_precision=16):
        super().__init__()
        self.entropy_coder_precision = int(entropy_coder_precision)
        self.use_likelihood_bound = likelihood_bound > 0
        if self.use_likelihood_bound:
            self.likelihood_lower_bound = LowerBound(likelihood_bound)
        self.register_buffer("_offset", torch.IntTensor())
        self.register_buffer("_quantized_cdf", torch.IntTensor())
        self.register_buffer("_cdf_length", torch.IntTensor())

    def quantize(self, inputs: Tensor, mode: str, means: Optional[Tensor] = None) -> Tensor:
        if mode not in ("noise", "dequantize", "symbols"):
            raise ValueError(f'Invalid quantization mode: "{mode}"')
        if mode == "noise":
            half = float(0.5)
            noise = torch.empty_like(inputs).uniform_(-half, half)
            return inputs + noise
        outputs = inputs.clone()
        if means is not None:
            outputs -= means
        outputs = torch.round(outputs)
        if mode == "dequantize":
            if means is not None:
                outputs += means
            return outputs
        return outputs.int()

    @staticmethod
    def dequantize(inputs: Tensor, means: Optional[Tensor] = None, dtype=torch.float) -> Tensor:
        if means is not None:
            outputs = inputs.type_as(means)
            outputs += means
        else:
            outputs = inputs.type(dtype)
        return outputs


class EntropyBottleneck(EntropyModel):
    def __init__(self, channels: int, *args: Any, tail_mass: float = 1e-9, init_scale: float = 10,
                 filters: Tuple[int, ...] = (3, 3, 3, 3), **kwargs: Any):
        super().__init__(*args, **kwargs)
        self.channels = int(channels)
        self.filters = tuple(int(f) for f in filters)
        self.init_scale = float(init_scale)
        self.tail_mass = float(tail_mass)
        filters = (1,) + self.filters + (1,)
        scale = self.init_scale ** (1 / (len(self.filters) + 1))
        channels = self.channels
        for i in range(len(self.filters) + 1):
            init = np.log(np.expm1(1 / scale / filters[i + 1]))
            matrix = torch.Tensor(channels, filters[i + 1], filters[i])
            matrix.data.fill_(init)
            self.register_parameter(f"_matrix{i:d}", nn.Parameter(matrix))
            bias = torch.Tensor(channels, filters[i + 1], 1)
            nn.init.uniform_(bias, -0.5, 0.5)
            self.register_parameter(f"_bias{i:d}", nn.Parameter(bias))
            if i < len(self.filters):
                factor = torch.Tensor(channels, filters[i + 1], 1)
                nn.init.zeros_(factor)
                self.register_parameter(f"_factor{i:d}", nn.Parameter(factor))
        self.quantiles = nn.Parameter(torch.Tensor(channels, 1, 3))
        init = torch.Tensor([-self.init_scale, 0, self.init_scale])
        self.quantiles.data = init.repeat(self.quantiles.size(0), 1, 1)
        target = np.log(2 / self.tail_mass - 1)
        self.register_buffer("target", torch.Tensor([-target, 0, target]))

    def _get_medians(self) -> Tensor:
        return self.quantiles[:, :, 1:2]

    def loss(self) -> Tensor:
        logits = self._logits_cumulative(self.quantiles, stop_gradient=True)
        return torch.abs(logits - self.target).sum()

    def _logits_cumulative(self, inputs: Tensor, stop_gradient: bool) -> Tensor:
        logits = inputs
        for i in range(len(self.filters) + 1):
            matrix = getattr(self, f"_matrix{i:d}")
            if stop_gradient:
                matrix = matrix.detach()
            logits = torch.matmul(F.softplus(matrix), logits)
            bias = getattr(self, f"_bias{i:d}")
            if stop_gradient:
                bias = bias.detach()
            logits = logits + bias
            if i < len(self.filters):
                factor = getattr(self, f"_factor{i:d}")
                if stop_gradient:
                    factor = factor.detach()
                logits = logits + torch.tanh(factor) * torch.tanh(logits)
        return logits

    def _likelihood(self, inputs: Tensor, stop_gradient: bool = False):
        half = float(0.5)
        lower = self._logits_cumulative(inputs - half, stop_gradient=stop_gradient)
        upper = self._logits_cumulative(inputs + half, stop_gradient=stop_gradient)
        likelihood = torch.sigmoid(upper) - torch.sigmoid(lower)
        return likelihood, lower, upper

    def forward(self, x: Tensor, training: Optional[bool] = None):
        if training is None:
            training = self.training
        perm = np.arange(len(x.shape))
        perm[0], perm[1] = perm[1], perm[0]
        inv_perm = np.arange(len(x.shape))[np.argsort(perm)]
        x = x.permute(*perm).contiguous()
        shape = x.size()
        values = x.reshape(x.size(0), 1, -1)
        outputs = self.quantize(values, "noise" if training else "dequantize", self._get_medians())
        likelihood, _, _ = self._likelihood(outputs)
        if self.use_likelihood_bound:
            likelihood = self.likelihood_lower_bound(likelihood)
        outputs = outputs.reshape(shape).permute(*inv_perm).contiguous()
        likelihood = likelihood.reshape(shape).permute(*inv_perm).contiguous()
        return outputs, likelihood


class GaussianConditional(EntropyModel):
    def __init__(self, scale_table, *args: Any, scale_bound: float = 0.11, tail_mass: float = 1e-9,
                 **kwargs: Any):
        super().__init__(*args, **kwargs)
        self.register_buffer("scale_table",
                             torch.Tensor(tuple(float(s) for s in scale_table)) if scale_table
                             else torch.Tensor())
        self.register_buffer("scale_bound",
                             torch.Tensor([float(scale_bound)]) if scale_bound is not None else None)
        self.tail_mass = float(tail_mass)
        self.lower_bound_scale = LowerBound(scale_bound)

    @staticmethod
    def _standardized_cumulative(inputs: Tensor) -> Tensor:
        half = float(0.5)
        const = float(-(2 ** -0.5))
        return half * torch.erfc(const * inputs)

    def _likelihood(self, inputs: Tensor, scales: Tensor, means: Optional[Tensor] = None) -> Tensor:
        half = float(0.5)
        values = inputs - means if means is not None else inputs
        scales = self.lower_bound_scale(scales)
        values = torch.abs(values)
        upper = self._standardized_cumulative((half - values) / scales)
        lower = self._standardized_cumulative((-half - values) / scales)
        return upper - lower

    def update_scale_table(self, scale_table, force=False):
        self.scale_table = torch.Tensor(tuple(float(s) for s in scale_table))
        return True

    def forward(self, inputs: Tensor, scales: Tensor, means: Optional[Tensor] = None,
                training: Optional[bool] = None):
        if training is None:
            training = self.training
        outputs = self.quantize(inputs, "noise" if training else "dequantize", means)
        likelihood = self._likelihood(outputs, scales, means)
        if self.use_likelihood_bound:
            likelihood = self.likelihood_lower_bound(likelihood)
        return outputs, likelihood


class CompressionModel(nn.Module):
    def __init__(self, entropy_bottleneck_channels=None, init_weights=None):
        super().__init__()
        if entropy_bottleneck_channels is not None:
            self.entropy_bottleneck = EntropyBottleneck(entropy_bottleneck_channels)

    def aux_loss(self) -> Tensor:
        return sum(m.loss() for m in self.modules() if isinstance(m, EntropyBottleneck))

    def update(self, scale_table=None, force=False):
        return False


# --------------------------------------------------------------------------------------------
# sys.modules installation (used only by tests/golden/make_golden.py)
# --------------------------------------------------------------------------------------------
def install_as_compressai() -> None:
    """Register this restatement as the ``compressai`` package surface the reference imports."""
    import sys

    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    pkg = mod("compressai")
    pkg.__path__ = []  # mark as package
    mod("compressai.entropy_models", EntropyBottleneck=EntropyBottleneck,
        GaussianConditional=GaussianConditional, EntropyModel=EntropyModel)
    mod("compressai.layers", GDN=GDN, conv1x1=conv1x1, conv3x3=conv3x3,
        ResidualBottleneckBlock=ResidualBottleneckBlock)
    models = mod("compressai.models", CompressionModel=CompressionModel)
    models.__path__ = []
    mod("compressai.models.base", CompressionModel=CompressionModel)
    mod("compressai.models.sensetime", ResidualBottleneckBlock=ResidualBottleneckBlock)
    mod("compressai.models.utils", conv=conv, deconv=deconv,
        update_registered_buffers=update_registered_buffers)
    mod("compressai.ops", quantize_ste=quantize_ste, LowerBound=LowerBound,
        NonNegativeParametrizer=NonNegativeParametrizer)
