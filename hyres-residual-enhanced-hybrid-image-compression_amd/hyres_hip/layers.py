"""nn.Module layer set of the HyRES hot path with HIP forward/backward.

Every module keeps the reference's parameter/buffer names (state_dict keys identical to the
reference + compressai 1.2.6) and adds ``hip(tape, x: Node, ...) -> Node``, the
NHWC HIP implementation.  ``forward`` on NCHW tensors is provided for every module through
``runtime.module_forward`` (an autograd Function that runs the HIP tape), so each layer can be used —
and parity-tested — on its own exactly like its reference counterpart.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch
import torch.nn as nn
from torch import Tensor

from . import _lib as L
from . import entropy_ops as E
from . import ops as O
from .ops import Node, Tape


class HipModule(nn.Module):
    """Mixin: NCHW ``forward`` runs the module's ``hip`` through the tape Function."""

    def forward(self, x: Tensor) -> Tensor:  # noqa: D401
        from .runtime import module_forward
        return module_forward(self, x)


# --------------------------------------------------------------------------------------------------
# compressai-equivalent parametrisation helpers (buffers only; math is in the HIP kernels)
# --------------------------------------------------------------------------------------------------
class LowerBound(nn.Module):
    """compressai.ops.LowerBound: holds ``bound`` (the max() and its gradient rule run in HIP)."""

    def __init__(self, bound: float):
        super().__init__()
        self.register_buffer("bound", torch.Tensor([float(bound)]))


class NonNegativeParametrizer(nn.Module):
    """compressai.ops.NonNegativeParametrizer: out = LowerBound(x)^2 - pedestal (in HIP)."""

    def __init__(self, minimum: float = 0, reparam_offset: float = 2 ** -18):
        super().__init__()
        self.minimum = float(minimum)
        self.reparam_offset = float(reparam_offset)
        self.register_buffer("pedestal", torch.Tensor([self.reparam_offset ** 2]))
        self.lower_bound = LowerBound((self.minimum + self.reparam_offset ** 2) ** 0.5)

    def init(self, x: Tensor) -> Tensor:
        return torch.sqrt(torch.max(x + self.pedestal, self.pedestal))


# --------------------------------------------------------------------------------------------------
# convolutions
# --------------------------------------------------------------------------------------------------
class Conv2d(nn.Conv2d, HipModule):
    """nn.Conv2d with the HIP implicit-GEMM implementation (same parameters / init)."""

    def hip(self, tape: Optional[Tape], x: Node, act=L.ACT_NONE, slope=None, res=None, out=None) -> Node:
        assert self.groups == 1 and self.stride[0] == self.stride[1]
        return O.conv2d(tape, x, self.weight, self.bias, stride=self.stride[0], pad=self.padding[0],
                        dil=self.dilation[0], act=act, slope=slope, res=res, out=out)

    forward = HipModule.forward


class ConvTranspose2d(nn.ConvTranspose2d, HipModule):
    def hip(self, tape: Optional[Tape], x: Node, act=L.ACT_NONE, out=None) -> Node:
        assert self.stride == (2, 2) and self.output_padding == (1, 1) and self.padding[0] == self.kernel_size[0] // 2
        return O.deconv2d(tape, x, self.weight, self.bias, act=act, out=out)

    forward = HipModule.forward


def conv1x1(in_ch: int, out_ch: int, stride: int = 1) -> Conv2d:
    """models/layers/common.py:4-6."""
    return Conv2d(in_ch, out_ch, kernel_size=1, stride=stride)


def conv3x3(in_ch: int, out_ch: int, stride: int = 1) -> Conv2d:
    """models/layers/common.py:9-11."""
    return Conv2d(in_ch, out_ch, kernel_size=3, stride=stride, padding=1)


def conv(in_channels, out_channels, kernel_size=5, stride=2) -> Conv2d:
    """compressai.models.utils.conv."""
    return Conv2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride, padding=kernel_size // 2)


def deconv(in_channels, out_channels, kernel_size=5, stride=2) -> ConvTranspose2d:
    """compressai.models.utils.deconv."""
    return ConvTranspose2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                           output_padding=stride - 1, padding=kernel_size // 2)


class ReLU(nn.ReLU):
    """Fused into the producing conv's epilogue by ``run_sequential``."""


class PReLU(nn.PReLU):
    """nn.PReLU() (single shared slope); fused into the producing conv's epilogue."""


def _is_relu(m):
    return isinstance(m, nn.ReLU)


def run_sequential(tape: Optional[Tape], seq: nn.Sequential, x: Node, out: Optional[Node] = None) -> Node:
    """Run an nn.Sequential of HIP modules, fusing ReLU / PReLU into the preceding conv."""
    mods = list(seq)
    i = 0
    n = len(mods)
    while i < n:
        m = mods[i]
        last = i == n - 1
        nxt = mods[i + 1] if i + 1 < n else None
        if isinstance(m, (Conv2d, ConvTranspose2d)):
            act, slope, step = L.ACT_NONE, None, 1
            if isinstance(nxt, nn.PReLU):
                assert nxt.weight.numel() == 1
                act, slope, step = L.ACT_PRELU, nxt.weight, 2
            elif _is_relu(nxt):
                act, step = L.ACT_RELU, 2
            tail = i + step >= n
            o = out if tail else None
            if isinstance(m, Conv2d):
                x = m.hip(tape, x, act=act, slope=slope, out=o)
            else:
                assert act != L.ACT_PRELU
                x = m.hip(tape, x, act=act, out=o)
            i += step
        else:
            assert hasattr(m, "hip"), f"no HIP implementation for {type(m).__name__}"
            if last and out is not None:
                raise RuntimeError("run_sequential: out= needs a conv as the last module")
            x = m.hip(tape, x)
            i += 1
    return x


class Sequential(nn.Sequential, HipModule):
    def hip(self, tape: Optional[Tape], x: Node, out: Optional[Node] = None) -> Node:
        return run_sequential(tape, self, x, out)

    forward = HipModule.forward


# --------------------------------------------------------------------------------------------------
# compressai layers
# --------------------------------------------------------------------------------------------------
class GDN(HipModule):
    """compressai.layers.GDN(in_channels, inverse) — same parameters/buffers; HIP fused GEMM."""

    def __init__(self, in_channels: int, inverse: bool = False, beta_min: float = 1e-6, gamma_init: float = 0.1):
        super().__init__()
        if float(beta_min) != 1e-6:
            raise NotImplementedError("HIP GDN kernels hard-code compressai's beta_min=1e-6")
        self.inverse = bool(inverse)
        self.beta_reparam = NonNegativeParametrizer(minimum=float(beta_min))
        self.beta = nn.Parameter(self.beta_reparam.init(torch.ones(in_channels)))
        self.gamma_reparam = NonNegativeParametrizer()
        self.gamma = nn.Parameter(self.gamma_reparam.init(float(gamma_init) * torch.eye(in_channels)))

    def hip(self, tape: Optional[Tape], x: Node) -> Node:
        return O.gdn(tape, x, self.beta, self.gamma, self.inverse)


class ResidualBottleneckBlock(HipModule):
    """compressai ResidualBottleneckBlock(in_ch, out_ch): x + conv1x1(relu(conv3x3(relu(conv1x1(x)))))."""

    def __init__(self, in_ch: int, out_ch: int):
        super().__init__()
        mid_ch = min(in_ch, out_ch) // 2
        self.conv1 = conv1x1(in_ch, mid_ch)
        self.relu = ReLU(inplace=True)
        self.conv2 = conv3x3(mid_ch, mid_ch)
        self.conv3 = conv1x1(mid_ch, out_ch)
        if in_ch != out_ch:
            raise NotImplementedError("HyRES only uses ResidualBottleneckBlock(N, N)")
        self.skip = nn.Identity()

    def hip(self, tape: Optional[Tape], x: Node) -> Node:
        y = O.residual_unit_fused(tape, x, self.conv1, self.conv2, self.conv3, final_relu=False)
        if y is not None:  # autocast with fp16 activations: one launch (csrc/ru_fused.hip)
            return y
        t = self.conv1.hip(tape, x, act=L.ACT_RELU)
        t = self.conv2.hip(tape, t, act=L.ACT_RELU)
        return self.conv3.hip(tape, t, res=x)


# --------------------------------------------------------------------------------------------------
# entropy models
# --------------------------------------------------------------------------------------------------
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


class EntropyBottleneck(EntropyModel):
    """compressai EntropyBottleneck(channels) — identical parameters; likelihood + STE in HIP."""

    def __init__(self, channels: int, *args, tail_mass: float = 1e-9, init_scale: float = 10,
                 filters=(3, 3, 3, 3), **kwargs):
        super().__init__(*args, **kwargs)
        if tuple(filters) != (3, 3, 3, 3):
            raise NotImplementedError("HIP EntropyBottleneck kernels are specialised for filters (3,3,3,3)")
        self.channels = int(channels)
        self.filters = tuple(int(f) for f in filters)
        self.init_scale = float(init_scale)
        self.tail_mass = float(tail_mass)
        filters = (1,) + self.filters + (1,)
        scale = self.init_scale ** (1 / (len(self.filters) + 1))
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
        self.quantiles.data = torch.Tensor([-self.init_scale, 0, self.init_scale]).repeat(channels, 1, 1)
        target = np.log(2 / self.tail_mass - 1)
        self.register_buffer("target", torch.Tensor([-target, 0, target]))

    def _get_medians(self) -> Tensor:
        return self.quantiles[:, :, 1:2]

    def loss(self) -> Tensor:
        """Aux loss (HIP kernel): sum |logits(quantiles) - target|."""
        return E.eb_aux_loss(self)

    def hip(self, tape, z: Node, training: bool, noisequant: bool, noise: E.NoiseSource):
        return E.entropy_bottleneck(tape, self, z, training, noisequant, noise)

    def update(self, force: bool = False) -> bool:
        """compressai EntropyBottleneck.update: quantized CDF tables for rANS coding."""
        from . import entropy_coding as EC
        return EC.eb_update(self, force=force)


class GaussianConditional(EntropyModel):
    """compressai GaussianConditional(scale_table) — buffers only; the likelihood is fused into the
    checkerboard non-anchor kernel (hyres_ckbd_nonanchor_gc_fwd)."""

    def __init__(self, scale_table, *args, scale_bound: float = 0.11, tail_mass: float = 1e-9, **kwargs):
        super().__init__(*args, **kwargs)
        if float(scale_bound) != 0.11:
            raise NotImplementedError("HIP GaussianConditional kernels hard-code scale_bound=0.11")
        self.register_buffer("scale_table", torch.Tensor(tuple(float(s) for s in scale_table))
                             if scale_table else torch.Tensor())
        self.register_buffer("scale_bound", torch.Tensor([float(scale_bound)]))
        self.tail_mass = float(tail_mass)
        self.lower_bound_scale = LowerBound(scale_bound)

    def update_scale_table(self, scale_table, force: bool = False) -> bool:
        """compressai GaussianConditional.update_scale_table (+ update): CDF tables per scale."""
        if self._offset.numel() > 0 and not force:
            return False
        from . import entropy_coding as EC
        self.scale_table = torch.Tensor(tuple(float(s) for s in scale_table)).to(self.scale_bound.device)
        EC.gc_update(self)
        return True


class CompressionModel(nn.Module):
    """compressai.models.CompressionModel surface used by HyRES (aux_loss over all EBs)."""

    def __init__(self, entropy_bottleneck_channels=None, init_weights=None):
        super().__init__()
        if entropy_bottleneck_channels is not None:
            self.entropy_bottleneck = EntropyBottleneck(entropy_bottleneck_channels)

    def aux_loss(self) -> Tensor:
        losses = [m.loss() for m in self.modules() if isinstance(m, EntropyBottleneck)]
        out = losses[0]
        for l_ in losses[1:]:
            out = out + l_
        return out

    def update(self, scale_table=None, force=False):
        """compressai CompressionModel.update: CDF tables of every EntropyBottleneck and
        GaussianConditional (rANS coding for compress/decompress)."""
        from . import entropy_coding as EC
        if scale_table is None:
            scale_table = EC.get_scale_table()
        updated = False
        for _, module in self.named_modules():
            if isinstance(module, EntropyBottleneck):
                updated |= module.update(force=force)
            if isinstance(module, GaussianConditional):
                updated |= module.update_scale_table(scale_table, force=force)
        return updated
