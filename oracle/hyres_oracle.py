"""TEST INFRASTRUCTURE ONLY — CPU fp32 restatement of the HyRES hot path (the parity oracle).

Nothing in the shipped product imports this file: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg use it, and only as the checker / the CPU baseline.

It is a *functional* restatement of the reference forward pass on a flat ``state_dict`` (the exact
key layout of the reference's ``ResidualJPEGCompression.state_dict()``), written against plain
``torch`` CPU ops in fp32, with every intermediate exposed so each HIP kernel can be checked
stage-wise on the oracle's exact inputs (SURVEY.md §7 "Rounding-boundary flips").

Reference anchors (paths relative to /root/reference):
  * ``ResidualJPEGCompression.forward``      models/hyres.py:23-77
  * ``LightWeightCheckerboard.forward``      models/checkerboard.py:90-147
  * ``AttentionBlock`` / ``ResidualUnit``     models/layers/attention.py:7-47
  * ``CheckboardMaskedConv2d``                models/layers/checkerboard.py:26-50
  * ``MultiScaleRefine`` / SE / SpatialAttn  models/layers/enhancement.py:7-112
  * ``Quantizer``                             models/utils/quantization.py:5-14
  * ``RateDistortionLoss``                    src/losses/rd_loss.py:18-44
  * compressai 1.2.6 pieces                   oracle/compressai_restated.py

Parity pinning: the fixtures under ``tests/golden/`` are produced by running the reference's OWN
model files (imported from /root/reference with ``oracle/compressai_restated.py`` installed as the
``compressai`` package); ``tests/test_oracle_golden.py`` checks this restatement against them.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F
from torch import Tensor

from .compressai_restated import LowerBoundFunction

PEDESTAL = 2.0 ** -36
BETA_BOUND = (1e-6 + PEDESTAL) ** 0.5
GAMMA_BOUND = (0.0 + PEDESTAL) ** 0.5
SCALE_BOUND = 0.11
LIKELIHOOD_BOUND = 1e-9


def _lb(x: Tensor, bound: float) -> Tensor:
    return LowerBoundFunction.apply(x, torch.tensor([bound], dtype=x.dtype))


class Oracle:
    """Functional oracle over a state dict ``sd`` (keys as ResidualJPEGCompression.state_dict())."""

    def __init__(self, sd: Dict[str, Tensor], prefix: str = "residual_model."):
        self.sd = sd
        self.rp = prefix

    def p(self, key: str) -> Tensor:
        return self.sd[key]

    # ---------------------------------------------------------------- primitives
    def conv(self, x, key, stride=1, padding=0, dilation=1, bias=True):
        w = self.p(key + ".weight")
        b = self.p(key + ".bias") if bias else None
        return F.conv2d(x, w, b, stride=stride, padding=padding, dilation=dilation)

    def deconv(self, x, key):
        # compressai deconv: ConvTranspose2d(k5, s2, p2, output_padding=1)
        return F.conv_transpose2d(x, self.p(key + ".weight"), self.p(key + ".bias"),
                                  stride=2, padding=2, output_padding=1)

    def gdn(self, x, key, inverse):
        """compressai GDN (oracle/compressai_restated.py GDN.forward)."""
        C = x.shape[1]
        beta = _lb(self.p(key + ".beta"), BETA_BOUND) ** 2 - PEDESTAL
        gamma = (_lb(self.p(key + ".gamma"), GAMMA_BOUND) ** 2 - PEDESTAL).reshape(C, C, 1, 1)
        norm = F.conv2d(x ** 2, gamma, beta)
        norm = torch.sqrt(norm) if inverse else torch.rsqrt(norm)
        return x * norm

    def rbb(self, x, key):
        """compressai ResidualBottleneckBlock(N, N): 1x1 -> ReLU -> 3x3 -> ReLU -> 1x1, + x."""
        out = self.relu(self.conv(x, key + ".conv1"))
        out = self.relu(self.conv(out, key + ".conv2", padding=1))
        out = self.conv(out, key + ".conv3")
        return out + x

    def res_unit(self, x, key):
        """models/layers/attention.py:18-30."""
        out = self.relu(self.conv(x, key + ".conv.0"))
        out = self.relu(self.conv(out, key + ".conv.2", padding=1))
        out = self.conv(out, key + ".conv.4")
        out = out + x
        return self.relu(out)

    def attention(self, x, key):
        """models/layers/attention.py:41-47: out = a*sigmoid(b) + x."""
        a = x
        for i in range(3):
            a = self.res_unit(a, f"{key}.conv_a.{i}")
        b = x
        for i in range(3):
            b = self.res_unit(b, f"{key}.conv_b.{i}")
        b = self.conv(b, f"{key}.conv_b.3")
        return a * torch.sigmoid(b) + x

    # ---------------------------------------------------------------- transforms
    def g_a(self, x):
        """models/checkerboard.py:35-45."""
        k = self.rp + "g_a."
        x = self.conv(x, k + "0", stride=2, padding=2)
        x = self.gdn(x, k + "1", inverse=False)
        x = self.rbb(x, k + "2")
        x = self.attention(x, k + "3")
        x = self.conv(x, k + "4", stride=2, padding=2)
        x = self.gdn(x, k + "5", inverse=False)
        x = self.rbb(x, k + "6")
        x = self.conv(x, k + "7", stride=2, padding=2)
        x = self.attention(x, k + "8")
        return x

    def g_s(self, x):
        """models/checkerboard.py:48-58."""
        k = self.rp + "g_s."
        x = self.attention(x, k + "0")
        x = self.deconv(x, k + "1")
        x = self.rbb(x, k + "2")
        x = self.gdn(x, k + "3", inverse=True)
        x = self.deconv(x, k + "4")
        x = self.attention(x, k + "5")
        x = self.rbb(x, k + "6")
        x = self.gdn(x, k + "7", inverse=True)
        x = self.deconv(x, k + "8")
        return x

    def h_a(self, y):
        """models/checkerboard.py:61-67."""
        k = self.rp + "h_a."
        z = self.relu(self.conv(y, k + "0", padding=1))
        z = self.relu(self.conv(z, k + "2", stride=2, padding=2))
        return self.conv(z, k + "4", stride=2, padding=2)

    def h_s(self, z_hat):
        """models/checkerboard.py:69-75."""
        k = self.rp + "h_s."
        t = self.relu(self.deconv(z_hat, k + "0"))
        t = self.relu(self.deconv(t, k + "2"))
        return self.conv(t, k + "4", padding=1)

    def param_aggregation(self, t):
        """models/checkerboard.py:82-88 (three 1x1 convs 768->640->512->384)."""
        k = self.rp + "param_aggregation."
        t = self.relu(self.conv(t, k + "0"))
        t = self.relu(self.conv(t, k + "2"))
        return self.conv(t, k + "4")

    def context_prediction(self, y_anchor_hat):
        """models/layers/checkerboard.py:46-49: W *= mask (in place) then dense 5x5 conv, pad 2."""
        k = self.rp + "context_prediction."
        w = self.p(k + "weight")
        with torch.no_grad():  # ``weight.data *= mask``: in-place, outside autograd -> dense weight grad
            w.mul_(self.p(k + "mask"))
        return F.conv2d(y_anchor_hat, w, self.p(k + "bias"), padding=2)

    # ---------------------------------------------------------------- entropy models
    def eb_logits_cumulative(self, v, stop_gradient=False):
        """compressai EntropyBottleneck._logits_cumulative on values shaped [C, 1, L]."""
        k = self.rp + "entropy_bottleneck."
        logits = v
        for i in range(5):
            m = self.p(f"{k}_matrix{i}")
            b = self.p(f"{k}_bias{i}")
            if stop_gradient:
                m, b = m.detach(), b.detach()
            logits = torch.matmul(F.softplus(m), logits)
            logits = logits + b
            if i < 4:
                f = self.p(f"{k}_factor{i}")
                if stop_gradient:
                    f = f.detach()
                logits = logits + torch.tanh(f) * torch.tanh(logits)
        return logits

    def eb_medians(self):
        return self.p(self.rp + "entropy_bottleneck.quantiles")[:, :, 1:2]

    def entropy_bottleneck(self, z, training: bool, noise: Optional[Tensor] = None):
        """compressai EntropyBottleneck.forward; ``noise`` is NCHW-shaped U(-.5,.5) when training."""
        C = z.shape[1]
        zt = z.permute(1, 0, 2, 3).contiguous()
        shape = zt.shape
        values = zt.reshape(C, 1, -1)
        if training:
            nz = noise.permute(1, 0, 2, 3).reshape(C, 1, -1)
            outputs = values + nz
        else:
            med = self.eb_medians()
            outputs = torch.round(values - med) + med
        lower = self.eb_logits_cumulative(outputs - 0.5)
        upper = self.eb_logits_cumulative(outputs + 0.5)
        lik = torch.sigmoid(upper) - torch.sigmoid(lower)
        lik = _lb(lik, LIKELIHOOD_BOUND)
        outputs = outputs.reshape(shape).permute(1, 0, 2, 3).contiguous()
        lik = lik.reshape(shape).permute(1, 0, 2, 3).contiguous()
        return outputs, lik

    def eb_aux_loss(self):
        """compressai EntropyBottleneck.loss: sum |logits(quantiles) - target| (stop-grad MLP)."""
        k = self.rp + "entropy_bottleneck."
        logits = self.eb_logits_cumulative(self.p(k + "quantiles"), stop_gradient=True)
        return torch.abs(logits - self.p(k + "target")).sum()

    @staticmethod
    def gaussian_likelihood(values_hat, scales, means):
        """compressai GaussianConditional._likelihood + likelihood LowerBound."""
        half = 0.5
        const = float(-(2 ** -0.5))
        values = torch.abs(values_hat - means)
        scales = _lb(scales, SCALE_BOUND)
        upper = 0.5 * torch.erfc(const * ((half - values) / scales))
        lower = 0.5 * torch.erfc(const * ((-half - values) / scales))
        return _lb(upper - lower, LIKELIHOOD_BOUND)

    # ---------------------------------------------------------------- quantizer
    @staticmethod
    def ste(t):
        """models/utils/quantization.py:11-12: round(t) - t.detach() + t (op order kept)."""
        return torch.round(t) - t.detach() + t

    def quant_ste(self, v, m, key):
        """``Quantizer.quantize(v - m, "ste") + m`` / ``quantize_ste(v - m) + m``; ``key`` names the decision
        site ("z", "y_anchor", "y_non_anchor") so a test can make the round() follow another run's choice
        at a half-integer tie."""
        return self.ste(v - m) + m

    @staticmethod
    def anchor_mask(h, w):
        """models/checkerboard.py:109-110: anchor = (h+w) even."""
        i = torch.arange(h).view(h, 1)
        j = torch.arange(w).view(1, w)
        return ((i + j) % 2 == 0)

    # ---------------------------------------------------------------- codec forward
    def codec_forward(self, x, training=False, noisequant=False, noise=None, trace=None):
        """models/checkerboard.py:90-147. ``noise`` keys: z, y_anchor, y_non_anchor, y (NCHW)."""
        T = trace if trace is not None else {}
        y = self.g_a(x)
        T["y"] = y
        z = self.h_a(y)
        T["z"] = z
        z_hat, z_lik = self.entropy_bottleneck(z, training, noise["z"] if training else None)
        if not noisequant:
            med = self.eb_medians().reshape(1, -1, 1, 1)
            z_hat = self.quant_ste(z, med, "z")  # quantize_ste(z - m) + m, checkerboard.py:98-101
        T["z_hat"] = z_hat
        T["z_likelihoods"] = z_lik
        latent = self.h_s(z_hat)
        T["latent_params"] = latent
        H, W = y.shape[-2:]
        am = self.anchor_mask(H, W).to(y.dtype)
        y_anchor = y * am
        y_non_anchor = y * (1 - am)
        anchor_params = self.param_aggregation(torch.cat([latent, torch.zeros_like(latent)], 1))
        s_a, m_a = anchor_params.chunk(2, 1)
        T["scales_anchor"], T["means_anchor"] = s_a, m_a
        if noisequant:
            y_anchor_hat = y_anchor + noise["y_anchor"]
        else:
            y_anchor_hat = self.quant_ste(y_anchor, m_a, "y_anchor")
        T["y_anchor_hat"] = y_anchor_hat
        ctx = self.context_prediction(y_anchor_hat)
        T["ctx_params"] = ctx
        na_params = self.param_aggregation(torch.cat([latent, ctx], 1))
        s_na, m_na = na_params.chunk(2, 1)
        T["scales_non_anchor"], T["means_non_anchor"] = s_na, m_na
        if noisequant:
            y_non_anchor_hat = y_non_anchor + noise["y_non_anchor"]
        else:
            y_non_anchor_hat = self.quant_ste(y_non_anchor, m_na, "y_non_anchor")
        T["y_non_anchor_hat"] = y_non_anchor_hat
        y_hat = y_anchor_hat + y_non_anchor_hat
        T["y_hat"] = y_hat
        x_hat = self.g_s(y_hat)
        scales = s_a + s_na
        means = m_a + m_na
        T["scales"], T["means"] = scales, means
        # GaussianConditional.forward(y, scales, means)
        if training:
            y_q = y + noise["y"]
        else:
            y_q = torch.round(y - means) + means
        T["y_q"] = y_q
        y_lik = self.gaussian_likelihood(y_q, scales, means)
        T["y_likelihoods"] = y_lik
        T["residual_hat"] = x_hat
        return {"x_hat": x_hat, "likelihoods": {"y": y_lik, "z": z_lik}}

    # ---------------------------------------------------------------- activations (kink hooks)
    # every ReLU / PReLU of the network goes through these two methods, so a test can detect inputs within
    # rounding distance of the kink and evaluate the other branch (tests/test_parity_gpu.py)
    @staticmethod
    def relu(x):
        return F.relu(x)

    @staticmethod
    def prelu(x, a):
        return F.prelu(x, a)

    # ---------------------------------------------------------------- MultiScaleRefine

    def refine(self, x, trace=None):
        """models/layers/enhancement.py:85-112."""
        T = trace if trace is not None else {}
        k = "refine."
        feat = self.prelu(self.conv(x, k + "conv_in", padding=1), self.p(k + "act_in.weight"))
        T["refine_feat0"] = feat
        # SEBlock (enhancement.py:25-40)
        b, c = feat.shape[:2]
        s = feat.mean(dim=(2, 3))
        s = F.relu(F.linear(s, self.p(k + "se_block.fc.0.weight")))
        s = torch.sigmoid(F.linear(s, self.p(k + "se_block.fc.2.weight")))
        feat = feat * s.view(b, c, 1, 1)
        T["refine_feat"] = feat

        def block(t, name):
            t = self.prelu(self.conv(t, f"{k}{name}.0", padding=1), self.p(f"{k}{name}.1.weight"))
            t = self.prelu(self.conv(t, f"{k}{name}.2", padding=2, dilation=2),
                           self.p(f"{k}{name}.3.weight"))
            return t

        f1 = block(feat, "scale1")
        f2 = F.interpolate(feat, scale_factor=0.5, mode="bilinear", align_corners=False)
        f2 = block(f2, "scale2")
        T["refine_f2"] = f2
        f2 = F.interpolate(f2, size=feat.shape[2:], mode="bilinear", align_corners=False)
        f3 = F.interpolate(feat, scale_factor=0.25, mode="bilinear", align_corners=False)
        f3 = block(f3, "scale3")
        T["refine_f3"] = f3
        f3 = F.interpolate(f3, size=feat.shape[2:], mode="bilinear", align_corners=False)
        multi = torch.cat([f1, f2, f3], 1)
        T["refine_multi"] = multi
        avg = multi.mean(dim=1, keepdim=True)
        mx, _ = multi.max(dim=1, keepdim=True)
        attn = torch.sigmoid(F.conv2d(torch.cat([avg, mx], 1), self.p(k + "spatial_att.conv.weight"),
                                      None, padding=3))
        T["refine_attn"] = attn
        multi = multi * attn
        T["refine_multi_att"] = multi
        out = self.prelu(self.conv(multi, k + "fusion.0"), self.p(k + "fusion.1.weight"))
        out = self.conv(out, k + "fusion.2", padding=1)
        T["refined"] = out
        return out

    # ---------------------------------------------------------------- full model
    def forward(self, x, jpeg_decoded, jpeg_bpp=0.0, training=False, noisequant=False, noise=None,
                trace=None):
        """models/hyres.py:23-77 with the JPEG stage's outputs supplied (host stage, out of scope)."""
        T = trace if trace is not None else {}
        residual = x - jpeg_decoded
        T["residual"] = residual
        res = self.codec_forward(residual, training, noisequant, noise, T)
        residual_hat = res["x_hat"]
        x0 = jpeg_decoded + residual_hat
        T["x_hat_initial"] = x0
        refined = self.refine(x0, T)
        x_hat = torch.clamp(x0 + refined, 0, 1)
        T["x_hat"] = x_hat
        for v in T.values():  # keep activation gradients for stage-wise parity diagnostics
            if torch.is_tensor(v) and v.requires_grad:
                v.retain_grad()
        return {"x_hat": x_hat, "likelihoods": res["likelihoods"],
                "jpeg_bpp_loss": torch.tensor(jpeg_bpp), "jpeg_decoded": jpeg_decoded,
                "residual": residual, "residual_hat": residual_hat}


def rd_loss(output, target, lmbda):
    """src/losses/rd_loss.py:18-44 with alpha = 0 (train.sh:14; VGG weights unavailable offline)."""
    N, _, H, W = target.shape
    num_pixels = N * H * W
    out = {}
    out["y_bpp_loss"] = torch.log(output["likelihoods"]["y"]).sum() / (-math.log(2) * num_pixels)
    out["z_bpp_loss"] = torch.log(output["likelihoods"]["z"]).sum() / (-math.log(2) * num_pixels)
    out["residual_bpp_loss"] = out["y_bpp_loss"] + out["z_bpp_loss"]
    out["bpp_loss"] = out["residual_bpp_loss"] + output["jpeg_bpp_loss"]
    out["mse_loss"] = F.mse_loss(output["x_hat"], target) * 255 ** 2
    out["loss"] = lmbda * out["mse_loss"] + out["bpp_loss"]
    return out


def vgg_loss(features_sd, x, y, layer_ids=(2, 7, 14, 21, 28)):
    """src/losses/vgg16.py:41-61 (VGGLoss.forward) on torchvision vgg16().features weights
    ``features_sd`` ({"N.weight", "N.bias"}): Normalize(ImageNet mean/std) both inputs, then for each slice
    [previous id + 1 .. id] the convs (3x3, pad 1) / ReLU / MaxPool2d(2, 2) of VGG16, and the sum over slices
    of mean |f(x) - f(y)|."""
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
    layers = []
    for v in cfg:
        layers += ["M"] if v == "M" else ["C", "R"]
    mean = torch.tensor([0.485, 0.456, 0.406], dtype=x.dtype).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], dtype=x.dtype).view(1, 3, 1, 1)
    x = (x - mean) / std
    y = (y - mean) / std
    loss = 0
    start = 0
    for lid in layer_ids:
        for i in range(start, lid + 1):
            kind = layers[i]
            if kind == "C":
                w, b = features_sd[f"{i}.weight"].to(x.dtype), features_sd[f"{i}.bias"].to(x.dtype)
                x, y = F.conv2d(x, w, b, padding=1), F.conv2d(y, w, b, padding=1)
            elif kind == "R":
                x, y = F.relu(x), F.relu(y)
            else:
                x, y = F.max_pool2d(x, 2, 2), F.max_pool2d(y, 2, 2)
        start = lid + 1
        loss = loss + torch.abs(x - y).mean()
    return loss
