"""MultiScaleRefine post-filter (models/layers/enhancement.py:7-112) on HIP.

Data flow (NHWC, one HBM buffer ``multi`` [B,H,W,3*mid] replaces torch.cat):
  feat = SE(PReLU(conv_in(x)))
  multi[..., 0:mid]      = scale1(feat)                                  (last conv writes the slice)
  multi[..., mid:2mid]   = up(scale2(down2(feat)))                       (bilinear up writes the slice)
  multi[..., 2mid:3mid]  = up(scale3(down4(feat)))
  out = fusion(multi * sigmoid(conv7x7([mean_c, max_c](multi))))
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from hyres_hip import _lib as L
from hyres_hip import refine_ops as R
from hyres_hip.layers import Conv2d, HipModule, PReLU, ReLU, Sequential
from hyres_hip import ops as O
from hyres_hip.ops import Node

# SpatialAttention's multiply folded into fusion[0]'s epilogue (HYRES_EPI_ROWSCALE): inference, and training with
# fp32 activations (refine_ops.sa_fold_fusion); tests flip it, HYRES_FOLD_SA_MUL=0 turns it off (A/B)
FOLD_SA_MUL = os.environ.get("HYRES_FOLD_SA_MUL", "1") == "1"

__all__ = ["SpatialAttention", "SEBlock", "dilated_conv", "MultiScaleRefine"]


class SpatialAttention(HipModule):
    """CBAM spatial attention: sigmoid(conv7x7([mean_c(x), max_c(x)])) (enhancement.py:7-21)."""

    def __init__(self, kernel_size: int = 7):
        super().__init__()
        if kernel_size != 7:
            raise NotImplementedError("HIP spatial attention is specialised for kernel_size=7")
        padding = (kernel_size - 1) // 2
        self.conv = Conv2d(2, 1, kernel_size, padding=padding, bias=False)
        self.sigmoid = nn.Sigmoid()

    def hip_mul(self, tape, x: Node) -> Node:
        """x * SpatialAttention(x) fused (how MultiScaleRefine uses it, enhancement.py:105-106)."""
        return R.spatial_attention_mul(tape, x, self.conv.weight)

    def hip(self, tape, x: Node) -> Node:
        # standalone forward returns the attention map [B,H,W,1] (forward only)
        assert tape is None, "standalone SpatialAttention is forward-only; use hip_mul inside MultiScaleRefine"
        import hyres_hip.ops as O
        B, H, W, C = x.B, x.H, x.W, x.C
        pooled2 = O._empty((B, H, W, 2), x.device)
        argmax = torch.empty((B, H, W), dtype=torch.int32, device=x.device)
        attn = Node.new(B, H, W, 1, x.device)
        y = O._empty((B, H, W, C), x.device)
        L.call("hyres_spatial_attn_fwd", x.ptr(), self.conv.weight.data_ptr(), pooled2.data_ptr(), argmax.data_ptr(),
               attn.ptr(), y.data_ptr(), B, H, W, C, L.stream())
        return attn


class SEBlock(HipModule):
    """Squeeze-and-excitation (enhancement.py:25-40)."""

    def __init__(self, channel, reduction=16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Sequential(
            nn.Linear(channel, channel // reduction, bias=False),
            ReLU(inplace=True),
            nn.Linear(channel // reduction, channel, bias=False),
            nn.Sigmoid(),
        )

    def hip(self, tape, x: Node) -> Node:
        return R.se_block(tape, x, self.fc[0].weight, self.fc[2].weight)


def dilated_conv(ch_in, ch_out, dilation):
    """enhancement.py:44-51."""
    return Conv2d(ch_in, ch_out, kernel_size=3, padding=dilation, dilation=dilation, bias=True)


class MultiScaleRefine(HipModule):
    def __init__(self, in_channels=3, mid_channels=64):
        super().__init__()
        self.mid = mid_channels
        self.conv_in = Conv2d(in_channels, mid_channels, kernel_size=3, padding=1)
        self.act_in = PReLU()
        self.se_block = SEBlock(mid_channels, reduction=16)

        def make_block():
            return Sequential(
                dilated_conv(mid_channels, mid_channels, dilation=1),
                PReLU(),
                dilated_conv(mid_channels, mid_channels, dilation=2),
                PReLU(),
            )

        self.scale1 = make_block()
        self.scale2 = make_block()
        self.scale3 = make_block()
        self.spatial_att = SpatialAttention(kernel_size=7)
        self.fusion = Sequential(
            Conv2d(mid_channels * 3, mid_channels, kernel_size=1),
            PReLU(),
            Conv2d(mid_channels, in_channels, kernel_size=3, padding=1),
        )

    def hip(self, tape, x: Node) -> Node:
        mid = self.mid
        feat = self.conv_in.hip(tape, x, act=L.ACT_PRELU, slope=self.act_in.weight)
        feat = self.se_block.hip(tape, feat)
        B, H, W = feat.B, feat.H, feat.W
        assert H % 4 == 0 and W % 4 == 0, "MultiScaleRefine needs H, W divisible by 4"
        multi = Node.new(B, H, W, 3 * mid, feat.device, dtype=feat.v.dtype)  # fp16 under autocast inference

        def scale1(tape, f):  # scale 1 (orig), written into multi[..., 0:mid]
            self.scale1.hip(tape, f, out=multi.slice(0, mid))
            return None

        def scale2(tape, f):  # 1/2: F.interpolate(scale_factor=0.5) -> source scale 2.0; back with size=
            f2 = R.bilinear(tape, f, H // 2, W // 2, 2.0, 2.0)
            O.Trace.add("refine_f2_in", f2)
            f2 = self.scale2.hip(tape, f2)
            R.bilinear(tape, f2, H, W, (H // 2) / H, (W // 2) / W, out=multi.slice(mid, 2 * mid))
            return f2

        def scale3(tape, f):  # 1/4
            f3 = R.bilinear(tape, f, H // 4, W // 4, 4.0, 4.0)
            f3 = self.scale3.hip(tape, f3)
            R.bilinear(tape, f3, H, W, (H // 4) / H, (W // 4) / W, out=multi.slice(2 * mid, 3 * mid))
            return f3

        # the three scales are independent: three HIP streams, disjoint channel slices of ``multi``
        _, f2, f3 = O.run_branches(tape, feat, [scale1, scale2, scale3])
        from hyres_hip.ops import Trace
        if tape is None and FOLD_SA_MUL:
            # inference: multi * attn is never materialised — fusion[0] is a 1x1 conv, so
            # conv(multi * attn) = attn * conv_nobias(multi) + bias, formed in its epilogue (HYRES_EPI_ROWSCALE)
            attn = R.spatial_attention_map(multi, self.spatial_att.conv.weight)
            f0, f1, f2c = self.fusion[0], self.fusion[1], self.fusion[2]
            h = O.conv2d(None, multi, f0.weight, f0.bias, act=L.ACT_PRELU, slope=f1.weight, rowscale=attn)
            out = f2c.hip(None, h)
            m = None
        elif FOLD_SA_MUL and ((not multi.half and not O.f16_convs())
                              or R.sa_fold_amp_ok(tape, multi, self.fusion[0].weight.shape[0])):
            # training (fp32 activations; round 6: also AMP with fp16 activations and gradients): the same fold, with
            # its backward (refine_ops.sa_fold_fusion)
            f0, f1, f2c = self.fusion[0], self.fusion[1], self.fusion[2]
            h = R.sa_fold_fusion(tape, multi, self.spatial_att.conv.weight, f0.weight, f0.bias, f1.weight)
            out = f2c.hip(tape, h)
            m = None
        else:
            m = self.spatial_att.hip_mul(tape, multi)
            out = self.fusion.hip(tape, m)
        for name, n in (("refine_feat", feat), ("refine_f2", f2), ("refine_f3", f3), ("refine_multi", multi),
                        ("refine_multi_att", m), ("refined", out)):
            if n is not None:
                Trace.add(name, n)
        return out
