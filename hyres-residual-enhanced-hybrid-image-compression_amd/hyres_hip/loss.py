"""RateDistortionLoss (src/losses/rd_loss.py:18-44) with HIP reductions.

The bpp log-sums and the MSE are deterministic two-pass block reductions; the six scalars are
finalised on device (no host sync).  The VGG16 perceptual term (rd_loss.py:40, alpha * vgg * 255^2) runs
on the HIP path (hyres_hip.vgg.VGGLoss) when alpha != 0; its ImageNet weights must be available locally
(HYRES_VGG16_WEIGHTS).  With alpha = 0 (train.sh:14) it is not evaluated — the reference computes it and
multiplies it by zero."""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib as L
from .ops import _empty, _ws


def _sum_into(name, args, n, out_ptr, device, slot):
    ws = _ws(L.load().hyres_reduce_workspace_bytes(n), device, slot=slot)
    L.call(name, *args, n, out_ptr, ws.data_ptr(), ws.numel(), L.stream())


class _RDLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lik_y, lik_z, x_hat, target, jpeg_bpp, lmbda):
        dev = x_hat.device
        lik_y = lik_y.contiguous()
        lik_z = lik_z.contiguous()
        x_hat = x_hat.contiguous()
        target = target.contiguous()
        sums = _empty((3,), dev)
        _sum_into("hyres_sum_log", (lik_y.data_ptr(),), lik_y.numel(), sums.data_ptr(), dev, 4)
        _sum_into("hyres_sum_log", (lik_z.data_ptr(),), lik_z.numel(), sums.data_ptr() + 4, dev, 4)
        _sum_into("hyres_sum_sqdiff", (x_hat.data_ptr(), target.data_ptr()), x_hat.numel(), sums.data_ptr() + 8,
                  dev, 4)
        N, _, H, W = target.shape
        npx = N * H * W
        outs = [_empty((), dev) for _ in range(6)]
        jb = None
        if jpeg_bpp is not None:
            jb = jpeg_bpp.to(device=dev, dtype=torch.float32).reshape(1).contiguous()
        L.call("hyres_rd_finalize", sums.data_ptr(), L.ptr(jb), float(lmbda), npx, x_hat.numel(),
               L.ptr_array(outs), L.stream())
        ctx.save_for_backward(lik_y, lik_z, x_hat, target)
        ctx.lmbda = float(lmbda)
        ctx.npx = npx
        return tuple(outs)

    @staticmethod
    def backward(ctx, g0, g1, g2, g3, g4, g5):
        lik_y, lik_z, x_hat, target = ctx.saved_tensors
        dev = x_hat.device
        gs = [g.contiguous() for g in (g0, g1, g2, g3, g4, g5)]
        coef = _empty((3,), dev)
        L.call("hyres_rd_bwd_coef", *[g.data_ptr() for g in gs], ctx.lmbda, ctx.npx, x_hat.numel(),
               coef.data_ptr(), L.stream())
        gy = _empty(lik_y.shape, dev)
        gz = _empty(lik_z.shape, dev)
        gx = _empty(x_hat.shape, dev)
        L.call("hyres_scale_recip", lik_y.data_ptr(), coef.data_ptr(), 1.0, gy.data_ptr(), lik_y.numel(), L.stream())
        L.call("hyres_scale_recip", lik_z.data_ptr(), coef.data_ptr() + 4, 1.0, gz.data_ptr(), lik_z.numel(),
               L.stream())
        L.call("hyres_scale_diff", x_hat.data_ptr(), target.data_ptr(), coef.data_ptr() + 8, 1.0, gx.data_ptr(),
               x_hat.numel(), L.stream())
        return gy, gz, gx, None, None, None


class RateDistortionLoss(nn.Module):
    """Custom rate distortion loss with a Lagrangian parameter (src/losses/rd_loss.py)."""

    def __init__(self, lmbda=0.004, alpha=0.001, vgg=None):
        super().__init__()
        self.lmbda = lmbda
        self.alpha = alpha
        if alpha != 0 and vgg is None:
            from .vgg import VGGLoss
            vgg = VGGLoss()  # ImageNet weights from HYRES_VGG16_WEIGHTS (raises when absent)
        self.vgg = vgg

    def forward(self, output, target):
        lik = output["likelihoods"]
        loss, bpp, res, yb, zb, mse = _RDLossFn.apply(lik["y"], lik["z"], output["x_hat"], target,
                                                      output.get("jpeg_bpp_loss"), self.lmbda)
        if self.alpha != 0:
            vgg = self.vgg(output["x_hat"], target) * 255 ** 2  # rd_loss.py:40
            loss = loss + self.alpha * vgg                      # rd_loss.py:42
        else:
            vgg = torch.zeros((), device=target.device)
        return {"loss": loss, "bpp_loss": bpp, "residual_bpp_loss": res, "y_bpp_loss": yb, "z_bpp_loss": zb,
                "mse_loss": mse, "vgg_loss": vgg}
