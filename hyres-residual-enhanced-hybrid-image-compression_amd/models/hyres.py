"""ResidualJPEGCompression (models/hyres.py:9-181) — the drop-in boundary of this build.

forward(x [B,3,H,W] in [0,1], noisequant=False) -> {'x_hat', 'likelihoods': {'y','z'}, 'jpeg_bpp_loss',
'jpeg_decoded', 'residual', 'residual_hat'} exactly as the reference (:70-77).  The JPEG base layer stays
a host stage (libjpeg-turbo); everything after the host->device copy — residual, LightWeightCheckerboard,
x_hat_initial, MultiScaleRefine, clamp — is ONE HIP tape (forward and backward on MI355X).

Fixed reference bugs (documented in DESIGN.md):
  * load_state_dict kept the ``refine.`` prefix and strict-loaded into ``self.refine`` (:150-163), so the
    model could not reload its own state_dict; here prefixes are stripped per sub-module;
  * the dead ``x.device == 'cuda'`` check (:39) is replaced by a real device test.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from hyres_hip import ops as O
from hyres_hip import refine_ops as R
from hyres_hip import runtime
from hyres_hip.layers import CompressionModel

from .checkerboard import LightWeightCheckerboard
from .layers.enhancement import MultiScaleRefine
from .utils.turbo_jpeg_compression import TurboJPEGCompression


class ResidualJPEGCompression(CompressionModel):
    def __init__(self, base_model=None, jpeg_quality=1, se_reduction=1, **kwargs):
        super().__init__()
        self.jpeg = TurboJPEGCompression(quality=jpeg_quality)
        self.residual_model = base_model if base_model is not None else LightWeightCheckerboard(**kwargs)
        self.refine = MultiScaleRefine(in_channels=3, mid_channels=64)

    # ------------------------------------------------------------------ HIP graph (device part)
    def hip(self, tape, x: O.Node, jpeg: O.Node, training: bool, noisequant: bool):
        residual = R.add(tape, x, jpeg, alpha=-1.0)                       # hyres.py:48
        residual_hat, y_lik, z_lik = self.residual_model.hip(tape, residual, training, noisequant)
        x0 = R.add(tape, jpeg, residual_hat)                              # hyres.py:62
        O.GradReady.mark(tape, "refine")  # backward: refine's gradients complete past this point
        with O.f16_region():  # fp16 activations under autocast inference (configs[4])
            refined = self.refine.hip(tape, x0)                           # hyres.py:65
        x_hat = R.add_clamp01(tape, x0, refined)                          # hyres.py:66-67
        O.Trace.add("x_hat_initial", x0)
        O.Trace.add("x_hat", x_hat)
        return x_hat, y_lik, z_lik, residual, residual_hat

    def forward_device(self, x: torch.Tensor, jpeg_decoded: torch.Tensor, jpeg_bpp=0.0,
                       noisequant: bool = False):
        """Device-only forward with the JPEG stage's outputs supplied (both on the GPU); ``jpeg_bpp`` is a
        float or a 0-dim device tensor (graph capture: hyres_hip.graphs.CapturedStep)."""
        training = self.training
        rm = self.residual_model

        def build(tape, tensors):
            xt, jt = tensors
            xn = O.to_nhwc(xt, rg=False)
            jn = O.to_nhwc(jt, rg=False)
            outs = self.hip(tape, xn, jn, training, noisequant)
            return [xn, jn], list(outs)

        x_hat, y_lik, z_lik, residual, residual_hat = runtime.run(build, [x, jpeg_decoded],
                                                                  list(self.parameters()))
        return {
            "x_hat": x_hat,
            "likelihoods": {"y": y_lik, "z": z_lik},
            "jpeg_bpp_loss": (jpeg_bpp if isinstance(jpeg_bpp, torch.Tensor)
                              else torch.tensor(jpeg_bpp, device=x.device)),
            "jpeg_decoded": jpeg_decoded,
            "residual": residual,
            "residual_hat": residual_hat,
        }

    def forward(self, x, noisequant=False, jpeg: Optional[Tuple[torch.Tensor, float]] = None):
        """models/hyres.py:23-77.  ``jpeg=(decoded, bpp)`` skips the host JPEG stage (precomputed)."""
        device = next(self.parameters()).device
        if jpeg is None:
            x_cpu = x.detach().cpu() if x.device.type != "cpu" else x
            jpeg_decoded_cpu, jpeg_bpp = self.jpeg(x_cpu)
            jpeg_decoded = jpeg_decoded_cpu.to(device, non_blocking=False)
        else:
            jpeg_decoded, jpeg_bpp = jpeg
            jpeg_decoded = jpeg_decoded.to(device)
        x_dev = x.to(device)
        return self.forward_device(x_dev, jpeg_decoded, float(jpeg_bpp), noisequant)

    @torch.no_grad()
    def compress(self, x):
        """models/hyres.py:78-98: JPEG buffers (host) + the residual model's rANS strings."""
        device = next(self.parameters()).device
        x_cpu = x.detach().cpu() if x.device.type != "cpu" else x
        jpeg_buffers = self.jpeg.compress(x_cpu)
        jpeg_decoded = self.jpeg.decompress(jpeg_buffers, device)
        residual = x.to(device) - jpeg_decoded
        residual_compressed = self.residual_model.compress(residual)
        residual_compressed["jpeg_buffers"] = jpeg_buffers
        return residual_compressed

    @torch.no_grad()
    def decompress(self, compressed_data):
        """models/hyres.py:100-131: JPEG decode + residual decode (clamped to [0, 1] by the reference's
        LightWeightCheckerboard.decompress) + MultiScaleRefine + clamp."""
        device = next(self.parameters()).device
        jpeg_decoded = self.jpeg.decompress(compressed_data["jpeg_buffers"], device)
        decompress_result = self.residual_model.decompress(compressed_data["strings"], compressed_data["shape"])
        x_hat_initial = jpeg_decoded + decompress_result["x_hat"]
        with O.f16_region():  # fp16 activations under autocast (configs[4])
            refined = self.refine(x_hat_initial)
        decompress_result["x_hat"] = torch.clamp(x_hat_initial + refined, 0, 1)
        return decompress_result

    def load_state_dict(self, state_dict, strict: bool = True, **kwargs):
        """models/hyres.py:136-167 with the refine-prefix bug fixed (keys are stripped per sub-module)."""
        rm, rf, rest = {}, {}, {}
        for k, v in state_dict.items():
            if k.startswith("residual_model."):
                rm[k[len("residual_model."):]] = v
            elif k.startswith("refine."):
                rf[k[len("refine."):]] = v
            elif k.startswith("se_block."):
                rf[k] = v
            else:
                rest[k] = v
        if rm:
            self.residual_model.load_state_dict(rm, strict=strict)
        if rf:
            torch.nn.Module.load_state_dict(self.refine, rf, strict=strict)
        if rest and strict:
            raise RuntimeError(f"Unexpected key(s) in state_dict: {sorted(rest)[:5]}")
        O.bump_weight_epoch()

    @classmethod
    def from_state_dict(cls, state_dict, jpeg_quality=None):
        kwargs = {}
        if jpeg_quality is not None:
            kwargs["jpeg_quality"] = jpeg_quality
        net = cls(**kwargs)
        net.load_state_dict(state_dict)
        return net

    def update(self, scale_table=None, force=False, **kwargs):
        return self.residual_model.update(scale_table=scale_table, force=force, **kwargs)
