"""VGG16 perceptual loss (src/losses/vgg16.py:7-61; rd_loss.py:40) on the HIP path — SURVEY §8f row f4.

Same module layout and state_dict keys as the reference's VGGLoss: ``slices`` is a ModuleList of the
torchvision ``vgg16().features`` pieces cut after layers [2, 7, 14, 21, 28], each piece keeping the
original child names (``slices.1.5.weight`` is features.5), so a reference VGGLoss state dict loads as is
and ``load_torchvision(state_dict)`` takes torchvision's ``features.N.*`` keys.

ImageNet weights cannot be downloaded here: ``VGGLoss()`` loads them from ``HYRES_VGG16_WEIGHTS`` or
torchvision's cache file (``~/.cache/torch/hub/checkpoints/vgg16-397923af.pth``) with
``torch.load(weights_only=True)``, and raises if neither exists (``pretrained=False`` builds it with
torchvision's init instead — the tests' parity checks run on such weights).

Forward: Normalize (x - mean) / std, then per slice the convs (implicit-GEMM HIP kernels; a ReLU inside a
slice is fused into its conv's epilogue, the ReLU that opens a slice is a separate pass because the
previous slice ends on the pre-activation), 2x2 max pools, and mean |f(x) - f(y)| summed over the slices.
The reference path (y = target) needs no gradient and runs without a tape; x (= x_hat) is taped and its
gradient flows back into the model through torch autograd.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn

from . import _lib as L
from . import ops as O
from .layers import Conv2d
from .ops import Node, _empty, _ws
from .runtime import run

VGG16_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
TORCHVISION_FILE = "vgg16-397923af.pth"


def vgg16_features() -> nn.Sequential:
    """torchvision.models.vgg16().features (31 children), HIP conv modules, torchvision's init."""
    layers, c = [], 3
    for v in VGG16_CFG:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            conv = Conv2d(c, v, kernel_size=3, padding=1)
            nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
            nn.init.constant_(conv.bias, 0)
            layers += [conv, nn.ReLU(inplace=True)]
            c = v
    return nn.Sequential(*layers)


def _default_weights_path() -> Optional[str]:
    p = os.environ.get("HYRES_VGG16_WEIGHTS")
    if p:
        return p
    hub = os.path.join(os.path.expanduser(os.environ.get("TORCH_HOME", "~/.cache/torch")), "hub", "checkpoints",
                       TORCHVISION_FILE)
    return hub if os.path.exists(hub) else None


class VGGLoss(nn.Module):
    """VGG-based perceptual loss (src/losses/vgg16.py:7-61)."""

    def __init__(self, layer_ids=None, pretrained: bool = True, weights_path: Optional[str] = None):
        super().__init__()
        if layer_ids is None:
            layer_ids = [2, 7, 14, 21, 28]
        vgg = vgg16_features()
        if pretrained:
            path = weights_path or _default_weights_path()
            if path is None or not os.path.exists(path):
                raise RuntimeError(
                    "VGGLoss needs torchvision's ImageNet VGG16 weights (the reference downloads them with "
                    "models.vgg16(pretrained=True)); no network here: set HYRES_VGG16_WEIGHTS to a local copy of "
                    f"{TORCHVISION_FILE}")
            load_torchvision(vgg, torch.load(path, map_location="cpu", weights_only=True))
        vgg.eval()
        for p in vgg.parameters():
            p.requires_grad = False
        self.slices = nn.ModuleList()
        start = 0
        for layer_id in layer_ids:
            self.slices.append(vgg[start:layer_id + 1])
            start = layer_id + 1
        self.layer_ids = list(layer_ids)

    # ------------------------------------------------------------------ HIP graph
    def _normalize(self, tape, x: Node) -> Node:
        mean = (torch.tensor(IMAGENET_MEAN, dtype=torch.float32)).numpy()
        std = (torch.tensor(IMAGENET_STD, dtype=torch.float32)).numpy()
        y = Node.new(x.B, x.H, x.W, x.C, x.device, rg=x.rg)
        assert x.contiguous
        L.call("hyres_normalize_fwd", x.ptr(), y.ptr(), x.P, x.C, mean.ctypes.data, std.ctypes.data, L.stream())
        if tape is not None and x.rg:
            def bwd():
                g = y.grad()
                if g is None:
                    return
                tgt, acc = x.grad_target()
                L.call("hyres_normalize_bwd", g.data_ptr(), tgt.data_ptr(), x.P, x.C, mean.ctypes.data, std.ctypes.data,
                       acc, L.stream())
            tape.push(bwd)
        return y

    @staticmethod
    def _relu(tape, x: Node) -> Node:
        y = Node.new(x.B, x.H, x.W, x.C, x.device, rg=x.rg)
        L.call("hyres_relu_fwd", x.ptr(), y.ptr(), x.P * x.C, L.stream())
        y.relu_out = True
        if tape is not None and x.rg:
            def bwd():
                g = y.grad()
                if g is None:
                    return
                tgt, acc = x.grad_target()
                if acc:
                    t = _empty(tuple(x.v.shape), x.device)
                    L.call("hyres_relu_bwd", y.ptr(), g.data_ptr(), t.data_ptr(), x.P * x.C, L.stream())
                    L.call("hyres_accumulate", t.data_ptr(), tgt.data_ptr(), t.numel(), L.stream())
                else:
                    L.call("hyres_relu_bwd", y.ptr(), g.data_ptr(), tgt.data_ptr(), x.P * x.C, L.stream())
            tape.push(bwd)
        return y

    @staticmethod
    def _pool(tape, x: Node) -> Node:
        y = Node.new(x.B, x.H // 2, x.W // 2, x.C, x.device, rg=x.rg)
        arg = torch.empty(y.P * y.C, dtype=torch.uint8, device=x.device)
        L.call("hyres_maxpool2_fwd", x.ptr(), y.ptr(), arg.data_ptr(), x.B, x.H, x.W, x.C, L.stream())
        if tape is not None and x.rg:
            def bwd():
                g = y.grad()
                if g is None:
                    return
                tgt, acc = x.grad_target()
                L.call("hyres_maxpool2_bwd", g.data_ptr(), arg.data_ptr(), tgt.data_ptr(), x.B, x.H, x.W, x.C, acc,
                       L.stream())
            tape.push(bwd)
        return y

    def _slice(self, tape, seq: nn.Sequential, x: Node) -> Node:
        mods = list(seq)
        i = 0
        while i < len(mods):
            m = mods[i]
            if isinstance(m, Conv2d):
                fuse = i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
                x = m.hip(tape, x, act=L.ACT_RELU if fuse else L.ACT_NONE)
                i += 2 if fuse else 1
            elif isinstance(m, nn.ReLU):
                x = self._relu(tape, x)
                i += 1
            elif isinstance(m, nn.MaxPool2d):
                x = self._pool(tape, x)
                i += 1
            else:
                raise TypeError(f"unexpected VGG layer {m}")
        return x

    def hip(self, tape, x: Node, y: Node) -> Node:
        """Perceptual loss as a [1,1,1,1] node; ``y`` (the target) is processed without the tape."""
        fx = self._normalize(tape, x)
        with torch.no_grad():
            fy = self._normalize(None, y)
        loss = Node.new(1, 1, 1, 1, x.device)
        for k, seq in enumerate(self.slices):
            fx = self._slice(tape, seq, fx)
            fy = self._slice(None, seq, fy)
            n = fx.P * fx.C
            ws = _ws(L.load().hyres_absdiff_workspace_bytes(n), x.device, slot=6)
            L.call("hyres_absdiff_mean", fx.ptr(), fy.ptr(), n, loss.ptr(), int(k > 0), ws.data_ptr(), ws.numel(),
                   L.stream())
            if tape is not None and x.rg:
                def bwd(fx=fx, fy=fy, n=n):
                    g = loss.grad()
                    if g is None:
                        return
                    tgt, acc = fx.grad_target()
                    L.call("hyres_absdiff_bwd", fx.ptr(), fy.ptr(), g.data_ptr(), n, tgt.data_ptr(), acc, L.stream())
                tape.push(bwd)
        return loss

    def forward(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """x: reconstruction [B,3,H,W] in [0,1] (gradient flows), y: original (no gradient)."""

        def build(tape, tensors):
            xt, yt = tensors
            xn = O.to_nhwc(xt, rg=xt.requires_grad)
            yn = O.to_nhwc(yt.detach(), rg=False)
            return [xn, None], [self.hip(tape, xn, yn)]

        (loss,) = run(build, [x, y], [])
        return loss.reshape(())


def load_torchvision(features: nn.Sequential, sd) -> None:
    """Load torchvision vgg16 weights: ``features.N.weight`` keys (the full model's state dict) or the
    features module's own ``N.weight`` keys."""
    own = {}
    for k, v in sd.items():
        if k.startswith("features."):
            own[k[len("features."):]] = v
        elif k[0].isdigit():
            own[k] = v
    torch.nn.Module.load_state_dict(features, own, strict=True)
    O.bump_weight_epoch()
