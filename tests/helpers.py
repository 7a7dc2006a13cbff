"""Shared test helpers: recipe weights, golden fixtures, oracle construction."""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from conftest import GOLDEN


def load_npz(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: torch.from_numpy(z[k].copy()) for k in z.files}


def load_meta():
    with open(os.path.join(GOLDEN, "meta.json")) as f:
        return json.load(f)


def build_model(N=128, M=192, jpeg_quality=50):
    """The HIP model (constructible on CPU) with recipe weights loaded."""
    from models import ResidualJPEGCompression
    from hyres_hip.weights import synthetic_state_dict
    net = ResidualJPEGCompression(jpeg_quality=jpeg_quality, N=N, M=M)
    sd = synthetic_state_dict(net.state_dict())
    torch.nn.Module.load_state_dict(net, sd, strict=True)
    return net, sd


def recipe_state_dict():
    from models import ResidualJPEGCompression
    from hyres_hip.weights import synthetic_state_dict
    net = ResidualJPEGCompression(jpeg_quality=50)
    return synthetic_state_dict(net.state_dict())


def oracle_from(sd, requires_grad=False):
    from oracle import Oracle
    sd2 = {}
    for k, v in sd.items():
        t = v.detach().clone().float() if v.is_floating_point() else v.clone()
        if requires_grad and t.is_floating_point() and _is_param_key(k):
            t.requires_grad_(True)
        sd2[k] = t
    return Oracle(sd2), sd2


_BUFFER_SUFFIXES = ("pedestal", "bound", "mask", "target", "_offset", "_quantized_cdf", "_cdf_length",
                    "scale_table", "scale_bound")


def _is_param_key(k):
    return not k.endswith(_BUFFER_SUFFIXES)


def rel_err(a, b):
    a = a.double()
    b = b.double()
    return float((a - b).abs().max() / max(b.abs().max(), 1e-30))


# torchvision vgg16().features (configuration D): conv layer index -> (Co, Ci)
VGG16_CONVS = {0: (64, 3), 2: (64, 64), 5: (128, 64), 7: (128, 128), 10: (256, 128), 12: (256, 256), 14: (256, 256),
               17: (512, 256), 19: (512, 512), 21: (512, 512), 24: (512, 512), 26: (512, 512), 28: (512, 512)}


def vgg16_recipe_features(upto=28):
    """Deterministic stand-in for VGG16's ImageNet features (not downloadable here): He-scaled normal
    weights and small biases from one generator per layer, {"N.weight", "N.bias"} for conv layers <= upto.
    tests/golden/make_golden.py feeds the same tensors to the reference's own VGGLoss (src/losses/vgg16.py)."""
    sd = {}
    for i, (co, ci) in VGG16_CONVS.items():
        if i > upto:
            continue
        g = torch.Generator().manual_seed(1000 + i)
        sd[f"{i}.weight"] = torch.randn(co, ci, 3, 3, generator=g) * (2.0 / (ci * 9)) ** 0.5
        sd[f"{i}.bias"] = torch.randn(co, generator=g) * 0.01
    return sd
