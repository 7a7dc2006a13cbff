"""VGG16 perceptual loss (src/losses/vgg16.py:7-61, used by rd_loss.py:40 when alpha != 0).

torchvision and its ImageNet weights are not available here.  The restatement oracle/hyres_oracle.py:vgg_loss
is pinned to the reference's OWN VGGLoss code (src/losses/vgg16.py run by tests/golden/make_golden.py with a
torchvision stub: configuration-D features on deterministic recipe weights, Normalize restated —
vgg_b2_64.npz), and the HIP module is checked against both that fixture and the oracle; parity with the
ImageNet-pretrained network itself is unpinned (no weights to run)."""
import os

import pytest
import torch

from helpers import rel_err

# torchvision vgg16().features: conv layers at these indices
VGG_CONVS = [0, 2, 5, 7, 10, 12, 14, 17, 19, 21, 24, 26, 28]


def _expected_keys(layer_ids=(2, 7, 14, 21, 28)):
    keys, start = [], 0
    for s, lid in enumerate(layer_ids):
        for i in VGG_CONVS:
            if start <= i <= lid:
                keys += [f"slices.{s}.{i}.weight", f"slices.{s}.{i}.bias"]
        start = lid + 1
    return keys


def _vgg(seed=0):
    from hyres_hip.vgg import VGGLoss
    torch.manual_seed(seed)
    return VGGLoss(pretrained=False)


def test_vgg_state_dict_layout_matches_reference():
    """The reference's VGGLoss keeps vgg16().features' child names inside each slice (nn.Sequential slicing),
    so its state dict keys are slices.<s>.<features index>.{weight,bias}."""
    m = _vgg()
    assert list(m.state_dict().keys()) == _expected_keys()
    assert all(not p.requires_grad for p in m.parameters())
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert shapes["slices.0.0.weight"] == (64, 3, 3, 3) and shapes["slices.4.28.weight"] == (512, 512, 3, 3)


def test_vgg_needs_local_weights(monkeypatch, tmp_path):
    """models.vgg16(pretrained=True) downloads (vgg16.py:21): here the weights must be local."""
    from hyres_hip.vgg import VGGLoss, vgg16_features
    monkeypatch.delenv("HYRES_VGG16_WEIGHTS", raising=False)
    monkeypatch.setenv("TORCH_HOME", str(tmp_path / "none"))
    with pytest.raises(RuntimeError, match="HYRES_VGG16_WEIGHTS"):
        VGGLoss()
    # a torchvision-format file (full-model "features.N.*" keys) loads
    torch.manual_seed(3)
    feats = vgg16_features()
    sd = {f"features.{k}": v.clone() for k, v in feats.state_dict().items()}
    sd["classifier.0.weight"] = torch.zeros(2, 2)
    path = tmp_path / "vgg16-397923af.pth"
    torch.save(sd, path)
    monkeypatch.setenv("HYRES_VGG16_WEIGHTS", str(path))
    m = VGGLoss()
    assert torch.equal(m.state_dict()["slices.2.14.weight"], sd["features.14.weight"])


@pytest.mark.gpu
def test_vgg_loss_and_gradient_match_oracle():
    """HIP VGGLoss(x_hat, x) vs the oracle restatement on the same weights: loss within 1e-4 of fp32 torch-CPU,
    d loss / d x_hat within 1e-3 of fp64 in 2-norm and 5e-3 in max-norm (13 ReLUs between x_hat and the loss: a
    pre-activation at the kink may fall either way of it in any fp32 arithmetic; the fp32 torch-CPU gradient's own
    distance from fp64 is printed beside)."""
    from oracle.hyres_oracle import vgg_loss
    D = torch.device("cuda:0")
    m = _vgg(1)
    feats = {}
    for s in m.slices:
        for name, mod in s.named_children():
            if hasattr(mod, "weight"):
                feats[f"{name}.weight"] = mod.weight.detach().clone()
                feats[f"{name}.bias"] = mod.bias.detach().clone()
    g = torch.Generator().manual_seed(5)
    x = torch.rand(2, 3, 64, 64, generator=g)
    y = (x + 0.05 * torch.randn(2, 3, 64, 64, generator=g)).clamp(0, 1)
    ref32 = vgg_loss(feats, x, y)
    x64 = x.double().requires_grad_(True)
    vgg_loss(feats, x64, y.double()).backward()
    m = m.to(D)
    xd = x.to(D).requires_grad_(True)
    loss = m(xd, y.to(D))
    loss.backward()
    torch.cuda.synchronize()
    assert abs(float(loss) - float(ref32)) <= 1e-4 * abs(float(ref32)), (float(loss), float(ref32))
    x32 = x.clone().requires_grad_(True)
    vgg_loss(feats, x32, y).backward()
    gd, g64 = xd.grad.cpu().double(), x64.grad
    fro = float((gd - g64).norm() / g64.norm())
    print(f"d loss / d x_hat vs fp64: HIP {rel_err(gd, g64):.2e} max-norm, {fro:.2e} 2-norm; "
          f"fp32 torch-CPU {rel_err(x32.grad.double(), g64):.2e} max-norm")
    assert fro < 1e-3 and rel_err(gd, g64) < 5e-3


@pytest.mark.gpu
def test_rd_loss_with_vgg_term():
    """RateDistortionLoss(alpha > 0): loss = lambda * mse + bpp + alpha * vgg * 255^2 (rd_loss.py:40-42), and
    the perceptual term's gradient reaches x_hat through autograd next to the RD loss's own."""
    from oracle.hyres_oracle import vgg_loss
    from hyres_hip.loss import RateDistortionLoss
    D = torch.device("cuda:0")
    m = _vgg(2)
    feats = {f"{n}.{k}": getattr(mod, k).detach().clone() for s in m.slices for n, mod in s.named_children()
             if hasattr(mod, "weight") for k in ("weight", "bias")}
    g = torch.Generator().manual_seed(9)
    x = torch.rand(2, 3, 32, 32, generator=g)
    x_hat = (x + 0.1 * torch.randn(2, 3, 32, 32, generator=g)).clamp(0, 1)
    lik_y = torch.rand(2, 192, 4, 4, generator=g) * 0.9 + 0.05
    lik_z = torch.rand(2, 128, 1, 1, generator=g) * 0.9 + 0.05
    alpha, lmbda = 0.01, 0.045
    crit = RateDistortionLoss(lmbda=lmbda, alpha=alpha, vgg=m.to(D))
    xh = x_hat.to(D).requires_grad_(True)
    out = {"x_hat": xh, "likelihoods": {"y": lik_y.to(D), "z": lik_z.to(D)},
           "jpeg_bpp_loss": torch.tensor(0.5, device=D)}
    c = crit(out, x.to(D))
    c["loss"].backward()
    torch.cuda.synchronize()
    import math
    npx = 2 * 32 * 32
    bpp = (lik_y.log().sum() + lik_z.log().sum()) / (-math.log(2) * npx) + 0.5
    mse = torch.nn.functional.mse_loss(x_hat, x) * 255 ** 2
    v = vgg_loss(feats, x_hat, x) * 255 ** 2
    ref = lmbda * mse + bpp + alpha * v
    assert abs(float(c["vgg_loss"]) - float(v)) <= 1e-4 * float(v)
    assert abs(float(c["loss"]) - float(ref)) <= 1e-4 * abs(float(ref))
    xr = x_hat.double().requires_grad_(True)
    (lmbda * torch.nn.functional.mse_loss(xr, x.double()) * 255 ** 2 +
     alpha * vgg_loss(feats, xr, x.double()) * 255 ** 2).backward()
    assert rel_err(xh.grad.cpu(), xr.grad) < 1e-3


def _recipe_vgg_loss_module():
    """The product's VGGLoss holding tests/helpers.vgg16_recipe_features() (the weights the reference's own
    VGGLoss ran on in tests/golden/make_golden.py vgg_fixture)."""
    from helpers import vgg16_recipe_features
    from hyres_hip.vgg import VGGLoss
    m = VGGLoss(pretrained=False)
    sd = vgg16_recipe_features()
    with torch.no_grad():
        for s in m.slices:
            for name, mod in s.named_children():
                if hasattr(mod, "weight"):
                    mod.weight.copy_(sd[f"{name}.weight"])
                    mod.bias.copy_(sd[f"{name}.bias"])
    return m


def test_vgg_oracle_matches_reference_vggloss():
    """The oracle restatement (oracle/hyres_oracle.py:vgg_loss) against the reference's OWN VGGLoss code
    (src/losses/vgg16.py executed by make_golden.py with torchvision stubbed: configuration-D features on
    recipe weights, Normalize restated): loss 1e-5, d loss / d x_hat 1e-4 normwise."""
    from helpers import load_npz, vgg16_recipe_features
    from oracle.hyres_oracle import vgg_loss
    g = load_npz("vgg_b2_64.npz")
    sd = vgg16_recipe_features()
    xh = g["x_hat"].clone().requires_grad_(True)
    loss = vgg_loss(sd, xh, g["x"])
    loss.backward()
    assert abs(float(loss) - float(g["loss"])) <= 1e-5 * abs(float(g["loss"])), (float(loss), float(g["loss"]))
    assert rel_err(xh.grad, g["grad_x_hat"]) < 1e-4
    # the product module's slicing / state-dict layout carries the same weights
    m = _recipe_vgg_loss_module()
    assert torch.equal(m.state_dict()["slices.4.28.weight"], sd["28.weight"])


@pytest.mark.gpu
def test_vgg_loss_matches_reference_fixture_gpu():
    """The HIP VGGLoss (csrc/vgg.hip + HIP convs) against the reference VGGLoss fixture: loss 1e-4, input
    gradient 1e-3 normwise."""
    from helpers import load_npz
    g = load_npz("vgg_b2_64.npz")
    D = torch.device("cuda:0")
    m = _recipe_vgg_loss_module().to(D)
    xd = g["x_hat"].to(D).requires_grad_(True)
    loss = m(xd, g["x"].to(D))
    loss.backward()
    torch.cuda.synchronize()
    assert abs(float(loss) - float(g["loss"])) <= 1e-4 * abs(float(g["loss"])), (float(loss), float(g["loss"]))
    assert rel_err(xd.grad.cpu(), g["grad_x_hat"]) < 1e-3
