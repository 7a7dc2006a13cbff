"""CPU: pin the oracle (oracle/hyres_oracle.py) against fixtures produced by the REFERENCE's own model
code (tests/golden/make_golden.py), and check this package's module tree / key layout against it."""
import math

import numpy as np
import pytest
import torch

from helpers import build_model, load_meta, load_npz, oracle_from, recipe_state_dict, rel_err


def test_state_dict_layout_matches_reference():
    meta = load_meta()
    net, sd = build_model()
    assert list(sd.keys()) == meta["state_dict_keys"]
    for k, v in sd.items():
        assert list(v.shape) == meta["state_dict_shapes"][k], k
    assert sum(p.numel() for p in net.parameters()) == meta["n_params"] == 10375280
    assert sum(p.numel() for p in net.residual_model.parameters()) == meta["n_params_codec"] == 10137219


def test_recipe_is_deterministic():
    a = recipe_state_dict()
    b = recipe_state_dict()
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_checkerboard_sets_bit_exact():
    g = load_npz("checkerboard_sets.npz")
    from oracle import Oracle
    am = Oracle.anchor_mask(4, 4)
    yy = torch.arange(16.0).view(4, 4)
    assert torch.equal(yy * am, g["anchor"].float())
    assert torch.equal(yy * (~am), g["non_anchor"].float())
    # CheckboardMaskedConv2d mask: 1 where (kh + kw) odd
    from models.layers.checkerboard import CheckboardMaskedConv2d
    m = CheckboardMaskedConv2d(4, 8, kernel_size=5, padding=2).mask[0, 0]
    assert torch.equal(m.int(), g["mask"].int())
    kh, kw = torch.meshgrid(torch.arange(5), torch.arange(5), indexing="ij")
    assert torch.equal(m.bool(), ((kh + kw) % 2 == 1))


@pytest.mark.parametrize("fixture", ["hyres_eval_b2_64.npz", "kodim01_crop64_eval.npz"])
def test_oracle_matches_reference_eval(fixture):
    torch.set_num_threads(8)
    g = load_npz(fixture)
    sd = recipe_state_dict()
    orc, _ = oracle_from(sd)
    T = {}
    with torch.no_grad():
        out = orc.forward(g["x"], g["jpeg_decoded"], float(g["jpeg_bpp"]), training=False, trace=T)
    for k in ("x_hat", "residual_hat"):
        assert rel_err(out[k], g[k]) < 1e-5, k
    assert rel_err(out["likelihoods"]["y"], g["y_likelihoods"]) < 1e-5
    assert rel_err(out["likelihoods"]["z"], g["z_likelihoods"]) < 1e-5
    if "y" in g:
        for k in ("y", "z", "z_hat", "latent_params", "y_anchor_hat", "ctx_params", "y_hat", "refined"):
            assert rel_err(T[k], g[k]) < 1e-5, k


def test_oracle_matches_reference_train_step():
    """Train-mode forward with the recorded noise draws + the RD loss + aux loss + parameter grads."""
    torch.set_num_threads(8)
    g = load_npz("hyres_train_b2_64.npz")
    meta = load_meta()
    sd = recipe_state_dict()
    orc, sd2 = oracle_from(sd, requires_grad=True)
    from oracle import rd_loss
    noise = {"z": g["noise_z"], "y": g["noise_y"]}
    out = orc.forward(g["x"], g["jpeg_decoded"], 0.0, training=True, noisequant=False, noise=noise)
    # jpeg bpp is a constant in the loss; the fixture's loss includes it
    jb = float(g["loss"]) - (meta["train_lambda"] * float(g["mse_loss"]) + float(g["y_bpp"]) + float(g["z_bpp"]))
    out["jpeg_bpp_loss"] = torch.tensor(jb)
    crit = rd_loss(out, g["x"], meta["train_lambda"])
    assert abs(float(crit["mse_loss"]) - float(g["mse_loss"])) <= 1e-5 * abs(float(g["mse_loss"]))
    assert abs(float(crit["y_bpp_loss"]) - float(g["y_bpp"])) <= 1e-5 * abs(float(g["y_bpp"]))
    assert abs(float(crit["z_bpp_loss"]) - float(g["z_bpp"])) <= 1e-5 * abs(float(g["z_bpp"]))
    assert rel_err(out["likelihoods"]["y"], g["y_likelihoods"]) < 1e-5
    crit["loss"].backward()
    aux = orc.eb_aux_loss()
    assert abs(float(aux) - float(g["aux_loss"])) <= 1e-5 * abs(float(g["aux_loss"]))
    # parameter gradients vs the reference's autograd (summaries: sum, sum of squares, samples)
    bad = []
    for k, summ in meta["train_grads"].items():
        t = sd2[k]
        if summ is None:
            assert t.grad is None or float(t.grad.abs().max()) == 0.0, k
            continue
        gd = t.grad.double()
        ss = float((gd * gd).sum())
        if abs(ss - summ["sumsq"]) > 1e-4 * max(summ["sumsq"], 1e-30):
            bad.append((k, ss, summ["sumsq"]))
    assert not bad, bad[:5]
