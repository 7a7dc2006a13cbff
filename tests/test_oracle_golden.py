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


def _nq_noise(g):
    return {"z": g["noise_z"], "y_anchor": g["noise_y_anchor"], "y_non_anchor": g["noise_y_non_anchor"],
            "y": g["noise_y"]}


def test_oracle_matches_reference_train_step_noisequant():
    """noisequant=True train step (the reference's default for epochs <= 400, src/training.py:238-243):
    EB noise on z feeds h_s directly (no STE), Quantizer "noise" on the anchor and non-anchor halves
    (models/checkerboard.py:121-122,132-133, noise added at EVERY position), GC noise on y."""
    import json
    import os
    from conftest import GOLDEN
    torch.set_num_threads(8)
    g = load_npz("hyres_train_nq_b2_64.npz")
    with open(os.path.join(GOLDEN, "hyres_train_nq_b2_64.json")) as f:
        meta = json.load(f)
    orc, sd2 = oracle_from(recipe_state_dict(), requires_grad=True)
    from oracle import rd_loss
    out = orc.forward(g["x"], g["jpeg_decoded"], float(g["jpeg_bpp"]), training=True, noisequant=True,
                      noise=_nq_noise(g))
    crit = rd_loss(out, g["x"], meta["lambda"])
    for k, r in (("mse_loss", "mse_loss"), ("y_bpp_loss", "y_bpp"), ("z_bpp_loss", "z_bpp"), ("loss", "loss")):
        assert abs(float(crit[k].detach()) - float(g[r])) <= 1e-5 * abs(float(g[r])), k
    assert rel_err(out["likelihoods"]["y"].detach(), g["y_likelihoods"]) < 1e-5
    assert rel_err(out["likelihoods"]["z"].detach(), g["z_likelihoods"]) < 1e-5
    assert rel_err(out["x_hat"].detach(), g["x_hat"]) < 1e-5
    crit["loss"].backward()
    aux = orc.eb_aux_loss()
    assert abs(float(aux) - float(g["aux_loss"])) <= 1e-5 * abs(float(g["aux_loss"]))
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


def test_entropy_coder_tables_match_restatement():
    """update() (models/checkerboard.py:261-267 -> compressai EntropyBottleneck.update /
    GaussianConditional.update_scale_table, run on the host as src/updata.py does) builds CDF tables identical
    to the compressai-1.2.6 restatement in oracle/entropy_coding.py, entry for entry."""
    from oracle.entropy_coding import eb_tables, gc_tables
    net, sd = build_model()
    rm = net.residual_model
    assert rm.update(force=True)
    orc, _ = oracle_from(sd)
    cdf, ln, off = eb_tables(sd["residual_model.entropy_bottleneck.quantiles"], orc.eb_logits_cumulative)
    eb = rm.entropy_bottleneck
    assert np.array_equal(eb._quantized_cdf.numpy(), cdf)
    assert np.array_equal(eb._cdf_length.numpy(), ln) and np.array_equal(eb._offset.numpy(), off)
    gc = rm.gaussian_conditional
    cdf, ln, off = gc_tables(gc.scale_table.numpy())
    assert np.array_equal(gc._quantized_cdf.numpy(), cdf)
    assert np.array_equal(gc._cdf_length.numpy(), ln) and np.array_equal(gc._offset.numpy(), off)


def test_reference_compress_restatement_roundtrips():
    """The oracle's LightWeightCheckerboard.compress restatement decodes back to its own symbols (so the
    byte-equality test of the HIP compress() against it is meaningful)."""
    from oracle.entropy_coding import rans_decode, reference_compress
    from models.checkerboard import get_scale_table
    torch.set_num_threads(8)
    g = load_npz("kodim01_crop64_eval.npz")
    orc, _ = oracle_from(recipe_state_dict())
    table = get_scale_table().numpy().astype(np.float32)
    strings, it = reference_compress(orc, g["x"] - g["jpeg_decoded"], table)
    cdf, ln, off = it["gc_tables"]
    dec = rans_decode(strings[0][1][0], it["non_anchor_idx"][0].reshape(-1).tolist(), cdf.tolist(), ln.tolist(),
                      off.tolist())
    assert dec == it["non_anchor_sym"][0].reshape(-1).tolist()
    cdf, ln, off = it["eb_tables"]
    C, h, w = it["z_sym"].shape[1:]
    dec = rans_decode(strings[1][0], np.repeat(np.arange(C), h * w).tolist(), cdf.tolist(), ln.tolist(), off.tolist())
    assert dec == it["z_sym"][0].reshape(-1).tolist()
