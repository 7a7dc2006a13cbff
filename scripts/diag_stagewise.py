"""Diagnostic: stage-wise activation values / gradients of the HIP train step vs the fp64 oracle, for the
noisequant=False and noisequant=True fixtures.  python scripts/diag_stagewise.py"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "hyres-residual-enhanced-hybrid-image-compression_amd"), REPO]
from helpers import load_meta, load_npz, recipe_state_dict, rel_err  # noqa: E402
import test_parity_gpu as T  # noqa: E402

KEYS = T.TRACE_KEYS + ["z_likelihoods", "y_likelihoods"]


def run(nq):
    from hyres_hip.loss import RateDistortionLoss
    from hyres_hip import ops as O
    from oracle import Oracle, rd_loss
    D = torch.device("cuda:0")
    if nq:
        g = load_npz("hyres_train_nq_b2_64.npz")
        keys = T.NQ_KEYS
        jb = float(g["jpeg_bpp"])
    else:
        g = load_npz("hyres_train_b2_64.npz")
        meta = load_meta()
        keys = {"z": "noise_z", "y": "noise_y"}
        jb = float(g["loss"]) - (meta["train_lambda"] * float(g["mse_loss"]) + float(g["y_bpp"]) + float(g["z_bpp"]))
    net, _ = T._hip_model()
    net.train()
    net.residual_model.noise.injected = T._nhwc_noise(g, keys, D)
    O.Trace.nodes = {}
    out = net(g["x"], noisequant=nq, jpeg=(g["jpeg_decoded"], jb))
    crit = RateDistortionLoss(lmbda=0.045, alpha=0)(out, g["x"].to(D))
    out["likelihoods"]["y"].retain_grad()
    out["likelihoods"]["z"].retain_grad()
    crit["loss"].backward()
    hv = {k: O.Trace.value(k).cpu() for k in O.Trace.nodes}
    hg = {k: (None if O.Trace.grad(k) is None else O.Trace.grad(k).cpu()) for k in O.Trace.nodes}
    O.Trace.nodes = None
    hv["y_likelihoods"], hg["y_likelihoods"] = out["likelihoods"]["y"].detach().cpu(), out["likelihoods"]["y"].grad.cpu()
    hv["z_likelihoods"], hg["z_likelihoods"] = out["likelihoods"]["z"].detach().cpu(), out["likelihoods"]["z"].grad.cpu()
    sd64 = {k: (v.clone().double() if v.is_floating_point() else v.clone()) for k, v in recipe_state_dict().items()}
    for k, v in sd64.items():
        if v.is_floating_point() and k.endswith(("weight", "bias")):
            v.requires_grad_(True)
    Tr = {}
    o = Oracle(sd64).forward(g["x"].double(), g["jpeg_decoded"].double(), jb, training=True, noisequant=nq,
                             noise={k: g[v].double() for k, v in keys.items()}, trace=Tr)
    for k in ("y_likelihoods", "z_likelihoods"):
        Tr[k].retain_grad()
    rd_loss(o, g["x"].double(), 0.045)["loss"].backward()
    print(f"=== noisequant={nq}")
    for k in KEYS:
        if k not in hv or k not in Tr:
            continue
        ge = None
        if hg.get(k) is not None and Tr[k].grad is not None:
            ge = rel_err(hg[k], Tr[k].grad)
        print(f"{k:18s} fwd {rel_err(hv[k], Tr[k].detach()):.2e} grad {'-' if ge is None else f'{ge:.2e}'}")


if __name__ == "__main__":
    torch.set_num_threads(16)
    run(False)
    run(True)
