"""The gradient-path tail (reference src/utils/engine.py:56-90, src/utils/optimizers.py:4-35,
src/training.py:219-226): FusedAdam (+ fused clip_grad_norm_, GradScaler, NaN skip) against torch.optim.Adam +
torch.nn.utils.clip_grad_norm_ + torch.amp.GradScaler, and checkpoint compatibility with torch Adam state dicts.

CPU tests cover the state-dict conversion (host plumbing, no kernels); ``-m gpu`` tests run the HIP kernels."""
import math

import pytest
import torch

SHAPES = [(64, 3, 5, 5), (64,), (7, 3), (129,), (1,), (33, 17)]  # odd sizes: 16-byte padding between views


def _params(seed, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    return [torch.nn.Parameter((torch.rand(s, generator=g) - 0.5).to(device)) for s in SHAPES]


def _grads(seed, scale):
    g = torch.Generator().manual_seed(seed)
    return [(torch.rand(s, generator=g) - 0.5) * scale for s in SHAPES]


def _torch_adam_after(steps, lr=1e-3):
    ps = _params(0)
    opt = torch.optim.Adam(ps, lr=lr, betas=(0.9, 0.999))
    for k in range(steps):
        for p, gr in zip(ps, _grads(100 + k, 0.3)):
            p.grad = gr.clone()
        opt.step()
    return ps, opt


def test_fused_adam_loads_torch_adam_state_cpu():
    """A reference checkpoint's ``optimizer`` entry (torch.optim.Adam) resumes into FusedAdam's flat buffers."""
    from hyres_hip.optim import FusedAdam
    ps, topt = _torch_adam_after(2)
    sd = topt.state_dict()
    mine = FusedAdam([torch.nn.Parameter(p.detach().clone()) for p in ps], lr=5.0)
    mine.load_state_dict(sd)
    assert mine.param_groups[0]["lr"] == 1e-3 and mine.param_groups[0]["betas"] == (0.9, 0.999)
    assert float(mine.step_dev[0]) == 2.0
    for i, (p, o) in enumerate(zip(mine.flat.params, mine.flat.offsets)):
        k = p.numel()
        assert torch.equal(mine.exp_avg[o:o + k].view_as(p), topt.state[ps[i]]["exp_avg"])
        assert torch.equal(mine.exp_avg_sq[o:o + k].view_as(p), topt.state[ps[i]]["exp_avg_sq"])


def test_fused_adam_state_dict_loads_into_torch_adam_cpu():
    """A checkpoint written by this build resumes in the reference's torch.optim.Adam (both directions)."""
    from hyres_hip.optim import FusedAdam
    ps, topt = _torch_adam_after(3)
    mine = FusedAdam([torch.nn.Parameter(p.detach().clone()) for p in ps], lr=1e-3)
    mine.load_state_dict(topt.state_dict())
    sd = mine.state_dict()
    assert sorted(sd["state"]) == list(range(len(SHAPES)))
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    t2 = torch.optim.Adam(qs, lr=0.5)
    t2.load_state_dict(sd)
    assert t2.param_groups[0]["lr"] == 1e-3
    for q, p in zip(qs, ps):
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(t2.state[q][k], topt.state[p][k])
        assert float(t2.state[q]["step"]) == 3.0
    # and the continued steps agree (torch Adam on both sides: the state really carried over)
    for p, q, gr in zip(ps, qs, _grads(7, 0.3)):
        p.grad, q.grad = gr.clone(), gr.clone()
    topt.step()
    t2.step()
    for p, q in zip(ps, qs):
        assert torch.equal(p, q)


def test_fused_adam_empty_state_cpu():
    """A fresh optimiser's state dict is a fresh torch Adam's (no per-parameter state before step 1)."""
    from hyres_hip.optim import FusedAdam
    mine = FusedAdam(_params(1), lr=1e-4)
    sd = mine.state_dict()
    assert sd["state"] == {}
    t = torch.optim.Adam(_params(1), lr=1e-3)
    t.load_state_dict(sd)
    assert t.param_groups[0]["lr"] == 1e-4
    with pytest.raises(ValueError):
        FusedAdam(_params(1)[:2]).load_state_dict(sd)


# ------------------------------------------------------------------------------------------------ GPU
def _dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / max(float(b.double().abs().max()), 1e-30))


@pytest.mark.gpu
def test_fused_adam_clip_matches_torch_gpu():
    """3 steps of FusedAdam(max_grad_norm=1.0) + the aux FusedAdam (no clip) vs torch.optim.Adam +
    clip_grad_norm_(1.0) (engine.py:76-82, 87-90) on the same gradients: parameters within 1e-6 relative.
    Gradient norms 2.6, 1.3 and 0.26: clipping engages on the first two steps only."""
    from hyres_hip.optim import FusedAdam
    D = _dev()
    ref = [torch.nn.Parameter(p.detach().to(D)) for p in _params(3)]
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    aux_ref = [torch.nn.Parameter(torch.rand(128, 1, 3, device=D))]
    aux_mine = [torch.nn.Parameter(aux_ref[0].detach().clone())]
    topt = torch.optim.Adam(ref, lr=1e-3, betas=(0.9, 0.999))
    taux = torch.optim.Adam(aux_ref, lr=1e-3, betas=(0.9, 0.999))
    fopt = FusedAdam(mine, lr=1e-3, betas=(0.9, 0.999), max_grad_norm=1.0)
    faux = FusedAdam(aux_mine, lr=1e-3, betas=(0.9, 0.999))
    norms = []
    for k, scale in enumerate((0.3, 0.15, 0.03)):
        grads = [gr.to(D) for gr in _grads(200 + k, scale)]
        norms.append(math.sqrt(sum(float((gr.double() ** 2).sum()) for gr in grads)))
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        fopt.zero_grad()
        for p, gr in zip(mine, grads):
            p.grad.copy_(gr)
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        topt.step()
        fopt.step()
        ga = torch.rand(aux_ref[0].shape, device=D) - 0.5
        aux_ref[0].grad = ga.clone()
        faux.zero_grad()
        aux_mine[0].grad.copy_(ga)
        taux.step()
        faux.step()
    torch.cuda.synchronize()
    assert norms[0] > 1.0 and norms[1] > 1.0 and norms[2] < 1.0, norms
    for p, q in zip(ref, mine):
        assert float((q.detach() - p.detach()).abs().max()) <= 1e-6 * float(p.detach().abs().max())
    assert float((aux_mine[0] - aux_ref[0]).detach().abs().max()) <= 1e-6 * float(aux_ref[0].detach().abs().max())
    assert fopt.steps == 3 and faux.steps == 3
    sd = fopt.state_dict()
    for i, p in enumerate(ref):
        assert _rel(sd["state"][i]["exp_avg"], topt.state[p]["exp_avg"]) < 1e-5
        assert _rel(sd["state"][i]["exp_avg_sq"], topt.state[p]["exp_avg_sq"]) < 1e-5


@pytest.mark.gpu
def test_fused_adam_resume_from_torch_checkpoint_gpu():
    """Resume (training.py:219-226): torch Adam runs 2 steps, its state dict loads into FusedAdam, and one
    more step on each side agrees (moments and bias correction carried over, not restarted)."""
    from hyres_hip.optim import FusedAdam
    D = _dev()
    ref = [torch.nn.Parameter(p.detach().to(D)) for p in _params(5)]
    topt = torch.optim.Adam(ref, lr=1e-3)
    for k in range(2):
        for p, gr in zip(ref, _grads(300 + k, 0.2)):
            p.grad = gr.to(D)
        topt.step()
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    fopt = FusedAdam(mine, lr=1e-3)
    fopt.load_state_dict(topt.state_dict())
    grads = [gr.to(D) for gr in _grads(400, 0.2)]
    for p, gr in zip(ref, grads):
        p.grad = gr.clone()
    fopt.zero_grad()
    for p, gr in zip(mine, grads):
        p.grad.copy_(gr)
    topt.step()
    fopt.step()
    torch.cuda.synchronize()
    assert fopt.steps == 3
    for p, q in zip(ref, mine):
        assert float((q.detach() - p.detach()).abs().max()) <= 1e-6 * float(p.detach().abs().max())


@pytest.mark.gpu
def test_grad_scaler_skip_and_backoff_gpu():
    """AMP tail (engine.py:50-82) vs torch.amp.GradScaler: scaled gradients are unscaled before clipping; a
    step with an inf gradient is skipped and halves the scale; a NaN gradient (sum of squares NaN) also
    skips the aux step on the device; after growth_interval clean steps the scale doubles."""
    from hyres_hip.optim import DeviceGradScaler, FusedAdam
    D = _dev()
    ref = [torch.nn.Parameter(p.detach().to(D)) for p in _params(9)]
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    topt = torch.optim.Adam(ref, lr=1e-3)
    fopt = FusedAdam(mine, lr=1e-3, max_grad_norm=1.0)
    tsc = torch.amp.GradScaler("cuda", init_scale=2.0 ** 16, growth_interval=3)
    msc = DeviceGradScaler(D, init_scale=2.0 ** 16, growth_interval=3)
    tsc.scale(torch.ones((), device=D))  # torch's scaler allocates its state lazily on the first scale()
    aux = [torch.nn.Parameter(torch.ones(4, device=D))]
    faux = FusedAdam(aux, lr=1e-2)
    # "big": a finite scaled gradient whose fp32 sum of squares would overflow — torch's found_inf is
    # element-wise, so it must NOT skip the step or back the scale off (hyres_sumsq accumulates in fp64)
    plan = ["ok", "inf", "ok", "big", "nan", "ok", "ok", "ok"]
    aux_steps = 0
    for k, kind in enumerate(plan):
        S = tsc.get_scale()
        grads = [gr.to(D) * S for gr in _grads(500 + k, 0.3)]
        if kind == "inf":
            grads[2][0, 1] = float("inf")
        if kind == "nan":
            grads[3][7] = float("nan")
        if kind == "big":
            grads[1].view(-1)[:4] = 1e15 * S
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        fopt.zero_grad()
        for p, gr in zip(mine, grads):
            p.grad.copy_(gr)
        tsc.unscale_(topt)
        if not any(torch.isnan(p.grad).any() for p in ref):
            torch.nn.utils.clip_grad_norm_(ref, 1.0)
            tsc.step(topt)
            aux_steps += 1
        tsc.update()
        fopt.step(grad_scaler=msc)
        msc.update(fopt.sumsq)
        faux.zero_grad()
        aux[0].grad.fill_(1.0)
        faux.step(skip_if_nan=fopt.sumsq.clone())
        torch.cuda.synchronize()
        assert msc.get_scale() == tsc.get_scale(), (k, kind, msc.get_scale(), tsc.get_scale())
    assert fopt.steps == sum(k in ("ok", "big") for k in plan)
    assert faux.steps == aux_steps == sum(k != "nan" for k in plan)
    for p, q in zip(ref, mine):
        assert float((q.detach() - p.detach()).abs().max()) <= 2e-6 * float(p.detach().abs().max())
