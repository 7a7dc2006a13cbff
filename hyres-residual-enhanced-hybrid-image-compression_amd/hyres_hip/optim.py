"""Fused Adam over flat parameter/gradient buffers (one HIP kernel per step) with clip_grad_norm_.

Replaces the gradient-path tail of src/utils/engine.py:56-90 (clip_grad_norm_(1.0) -> Adam.step ->
zero_grad) and src/utils/optimizers.py:4-35 (main vs ``*.quantiles`` aux optimiser).  Parameters are
re-pointed into one contiguous buffer per optimiser and their ``.grad`` tensors are views of one
contiguous gradient buffer, so:
  * the HIP wgrad kernels accumulate straight into the flat gradient (no copies);
  * the global grad norm is one reduction, Adam is one launch, zero_grad is one memset;
  * the DDP reducer all-reduces the flat buffer in large buckets over RCCL.
Math = torch.optim.Adam (amsgrad=False, weight_decay=0, foreach formulation):
  m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2; p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps),
with g scaled by min(1, max_norm / (||g||_2 + 1e-6)) when clipping (and by 1/scale under the GradScaler).
"""
from __future__ import annotations

import warnings
from typing import Iterable, List, Optional

import torch

from . import _lib as L
from . import ops as O


class FlatParams:
    """Move a list of parameters into one contiguous buffer (+ a gradient buffer of views)."""

    def __init__(self, params: List[torch.nn.Parameter]):
        self.params = list(params)
        assert self.params, "no parameters"
        dev = self.params[0].device
        n = sum(p.numel() for p in self.params)
        # 16-byte align every parameter view (float4 loads in the kernels)
        offs = []
        cur = 0
        for p in self.params:
            offs.append(cur)
            cur += (p.numel() + 3) // 4 * 4
        self.numel = cur
        self.data = torch.empty(cur, dtype=torch.float32, device=dev)
        # CPU buffers only exist for the gloo tests of the reducer (host plumbing, no compute)
        self.grad = O.zeros((cur,), dev) if dev.type == "cuda" else torch.zeros(cur, dtype=torch.float32)
        for p, o in zip(self.params, offs):
            k = p.numel()
            view = self.data[o:o + k].view_as(p)
            view.copy_(p.data)
            p.data = view
            p.grad = self.grad[o:o + k].view_as(p)
        self.offsets = offs
        O.bump_weight_epoch()

    def zero_grad(self):
        for p, o in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad.data_ptr() + 4 * o:
                p.grad = self.grad[o:o + p.numel()].view_as(p)
        if self.grad.is_cuda:
            O.zero_(self.grad)
        else:
            self.grad.zero_()


_ADAM_DEFAULTS = dict(weight_decay=0, amsgrad=False, maximize=False, foreach=None, capturable=False,
                      differentiable=False, fused=None)


def _device_buffer(n: int, device) -> torch.Tensor:
    # CPU buffers only exist for the host-side state-dict tests (no compute runs on them)
    return O.zeros((n,), device) if device.type == "cuda" else torch.zeros(n, dtype=torch.float32)


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam over one flat buffer, one HIP launch per step (+ clip_grad_norm_, GradScaler).

    The step count lives on the device so that a step skipped by the GradScaler (non-finite gradients)
    or by the reference's NaN check needs no host synchronisation.  ``state_dict()`` is in torch.optim.Adam's
    per-parameter layout (``state[i] = {step, exp_avg, exp_avg_sq}``, param_groups with Adam's keys), so a
    checkpoint written here resumes in the reference (src/training.py:219-226) and a reference checkpoint
    resumes here."""

    def __init__(self, params: Iterable[torch.nn.Parameter], lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 max_grad_norm: float = 0.0):
        params = [p for p in params]
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, **_ADAM_DEFAULTS))
        self.max_grad_norm = float(max_grad_norm)
        self.flat = FlatParams(params)
        dev = params[0].device
        self.exp_avg = _device_buffer(self.flat.numel, dev)
        self.exp_avg_sq = _device_buffer(self.flat.numel, dev)
        self.step_dev = _device_buffer(1, dev)  # completed steps (float, as torch's Adam ``step`` tensor)
        # sum g^2 of the last step's gradient, fp64 (hyres_sumsq: no overflow of a finite sum, so a non-finite
        # value means a non-finite element, as torch's element-wise found_inf)
        self.sumsq = torch.zeros(1, dtype=torch.float64, device=dev)

    def compute_sumsq(self) -> torch.Tensor:
        """sum of squares of the flat gradient into ``self.sumsq`` (device; no sync)."""
        ws = O._ws(L.load().hyres_reduce_workspace_bytes(self.flat.numel), self.flat.data.device, slot=5)
        L.call("hyres_sumsq", self.flat.grad.data_ptr(), self.flat.numel, self.sumsq.data_ptr(), ws.data_ptr(),
               ws.numel(), L.stream())
        return self.sumsq

    @torch.no_grad()
    def step(self, closure=None, grad_scaler: Optional["DeviceGradScaler"] = None,
             skip_if_nan: Optional[torch.Tensor] = None):
        """clip_grad_norm_(max_grad_norm) + Adam.step (src/utils/engine.py:68-82).

        grad_scaler: gradients are scaled by ``grad_scaler.scale``: unscale on the fly and skip the step
        when they are not finite (GradScaler.unscale_ + step semantics).  skip_if_nan: a device sum of
        squares (another optimiser's ``sumsq``); skip this step when it is NaN (the reference's ``continue``
        on NaN gradients also skips the aux step, engine.py:60-74)."""
        assert closure is None
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        sumsq, skip, gscale = None, 0, None
        if self.max_grad_norm > 0 or grad_scaler is not None:
            sumsq = self.compute_sumsq().data_ptr()
        if grad_scaler is not None:
            gscale = grad_scaler.inv_scale.data_ptr()
            skip = 1
        elif skip_if_nan is not None:
            # the kernel reads one sum of squares for both clipping and the skip test
            assert self.max_grad_norm == 0, "skip_if_nan is for the unclipped aux optimiser"
            assert skip_if_nan.dtype == torch.float64 and skip_if_nan.is_cuda, "skip_if_nan: a FusedAdam.sumsq"
            sumsq, skip = skip_if_nan.data_ptr(), 2
        L.call("hyres_adam_step", self.flat.data.data_ptr(), self.flat.grad.data_ptr(), self.exp_avg.data_ptr(),
               self.exp_avg_sq.data_ptr(), self.flat.numel, float(g["lr"]), float(b1), float(b2), float(g["eps"]),
               self.step_dev.data_ptr(), sumsq, self.max_grad_norm, gscale, skip, L.stream())
        O.bump_weight_epoch()

    @property
    def steps(self) -> int:
        return int(round(float(self.step_dev[0])))

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    def grad_norm(self) -> torch.Tensor:
        """||g||_2 (device scalar) of the flat gradient (what clip_grad_norm_ returns)."""
        return self.compute_sumsq().sqrt().float()

    # ------------------------------------------------------------------ checkpoints (torch.optim.Adam layout)
    def state_dict(self):
        group = {k: v for k, v in self.param_groups[0].items() if k != "params"}
        group["params"] = list(range(len(self.flat.params)))
        step = float(self.step_dev[0])
        state = {}
        if step > 0:
            for i, (p, o) in enumerate(zip(self.flat.params, self.flat.offsets)):
                k = p.numel()
                state[i] = {"step": torch.tensor(step, dtype=torch.float32),
                            "exp_avg": self.exp_avg[o:o + k].view_as(p),
                            "exp_avg_sq": self.exp_avg_sq[o:o + k].view_as(p)}
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd):
        """Accepts torch.optim.Adam state dicts (a reference checkpoint's ``optimizer`` /
        ``aux_optimizer``) and this class's own (same layout; round-1 ``hyres_flat`` files too)."""
        groups = sd["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(self.flat.params):
            raise ValueError(f"optimizer state has {sum(len(gr['params']) for gr in groups)} params in "
                             f"{len(groups)} group(s); expected {len(self.flat.params)} in 1")
        for k, v in groups[0].items():
            if k != "params":
                self.param_groups[0][k] = tuple(v) if k == "betas" else v
        flat = sd.get("hyres_flat")
        if flat is not None:  # round-1 format
            self.exp_avg.copy_(flat["exp_avg"])
            self.exp_avg_sq.copy_(flat["exp_avg_sq"])
            self.step_dev.fill_(float(flat["steps"]))
            return
        state = sd.get("state", {})
        steps = set()
        O.zero_(self.exp_avg) if self.exp_avg.is_cuda else self.exp_avg.zero_()
        O.zero_(self.exp_avg_sq) if self.exp_avg_sq.is_cuda else self.exp_avg_sq.zero_()
        for i, (pid, p, o) in enumerate(zip(groups[0]["params"], self.flat.params, self.flat.offsets)):
            st = state.get(pid, state.get(str(pid)))
            if not st:
                continue
            k = p.numel()
            for name, buf in (("exp_avg", self.exp_avg), ("exp_avg_sq", self.exp_avg_sq)):
                t = st[name]
                if t.numel() != k:
                    raise ValueError(f"optimizer state {pid}.{name}: {tuple(t.shape)} != {tuple(p.shape)}")
                buf[o:o + k].copy_(t.reshape(-1).to(buf.device, torch.float32))
            steps.add(float(st["step"]))
        if len(steps) > 1:
            warnings.warn(f"per-parameter Adam step counts differ ({sorted(steps)[:4]}); the fused optimiser "
                          f"keeps one count and resumes from the largest")
        self.step_dev.fill_(max(steps) if steps else 0.0)
        O.bump_weight_epoch()


class DeviceGradScaler:
    """torch.cuda.amp.GradScaler (engine.py:23,51,59,73,79-80) with its state on the device: the loss is
    multiplied by ``scale``; FusedAdam.step(grad_scaler=...) unscales on the fly and skips on non-finite
    gradients; ``update(sumsq)`` applies the backoff / growth rule without a host sync."""

    def __init__(self, device, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000):
        self.scale = torch.full((1,), float(init_scale), dtype=torch.float32, device=device)
        self.inv_scale = torch.full((1,), 1.0 / float(init_scale), dtype=torch.float32, device=device)
        self.tracker = torch.zeros(1, dtype=torch.int32, device=device)
        self.growth_factor, self.backoff_factor, self.growth_interval = growth_factor, backoff_factor, growth_interval

    def scale_loss(self, loss: torch.Tensor) -> torch.Tensor:
        return loss * self.scale.reshape(())

    def update(self, sumsq: torch.Tensor) -> None:
        L.call("hyres_grad_scaler_update", sumsq.data_ptr(), self.scale.data_ptr(), self.inv_scale.data_ptr(),
               self.tracker.data_ptr(), float(self.growth_factor), float(self.backoff_factor),
               int(self.growth_interval), L.stream())

    def get_scale(self) -> float:
        return float(self.scale[0])

    def state_dict(self):
        return {"scale": self.get_scale(), "growth_factor": self.growth_factor, "backoff_factor": self.backoff_factor,
                "growth_interval": self.growth_interval, "_growth_tracker": int(self.tracker[0])}

    def load_state_dict(self, sd):
        self.scale.fill_(float(sd["scale"]))
        self.inv_scale.fill_(1.0 / float(sd["scale"]))
        self.tracker.fill_(int(sd["_growth_tracker"]))
        self.growth_factor, self.backoff_factor = sd["growth_factor"], sd["backoff_factor"]
        self.growth_interval = sd["growth_interval"]


def configure_optimizers(net, args, max_grad_norm: float = 0.0):
    """src/utils/optimizers.py:4-35: main params vs ``*.quantiles`` (aux), both Adam(0.9, 0.999)."""
    parameters = {n for n, p in net.named_parameters() if not n.endswith(".quantiles") and p.requires_grad}
    aux_parameters = {n for n, p in net.named_parameters() if n.endswith(".quantiles") and p.requires_grad}
    params_dict = dict(net.named_parameters())
    assert len(parameters & aux_parameters) == 0
    assert len(parameters | aux_parameters) == len(params_dict)
    optimizer = FusedAdam((params_dict[n] for n in sorted(parameters)), lr=args.learning_rate,
                          betas=(0.9, 0.999), max_grad_norm=max_grad_norm)
    aux_optimizer = FusedAdam((params_dict[n] for n in sorted(aux_parameters)), lr=args.aux_learning_rate,
                              betas=(0.9, 0.999))
    return optimizer, aux_optimizer
