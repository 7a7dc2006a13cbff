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
with g scaled by min(1, max_norm / (||g||_2 + 1e-6)) when clipping.
"""
from __future__ import annotations

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


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params: Iterable[torch.nn.Parameter], lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 max_grad_norm: float = 0.0):
        params = [p for p in params]
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))
        self.max_grad_norm = float(max_grad_norm)
        self.flat = FlatParams(params)
        self.exp_avg = O.zeros((self.flat.numel,), params[0].device)
        self.exp_avg_sq = O.zeros((self.flat.numel,), params[0].device)
        self.steps = 0
        self._sumsq = torch.empty(1, dtype=torch.float32, device=params[0].device)

    @torch.no_grad()
    def step(self, closure=None):
        assert closure is None
        self.steps += 1
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        sumsq = None
        if self.max_grad_norm > 0:
            ws = O._ws(L.load().hyres_reduce_workspace_bytes(self.flat.numel), self.flat.data.device, slot=5)
            L.call("hyres_sumsq", self.flat.grad.data_ptr(), self.flat.numel, self._sumsq.data_ptr(), ws.data_ptr(),
                   ws.numel(), L.stream())
            sumsq = self._sumsq.data_ptr()
        L.call("hyres_adam_step", self.flat.data.data_ptr(), self.flat.grad.data_ptr(), self.exp_avg.data_ptr(),
               self.exp_avg_sq.data_ptr(), self.flat.numel, float(g["lr"]), float(b1), float(b2), float(g["eps"]),
               self.steps, sumsq, self.max_grad_norm, L.stream())
        O.bump_weight_epoch()

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    def grad_norm(self) -> torch.Tensor:
        """||g||_2 (device scalar) of the flat gradient (what clip_grad_norm_ returns)."""
        ws = O._ws(L.load().hyres_reduce_workspace_bytes(self.flat.numel), self.flat.data.device, slot=5)
        out = torch.empty(1, dtype=torch.float32, device=self.flat.data.device)
        L.call("hyres_sumsq", self.flat.grad.data_ptr(), self.flat.numel, out.data_ptr(), ws.data_ptr(), ws.numel(),
               L.stream())
        return out.sqrt()

    def state_dict(self):
        sd = super().state_dict()
        sd["hyres_flat"] = {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "steps": self.steps}
        return sd

    def load_state_dict(self, sd):
        flat = sd.pop("hyres_flat", None)
        super().load_state_dict(sd)
        if flat is not None:
            self.exp_avg.copy_(flat["exp_avg"])
            self.exp_avg_sq.copy_(flat["exp_avg_sq"])
            self.steps = int(flat["steps"])


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
