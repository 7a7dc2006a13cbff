"""Bridge between torch autograd and the HIP tape.

``TapeFunction`` runs a HIP forward (recording backward closures when gradients are needed) and, in
``backward``, seeds the output gradients and replays the tape.  Parameter gradients are written
straight into ``param.grad`` by the HIP kernels, so the Function returns ``None`` for parameters; the
parameters are still passed as inputs so that torch knows the outputs require grad.
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple

import torch

from . import ops as O
from .ops import Node, Tape


class _Spec:
    __slots__ = ("build", "record")

    def __init__(self, build: Callable, record: bool):
        self.build = build
        self.record = record


class TapeFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec: _Spec, n_in: int, *args):
        tensors = args[:n_in]
        tape = Tape() if spec.record else None
        in_nodes, outs = spec.build(tape, tensors)
        out_tensors = []
        out_nodes = []
        for o in outs:
            if isinstance(o, Node):
                out_tensors.append(O.to_nchw(o))
                out_nodes.append(o)
            else:
                out_tensors.append(o)
                out_nodes.append(None)
        ctx.spec = spec
        ctx.tape = tape
        ctx.in_nodes = in_nodes
        ctx.out_nodes = out_nodes
        ctx.n_in = n_in
        ctx.n_params = len(args) - n_in
        return tuple(out_tensors)

    @staticmethod
    def backward(ctx, *grads):
        tape = ctx.tape
        if tape is None:
            raise RuntimeError("HIP tape was not recorded (forward ran without grad)")
        for node, g in zip(ctx.out_nodes, grads):
            if node is None or g is None:
                continue
            node.set_grad(O.nchw_grad_to_nhwc(g))
        tape.backward()  # joins the side stream (weight gradients) at its end
        in_grads = []
        for node in ctx.in_nodes:
            if node is None or not node.rg or node.grad() is None:
                in_grads.append(None)
            else:
                in_grads.append(O.to_nchw_grad(node))
        # drop every reference to the step's activations: a loss tensor kept alive by the caller (metrics)
        # must not pin the tape's NHWC buffers and their gradients
        ctx.tape = None
        ctx.in_nodes = None
        ctx.out_nodes = None
        ctx.spec = None
        return (None, None) + tuple(in_grads) + (None,) * ctx.n_params


def run(build: Callable, tensors: Sequence[torch.Tensor], params: Sequence[torch.Tensor]):
    """Run ``build(tape, tensors) -> (in_nodes, outputs)`` under a TapeFunction."""
    record = torch.is_grad_enabled() and (any(p.requires_grad for p in params) or
                                          any(t.requires_grad for t in tensors if t is not None))
    spec = _Spec(build, record)
    params = [p for p in params if p.requires_grad] if record else []
    outs = TapeFunction.apply(spec, len(tensors), *tensors, *params)
    return outs


def module_forward(module, x: torch.Tensor) -> torch.Tensor:
    """Generic NCHW forward for any HIP module with ``hip(tape, node)``."""

    def build(tape, tensors):
        (xt,) = tensors
        node = O.to_nhwc(xt, rg=xt.requires_grad)
        return [node], [module.hip(tape, node)]

    (out,) = run(build, [x], list(module.parameters()))
    return out
