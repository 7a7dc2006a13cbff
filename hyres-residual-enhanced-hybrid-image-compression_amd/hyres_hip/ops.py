"""HIP op library for the HyRES hot path: NHWC activation nodes, a reverse-mode tape, and one
function per reference operation, each launching libhyres_hip kernels on torch's current stream.

Design (MI355X-first, not a port):
  * activations live in HBM as NHWC fp32 (``Node``: a [B,H,W,C] view whose channel slice may sit
    inside a wider buffer — concatenations are free, producers write straight into the slice);
  * the forward pass records backward closures on a ``Tape``; backward replays them in reverse and
    launches the dgrad / wgrad / elementwise-backward kernels itself (no torch autograd kernels, no
    torch compute kernels: torch only allocates memory and supplies the stream);
  * parameter gradients are accumulated straight into ``param.grad`` by the HIP wgrad kernels.

Reference anchors are given per op; the math restated here is checked stage-by-stage against the
CPU oracle (oracle/hyres_oracle.py) in tests/test_parity_gpu.py.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import weakref
from typing import Callable, List, Optional

import torch

from . import _lib as L

# --------------------------------------------------------------------------------------------------
# infrastructure
# --------------------------------------------------------------------------------------------------
_WEIGHT_EPOCH = [0]


def bump_weight_epoch() -> None:
    """Invalidate cached weight re-layouts (called after optimiser steps / state loads)."""
    _WEIGHT_EPOCH[0] += 1


class Workspace:
    """Per-device scratch buffer, grown on demand; stream-ordered reuse is safe because every op
    finishes with its scratch before the next op's kernels start on the same stream."""

    _bufs = {}

    @classmethod
    def get(cls, nbytes: int, device: torch.device, slot: int = 0) -> torch.Tensor:
        # per (device, slot, stream): concurrent branches / the side stream never share scratch
        key = (device.index, slot, torch.cuda.current_stream(device).cuda_stream if device.type == "cuda" else 0)
        buf = cls._bufs.get(key)
        if buf is None or buf.numel() < nbytes:
            n = max(int(nbytes), 1 << 20)
            if buf is not None:
                n = max(n, int(buf.numel() * 1.5))
            buf = torch.empty(n, dtype=torch.uint8, device=device)
            cls._bufs[key] = buf
        return buf


def _empty(shape, device, dtype=torch.float32) -> torch.Tensor:
    return torch.empty(shape, dtype=dtype, device=device)


def zero_(t: torch.Tensor) -> torch.Tensor:
    L.call("hyres_zero", t.data_ptr(), t.numel() * t.element_size(), L.stream())
    return t


def zeros(shape, device) -> torch.Tensor:
    return zero_(_empty(shape, device))


class Node:
    """NHWC activation [B,H,W,C]; ``v`` may be a channel slice of a wider buffer (pixel stride ld)."""

    __slots__ = ("v", "B", "H", "W", "C", "ld", "rg", "parent", "c0", "_g", "gflag", "relu_out", "gmasked",
                 "pending", "prelu", "pmasked", "prelu_slices")

    def __init__(self, v: torch.Tensor, rg: bool = True, parent: "Node" = None, c0: int = 0):
        assert v.dim() == 4 and v.stride(3) == 1, "Node expects an NHWC tensor with unit channel stride"
        self.v = v
        self.B, self.H, self.W, self.C = v.shape
        self.ld = v.stride(2)
        assert v.stride(1) == self.W * self.ld and v.stride(0) == self.H * self.W * self.ld
        self.rg = rg
        self.parent = parent
        self.c0 = c0
        self._g = None
        self.gflag = False
        # ReLU-backward fusion: ``relu_out`` = v is the output of a ReLU fused into its producer;
        # ``gmasked`` = the gradient accumulated so far already carries the ReLU mask (set by a consumer
        # whose input-gradient epilogue applied it as the FIRST contribution; cleared by any later one).
        self.relu_out = False
        self.gmasked = False
        # PReLU-backward fusion: ``prelu`` = (pre-activation, slope) when v is the output of a PReLU fused into its
        # producer (training); ``pmasked`` = the one gradient writer applied the PReLU backward in its epilogue
        # (HYRES_ACT_PRELU_MASK) — unlike the ReLU mask it is not idempotent, so no second contribution may follow
        self.prelu = None
        self.pmasked = False
        # channel slices of this node written by a conv with a fused PReLU (training): the writer of this node's
        # gradient may apply their PReLU backward (refine_ops.sa_fold_fusion: MultiScaleRefine's scale 1 in multi)
        self.prelu_slices = None
        # deferred residual gradient (tensor, pixel stride): added by the next input-gradient conv's
        # epilogue (``grad_target_epi``) instead of a separate add pass, or materialised on first access
        self.pending = None

    @staticmethod
    def new(B, H, W, C, device, rg=True, dtype=torch.float32) -> "Node":
        return Node(_empty((B, H, W, C), device, dtype), rg)

    @property
    def half(self) -> bool:
        """fp16 storage (autocast inference with fp16 activations, see ``act_f16``)."""
        return self.v.dtype == torch.float16

    @property
    def ghalf(self) -> bool:
        """fp16 gradient storage: the gradient of an fp16 activation is fp16, as under torch autocast
        (src/utils/engine.py:32,50-53: autograd gives an fp16 tensor an fp16 gradient); HYRES_AMP_F16_GRAD=0
        keeps fp32 gradients for fp16 activations."""
        return AMP_F16_GRAD and self.v.dtype == torch.float16

    @property
    def gdt(self) -> torch.dtype:
        return torch.float16 if self.ghalf else torch.float32

    def slice(self, c0: int, c1: int, rg: Optional[bool] = None) -> "Node":
        return Node(self.v[..., c0:c1], self.rg if rg is None else rg, parent=self, c0=c0)

    @property
    def P(self) -> int:
        return self.B * self.H * self.W

    @property
    def device(self):
        return self.v.device

    @property
    def contiguous(self) -> bool:
        return self.ld == self.C

    def ptr(self) -> int:
        return self.v.data_ptr()

    # ---- gradients
    def grad(self) -> Optional[torch.Tensor]:
        """The accumulated gradient (same view structure as v) or None if nothing flowed here."""
        if self.pending is not None:
            self._materialize()
        if self.parent is not None:
            pg = self.parent.grad()
            return None if pg is None else pg[..., self.c0:self.c0 + self.C]
        return self._g if self.gflag else None

    def grad_ld(self) -> int:
        return self.parent.grad_ld() if self.parent is not None else self.C

    def defer_residual(self, g: torch.Tensor, ld: int) -> bool:
        """Record the residual-branch gradient ``g`` (pixel stride ``ld``) to be added inside the next writer's
        epilogue (False: not deferrable, the caller adds it now). Round 6: also onto a node that already holds a
        gradient (an AttentionBlock input: the gate's identity term arrives first) — the next input-gradient conv
        then writes old + (conv + g) with accumulate on, instead of an add2d pass before it (DEFER_ON_GRAD=False:
        the round-5 rule, first contribution only)."""
        if self.parent is not None or (self.gflag and not DEFER_ON_GRAD) or self.pending is not None:
            return False
        self.pending = (g, ld)
        return True

    def _materialize(self) -> None:
        g, ld = self.pending
        self.pending = None
        tgt, acc = self.grad_target()
        add2d(g, ld, tgt, self.C, self.P, self.C, acc)

    def grad_target_epi(self, e: "L.Epilogue"):
        """``grad_target`` for an input-gradient conv: a deferred residual gradient is folded into its
        epilogue as ``e.res`` (the ReLU mask, if the conv applies it, then covers both). Returns
        (tensor, accumulate, keep-alive tensor or None)."""
        # the conv reads e.res in the dtype of the gradient it writes: fold only a same-dtype pending gradient
        # (a mixed pair, e.g. an fp16 gradient deferred onto an fp32-gradient node, goes through add2d)
        if (self.pending is not None and self.parent is None and (DEFER_ON_GRAD or not self.gflag)
                and self.pending[0].dtype == self.gdt):
            g, ld = self.pending
            self.pending = None
            tgt, acc = self.grad_target()
            e.res = g.data_ptr()
            e.ldres = ld
            return tgt, acc, g
        tgt, acc = self.grad_target()
        return tgt, acc, None

    def grad_target(self):
        """(tensor, accumulate) for a kernel that adds its contribution to this node's gradient."""
        if self.pending is not None:
            self._materialize()
        if self.parent is not None:
            pg, _ = self.parent._zeroed_grad()
            return pg[..., self.c0:self.c0 + self.C], 1
        if self._g is None:
            self._g = _empty(self.v.shape, self.v.device, self.gdt)
        acc = 1 if self.gflag else 0
        if acc:
            if self.pmasked:
                raise RuntimeError("a second gradient contribution to a node whose PReLU backward was folded")
            self.gmasked = False  # a later, unmasked contribution: the producer re-applies the mask
        self.gflag = True
        return self._g, acc

    def relu_mask_epilogue(self, e: "L.Epilogue", acc: int) -> None:
        """Let an input-gradient conv writing this node's gradient apply the ReLU mask (first writer)."""
        if acc == 0 and self.relu_out and self.parent is None:
            e.act = L.ACT_RELU_MASK
            e.aux0 = self.ptr()
            e.ld0 = self.ld
            self.gmasked = True

    def prelu_mask_epilogue(self, e: "L.Epilogue", acc: int, g: "L.ConvGeom") -> None:
        """Let the input-gradient conv writing this node's gradient apply the PReLU backward (HYRES_ACT_PRELU_MASK,
        include/hyres_hip.h): this node is a fused PReLU's output, the conv is its first writer, fp32, and the launcher
        routes it to conv3x3_wres_bf6_kernel (MultiScaleRefine's scale blocks, enhancement.py:89-95: the dilation-2
        conv's input-gradient). Replaces prelu_bwd of that PReLU; its slope gradient sum is added by the same call."""
        if not (FOLD_PRELU and acc == 0 and self.prelu is not None and self.parent is None and not self.half
                and e.act == L.ACT_NONE and e.kind == L.EPI_BIAS and not e.accumulate and not e.io_f16
                and not Trace.traced(self)):
            return
        pre, slope = self.prelu
        if pre.dtype != torch.float32 or not pre.is_contiguous():
            return
        e.act = L.ACT_PRELU_MASK
        e.aux0, e.ld0 = pre.data_ptr(), self.C
        if not conv_variant(g, e, False).startswith("conv3x3_wres_bf6_kernel"):
            e.act, e.aux0, e.ld0 = L.ACT_NONE, None, 0
            return
        dslope = param_grad(slope) if slope.requires_grad else _empty((1,), self.device)
        part = _empty((L.PRELU_PARTIALS,), self.device)
        e.slope = slope.data_ptr()
        e.aux1 = dslope.data_ptr()
        e.aux2, e.ld2 = part.data_ptr(), L.PRELU_PARTIALS
        self.pmasked = True

    def _zeroed_grad(self):
        if self.pmasked:
            raise RuntimeError("a second gradient contribution to a node whose PReLU backward was folded")
        if self.pending is not None:
            self._materialize()
        self.gmasked = False  # the caller accumulates an unmasked contribution
        if self._g is None:
            self._g = zero_(_empty(self.v.shape, self.v.device, self.gdt))
            self.gflag = True
        elif not self.gflag:
            zero_(self._g)
            self.gflag = True
        return self._g, 1

    def set_grad(self, g: torch.Tensor) -> None:
        """Seed this node's gradient (accumulating if already present)."""
        tgt, acc = self.grad_target()
        add2d(g, g.stride(2), tgt, tgt.stride(2), self.P, self.C, acc)


def add2d(x: torch.Tensor, ldx: int, y: torch.Tensor, ldy: int, P: int, C: int, acc: int) -> None:
    """y[p, c] (+)= x[p, c] over [P][C] with pixel strides ldx / ldy, each side fp32 or fp16 (its tensor's dtype)."""
    io = (1 if x.dtype == torch.float16 else 0) | (2 if y.dtype == torch.float16 else 0)
    if io:
        L.call("hyres_add2d_f16", x.data_ptr(), ldx, y.data_ptr(), ldy, P, C, acc, io, L.stream())
    else:
        L.call("hyres_add2d", x.data_ptr(), ldx, y.data_ptr(), ldy, P, C, acc, L.stream())


def accumulate(x: torch.Tensor, y: torch.Tensor) -> None:
    """y += x elementwise (same dtype)."""
    assert x.dtype == y.dtype
    fn = "hyres_accumulate_f16" if x.dtype == torch.float16 else "hyres_accumulate"
    L.call(fn, x.data_ptr(), y.data_ptr(), x.numel(), L.stream())


class Tape:
    """Reverse-mode tape of backward closures over HIP launches."""

    def __init__(self):
        self.ops: List[Callable[[], None]] = []
        self.param_hooks: List[Callable[[], None]] = []

    def push(self, fn: Callable[[], None]) -> None:
        self.ops.append(fn)

    def backward(self) -> None:
        for fn in reversed(self.ops):
            fn()
        self.ops.clear()
        WgradBatch.flush()  # deferred weight-gradient reduces of the main stream
        SideStream.join()  # side-stream weight gradients complete before anyone reads .grad


class GradReady:
    """Backward-progress markers for overlapping the gradient all-reduce with backward.

    ``mark(tape, name)`` during forward pushes a closure; the tape replays closures in reverse, so in
    backward it runs once every layer built after the mark has launched its gradients (weight gradients
    are on the side stream). Listeners (hyres_hip.ddp.FlatGradReducer.on_marker) are called with
    ``name``; with no listener registered the mark costs nothing."""

    listeners: list = []

    @classmethod
    def mark(cls, tape: Optional["Tape"], name: str) -> None:
        if tape is None or not cls.listeners:
            return
        ls = list(cls.listeners)

        def fire():
            WgradBatch.flush()  # this segment's weight gradients final before the listeners act
            for f in ls:
                f(name)

        tape.push(fire)


class Trace:
    """Debug/parity hook: when ``Trace.nodes`` is a dict, named activations are kept (by reference) so
    tests can read their values (``value``) and, after backward, their gradients (``grad``)."""

    nodes = None
    # (kind, output node, pre-activation tensor or None) of every ReLU / PReLU fused into a conv epilogue,
    # in forward order (tests read the branch decisions to make the oracle follow them at the kink)
    acts = None

    @classmethod
    def add(cls, name: str, node: "Node") -> None:
        if cls.nodes is not None:
            cls.nodes[name] = node

    @classmethod
    def act(cls, node: "Node", act: int, pre: Optional[torch.Tensor]) -> None:
        if cls.acts is not None and act in (L.ACT_RELU, L.ACT_PRELU):
            cls.acts.append(("relu" if act == L.ACT_RELU else "prelu", node, pre))

    @classmethod
    def decisions(cls):
        """{"relu": [...], "prelu": [...]} NCHW bool masks (pre-activation > 0) in forward order."""
        out = {"relu": [], "prelu": []}
        for kind, node, pre in cls.acts or []:
            if pre is not None:
                d = pre.view(node.B, node.H, node.W, node.C).permute(0, 3, 1, 2) > 0
            else:
                d = to_nchw(node) > 0
            out[kind].append(d.cpu())
        return out

    @classmethod
    def traced(cls, node: "Node") -> bool:
        """``node`` is a named trace point: the PReLU-backward folds skip it, since they store the gradient of the
        pre-activation in the node's gradient buffer, and the trace reads the gradient of the node's own value."""
        return cls.nodes is not None and any(v is node for v in cls.nodes.values())

    @classmethod
    def value(cls, name: str) -> torch.Tensor:
        return to_nchw(cls.nodes[name])

    @classmethod
    def grad(cls, name: str) -> Optional[torch.Tensor]:
        n = cls.nodes[name]
        return None if n.grad() is None else to_nchw_grad(n)


def param_grad(p: torch.nn.Parameter) -> torch.Tensor:
    """param.grad, created zeroed if absent; HIP kernels always accumulate into it."""
    if p.grad is None:
        p.grad = zeros(p.shape, p.device)
    return p.grad


def wants_grad(p: Optional[torch.Tensor]) -> bool:
    return p is not None and p.requires_grad


# --------------------------------------------------------------------------------------------------
# weight re-layout cache
# --------------------------------------------------------------------------------------------------
def _prepped(weight: torch.Tensor, geom: L.ConvGeom, mode: int, Ci: int, Co: int, KH: int, KW: int,
             pad: int, mask: Optional[torch.Tensor] = None, key_extra=()) -> torch.Tensor:
    rows = Co if mode in (L.WPREP_CONV, L.WPREP_DECONV) else Ci
    cols = Ci if mode in (L.WPREP_CONV, L.WPREP_DECONV) else Co
    if mask is not None:  # masked weights are re-laid-out every call (the mask is applied on the fly)
        buf = _empty((rows, geom.ntaps * cols), weight.device)
        L.call("hyres_conv_weight_prep", ctypes.byref(geom), weight.data_ptr(), buf.data_ptr(), mode, Ci, Co,
               KH, KW, pad, mask.data_ptr(), L.stream())
        return buf
    key = (mode, geom.nphase, geom.ntaps) + tuple(key_extra)
    cache = getattr(weight, "_hyres_prep", None)
    if cache is None:
        cache = {}
        try:
            weight._hyres_prep = cache
        except Exception:
            pass
    stamp = (weight.data_ptr(), weight._version, _WEIGHT_EPOCH[0])
    ent = cache.get(key)
    if ent is not None and ent[0] == stamp:
        return ent[1]
    if ent is not None and PrepBatch.run(weight.device):  # re-lays out every registered weight at once
        ent = cache.get(key)
        if ent[0] == stamp:
            return ent[1]
    buf = ent[1] if ent is not None else _empty((rows, geom.ntaps * cols), weight.device)
    L.call("hyres_conv_weight_prep", ctypes.byref(geom), weight.data_ptr(), buf.data_ptr(), mode, Ci, Co,
           KH, KW, pad, None, L.stream())
    cache[key] = (stamp, buf)
    PrepBatch.register(weight, key, geom, buf, mode, Ci, Co, KH, KW)
    return buf


class PrepBatch:
    """All cached conv-weight re-layouts of a device as ONE batched launch per weight epoch (i.e. per
    optimiser step) instead of one small launch per layer and layout. Entries are registered on their first
    individual prep; the device descriptor table is (re)built outside graph capture, and the batch is run
    at the first cache miss of a new epoch, after which every registered entry is stamped fresh."""

    _state = {}  # device index -> dict(entries, table, n, total, epoch, dirty)

    @classmethod
    def register(cls, weight, key, geom, buf, mode, Ci, Co, KH, KW) -> None:
        if weight.device.type != "cuda":
            return
        st = cls._state.setdefault(weight.device.index, {"entries": {}, "table": None, "epoch": -1, "dirty": False,
                                                         "order": []})
        ek = (id(weight), key)
        ent = st["entries"].get(ek)
        if ent is None or ent[0]() is not weight or ent[3]() is not buf:
            g = L.ConvGeom()
            ctypes.memmove(ctypes.byref(g), ctypes.byref(geom), ctypes.sizeof(g))
            st["entries"][ek] = (weakref.ref(weight), key, g, weakref.ref(buf), mode, Ci, Co, KH, KW,
                                 weight.data_ptr(), buf.data_ptr())
            st["dirty"] = True

    @classmethod
    def _build(cls, st, device) -> None:
        lib = L.load()
        dsz = int(lib.hyres_prep_desc_bytes())
        live = {}
        for ek, e in st["entries"].items():
            w, buf = e[0](), e[3]()
            if w is not None and buf is not None and w.data_ptr() == e[9] and buf.data_ptr() == e[10]:
                live[ek] = e
        st["entries"] = live
        ents = [(e[0](), e[1], e[2], e[3](), *e[4:9]) for e in live.values()]
        if not ents:
            st.update(table=None, n=0, total=0, order=[], dirty=False)
            return
        host = (ctypes.c_ubyte * (dsz * len(ents)))()
        begin = 0
        for i, (w, key, g, buf, mode, Ci, Co, KH, KW) in enumerate(ents):
            cnt = ctypes.c_longlong(0)
            L.check(lib.hyres_prep_desc_fill(ctypes.addressof(host) + i * dsz, ctypes.byref(g), w.data_ptr(),
                                             buf.data_ptr(), mode, Ci, Co, KH, KW, begin, ctypes.byref(cnt)),
                    "hyres_prep_desc_fill")
            begin += cnt.value
        t = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(device)
        order = [(weakref.ref(e[0]), e[1], weakref.ref(e[3]), e[0].data_ptr(), e[3].data_ptr()) for e in ents]
        st.update(table=t, n=len(ents), total=begin, order=order, dirty=False)

    @staticmethod
    def _stale(st) -> bool:
        for wr, key, br, wp, bp in st["order"]:
            w, b = wr(), br()
            if w is None or b is None or w.data_ptr() != wp or b.data_ptr() != bp:
                return True
        return False

    @classmethod
    def table(cls, device) -> Optional[torch.Tensor]:
        """The current device descriptor table (a captured graph that recorded the batch launch holds it: a
        later eager rebuild must not free the table the graph's kernel reads)."""
        st = cls._state.get(device.index) if device.type == "cuda" else None
        return None if st is None else st["table"]

    @classmethod
    def prepare(cls, device) -> None:
        """Build the descriptor table now (outside graph capture) so a capture can record the batch."""
        st = cls._state.get(device.index) if device.type == "cuda" else None
        if st is not None and (st["dirty"] or st["table"] is None or cls._stale(st)):
            cls._build(st, device)

    @classmethod
    def run(cls, device) -> bool:
        st = cls._state.get(device.index) if device.type == "cuda" else None
        if st is None or st["epoch"] == _WEIGHT_EPOCH[0]:
            return False
        capturing = torch.cuda.is_current_stream_capturing()
        if st["dirty"] or st["table"] is None or cls._stale(st):
            if capturing:
                return False  # the table upload is a host->device copy: prep individually this time
            cls._build(st, device)
            if st["table"] is None:
                return False
        st["epoch"] = _WEIGHT_EPOCH[0]
        L.call("hyres_conv_weight_prep_batch", st["table"].data_ptr(), st["n"], st["total"], L.stream())
        for wr, key, br, _, _ in st["order"]:
            w = wr()
            w._hyres_prep[key] = ((w.data_ptr(), w._version, _WEIGHT_EPOCH[0]), br())
        return True


def _ws(nbytes: int, device, slot=0) -> torch.Tensor:
    return Workspace.get(int(nbytes), device, slot)


def _geom(fn: str, *args) -> L.ConvGeom:
    g = L.ConvGeom()
    L.call(fn, ctypes.byref(g), *[int(a) for a in args])
    return g


def _live_taps(mask: torch.Tensor):
    """Host copy of a spatial mask's live taps (KH*KW uint8), cached on the mask tensor.  Valid when the
    mask is the same for every (out, in) channel pair, as CheckboardMaskedConv2d's is."""
    keep = getattr(mask, "_hyres_keep", None)
    if keep is None:
        m = mask.detach().to("cpu")
        KW = m.shape[-1]
        plane = m[0, 0]
        assert torch.equal((m != 0), (plane != 0).expand_as(m)), "mask must be channel-independent"
        keep = ((ctypes.c_ubyte * plane.numel())(*[int(v != 0) for v in plane.flatten().tolist()]), KW)
        try:
            mask._hyres_keep = keep
        except Exception:
            pass
    return keep


def _filter_taps(g: L.ConvGeom, mask: Optional[torch.Tensor]) -> L.ConvGeom:
    if mask is not None:
        keep, KW = _live_taps(mask)
        L.call("hyres_geom_filter_taps", ctypes.byref(g), keep, KW)
    return g


class KernelTimer:
    """Optional HIP-event timing of conv_fwd_kernel launches, grouped by template instantiation (the same
    selection hyres_conv_forward makes), with their algorithmic FLOPs/bytes; ``summary`` reports the
    instantiation with the largest total time (the dominant kernel of bench.py's roofline line)."""

    enabled = False
    all_convs = False  # record every conv launch (layer table), not only the dominant variant
    events: list = []
    table: list = []

    @classmethod
    def reset(cls):
        cls.events = []
        cls.table = []

    @classmethod
    def groups(cls):
        """{instantiation: [total ms, FLOPs, algorithmic bytes, launches]} of the recorded launches."""
        torch.cuda.synchronize()
        groups = {}
        for s0, s1, fl, by, var in cls.events:
            e = groups.setdefault(var, [0.0, 0.0, 0.0, 0])
            e[0] += s0.elapsed_time(s1)
            e[1] += fl
            e[2] += by
            e[3] += 1
        return groups

    @classmethod
    def summary(cls, pick=None):
        """The instantiation with the largest total time (or the largest among those ``pick(name, group)``
        accepts)."""
        groups = cls.groups()
        if pick is not None:
            groups_all = groups
            groups = {k: v for k, v in groups.items() if pick(k, v)}
        if not groups:
            return {"kernel": None, "launches": 0, "total_ms": 0.0, "avg_us": 0.0, "flops": 0.0,
                    "flops_per_launch": 0.0, "bytes_per_launch": 0.0}
        var, (ms, flops, nbytes, n) = max(groups.items(), key=lambda kv: kv[1][0])
        if pick is not None:
            groups = groups_all
        return {"kernel": var, "launches": n, "total_ms": ms, "avg_us": 1000.0 * ms / n, "flops": flops,
                "flops_per_launch": flops / n, "bytes_per_launch": nbytes / n,
                "by_variant_ms": {k: round(v[0], 3) for k, v in groups.items()},
                "by_variant": {k: list(v) for k, v in groups.items()}}


def conv_variant(g: L.ConvGeom, e: L.Epilogue, splitk: bool) -> str:
    """The kernel hyres_conv_forward launches for (g, e), named by the launcher itself
    (hyres_conv_kernel_name: the same choice function, so the label cannot drift from the routing)."""
    buf = ctypes.create_string_buffer(96)
    L.call("hyres_conv_kernel_name", ctypes.byref(g), ctypes.byref(e), int(bool(splitk)), buf, len(buf))
    return buf.value.decode()


def conv_split(g: L.ConvGeom, e: L.Epilogue) -> int:
    """The split-K factor hyres_conv_forward will use for (g, e) (1 = fused epilogue)."""
    tile, ns = ctypes.c_int(0), ctypes.c_int(1)
    L.call("hyres_conv_plan", ctypes.byref(g), ctypes.byref(e), ctypes.byref(tile), ctypes.byref(ns))
    return ns.value


def conv_flops(g: L.ConvGeom) -> float:
    taps = sum(g.ntap[p] for p in range(g.nphase))
    return 2.0 * g.B * g.Hq * g.Wq * taps * g.Ci * g.Co


def conv_bytes(g: L.ConvGeom, e: L.Epilogue) -> float:
    """Algorithmic HBM bytes: input read once, weights once, output written (read too if accumulating),
    residual / aux operands read once — each at its storage width (``io_f16``: fp16 X; fp16 Y with its
    res / aux0 / out2 operands; fp16 saved activations aux0 / aux2 of a backward conv)."""
    px_in = g.B * g.Hi * g.Wi
    px_out = g.B * g.Hq * g.Wq * g.nphase
    io = int(e.io_f16)
    xw = 2.0 if io & L.IO_X16 else 4.0
    yw = 2.0 if io & L.IO_Y16 else 4.0
    auxw = 2.0 if io & (L.IO_Y16 | L.IO_AUX16) else 4.0
    b = xw * px_in * g.Ci + 4.0 * g.ntaps * g.Ci * g.Co + yw * px_out * g.Co * (2 if e.accumulate else 1)
    b += px_out * g.Co * (yw * sum(1 for p in (e.res, e.out2) if p) + auxw * (1 if e.aux0 else 0)
                          + 4.0 * (1 if e.aux1 else 0) + (auxw if io & L.IO_AUX16 else 4.0) * (1 if e.aux2 else 0))
    return b


AMP_WGRAD_F16 = int(os.environ.get("HYRES_AMP_WGRAD_F16", "1") == "1")


def f16_convs() -> bool:
    """``torch.autocast("cuda", dtype=torch.float16)`` is active (the reference's AMP path, train.sh
    --mixed-precision -> src/utils/engine.py:32, BASELINE configs[4]): convolutions started now take fp16
    operands on the f16 MFMA (fp32 accumulation, fp32 activations in HBM) — the forward conv and, decided
    at forward time like autocast's fp16 conv backward, its input-gradient and weight-gradient GEMMs
    (HYRES_AMP_WGRAD_F16=0 keeps the weight gradients in fp32)."""
    return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.float16


F16_ACT = os.environ.get("HYRES_F16_ACT", "1") == "1"
# PReLU backward folded into the input-gradient conv that writes the PReLU output's gradient (Node.prelu_mask_epilogue);
# HYRES_FOLD_PRELU=0: the separate prelu_bwd pass (A/B)
FOLD_PRELU = os.environ.get("HYRES_FOLD_PRELU", "1") == "1"
# a residual-branch gradient deferred into the next input-gradient conv's epilogue also when the node already holds a
# gradient (Node.defer_residual); HYRES_DEFER_ON_GRAD=0: only as the first contribution (A/B)
DEFER_ON_GRAD = os.environ.get("HYRES_DEFER_ON_GRAD", "1") == "1"
# AMP training stores the f16_region's activations (forward outputs saved for backward) as fp16 too, like
# torch autocast, whose conv outputs are fp16 tensors (src/utils/engine.py:32); gradients stay fp32
AMP_F16_ACT = os.environ.get("HYRES_AMP_F16_ACT", "1") == "1"
# ... and their gradients fp16 (autocast's own semantics; Node.ghalf)
AMP_F16_GRAD = os.environ.get("HYRES_AMP_F16_GRAD", "1") == "1"
_F16_REGION = [0]


@contextlib.contextmanager
def f16_region():
    """Marks the sub-graphs whose activations may live as fp16 in HBM: g_a above the latent resolution,
    g_s after its latent AttentionBlock, MultiScaleRefine (models/checkerboard.py, models/hyres.py)."""
    _F16_REGION[0] += 1
    try:
        yield
    finally:
        _F16_REGION[0] -= 1


def act_f16(tape: Optional["Tape"], H: int, W: int) -> bool:
    """Store this activation as fp16 in HBM under ``torch.autocast(float16)`` inside an ``f16_region``: inference
    (the reference's C5 configuration, "fp16 activations": autocast makes every conv output fp16) and AMP
    training (train.sh --mixed-precision; HYRES_AMP_F16_ACT=0 keeps fp32 activations there), where the saved
    activations are then read as fp16 by the backward kernels while gradients stay fp32. The latent-resolution
    entropy path (y, h_a, h_s, context, param_aggregation, the likelihoods, the rANS symbols) stays fp32, so
    encoder and decoder index the same CDFs at any image size. Arithmetic stays fp32 inside every kernel;
    HYRES_F16_ACT=0 keeps fp32 activations everywhere (fp16 operands only)."""
    return (tape is None or AMP_F16_ACT) and _F16_REGION[0] > 0 and F16_ACT and f16_convs()


def _io_flags(x: "Node", y: "Node", tape: Optional["Tape"]) -> int:
    return (L.IO_X16 if x.half else 0) | (L.IO_Y16 if y.half else 0)


def _launch_conv(g: L.ConvGeom, x_ptr: int, w2: torch.Tensor, ldw: int, y_ptr: int, e: L.Epilogue) -> None:
    nb = L.load().hyres_conv_workspace_bytes(ctypes.byref(g))  # > 0 iff a split-K plan exists
    timed = KernelTimer.enabled
    if timed:
        s0 = torch.cuda.Event(enable_timing=True)
        s1 = torch.cuda.Event(enable_timing=True)
        s0.record()
    ws = _ws(nb, w2.device, slot=6) if nb > 0 else None
    L.call("hyres_conv_forward", ctypes.byref(g), x_ptr, w2.data_ptr(), ldw, y_ptr, ctypes.byref(e),
           None if ws is None else ws.data_ptr(), 0 if ws is None else ws.numel(), L.stream())
    if timed:
        s1.record()
        KernelTimer.events.append((s0, s1, conv_flops(g), conv_bytes(g, e), conv_variant(g, e, conv_split(g, e) > 1)))
        if KernelTimer.all_convs:
            desc = (f"B{g.B} {g.Hi}x{g.Wi}x{g.Ci}->{g.Ho}x{g.Wo}x{g.Co} taps{g.ntaps} ph{g.nphase} "
                    f"s{g.ish} epi{e.kind}{'+acc' if e.accumulate else ''}{'+res' if e.res else ''}"
                    f"{'+mask' if e.act == L.ACT_RELU_MASK else ''}{' io%d' % e.io_f16 if e.io_f16 else ''} "
                    f"[{conv_variant(g, e, conv_split(g, e) > 1)}{'' if x_ptr % 16 == 0 else ', x not 16B-aligned'}]")
            KernelTimer.table.append((desc, s0, s1, conv_flops(g), conv_bytes(g, e)))


def _colsum_into(g: torch.Tensor, P: int, C: int, ld: int, dst: torch.Tensor, acc: int = 1) -> None:
    ws = _ws(L.load().hyres_colsum_workspace_bytes(P, C), g.device, slot=1)
    fn = "hyres_colsum_f16" if g.dtype == torch.float16 else "hyres_colsum"
    L.call(fn, g.data_ptr(), P, C, ld, dst.data_ptr(), acc, ws.data_ptr(), ws.numel(), L.stream())


def _dgrad_io(gp: torch.Tensor, x: "Node") -> int:
    """io_f16 of an input-gradient conv: X = the incoming gradient ``gp``, Y = x's gradient, the ReLU mask (x's
    values) fp16 with Y or alone (AUX16: fp16 activation, fp32 gradient)."""
    io = (L.IO_X16 if gp.dtype == torch.float16 else 0) | (L.IO_Y16 if x.ghalf else 0)
    if x.half and not x.ghalf:
        io |= L.IO_AUX16
    return io


class SideStream:
    """Weight gradients are independent of the input-gradient chain: with HYRES_SIDE_STREAM=1 conv/deconv
    wgrads run on a side HIP stream (forked from the main stream at the point their operands are ready,
    joined at the end of the tape backward).  Off by default since round 2: under graph replay the
    concurrent wgrads cost more in contention with the big dgrad convs than they fill (C2 step 44.4 ->
    43.0 ms fp32, 28.8 -> 28.2 ms AMP with it off; scripts/stream_policy.sh, profiles/r2_stream_policy.txt).
    Operand tensors are ``record_stream``-ed so the caching allocator does not recycle them early;
    the side stream owns workspace slot 2."""

    enabled = os.environ.get("HYRES_SIDE_STREAM", "0") == "1"
    count = 1  # weight-gradient streams (round robin)
    _streams = {}
    _rr = 0
    used = False

    @classmethod
    def get(cls, device: torch.device, rotate: bool = False) -> torch.cuda.Stream:
        sts = cls._streams.get(device.index)
        if sts is None:
            sts = [torch.cuda.Stream(device=device) for _ in range(cls.count)]
            cls._streams[device.index] = sts
        if rotate:
            cls._rr = (cls._rr + 1) % len(sts)
        return sts[cls._rr % len(sts)]

    @classmethod
    def all(cls, device: torch.device) -> list:
        cls.get(device)
        return list(cls._streams[device.index])

    @classmethod
    def join(cls) -> None:
        """Make the current stream wait for all side-stream work (end of backward)."""
        if not cls.used:
            return
        for idx, sts in cls._streams.items():
            for st in sts:
                torch.cuda.current_stream(torch.device("cuda", idx)).wait_stream(st)
        cls.used = False


class WgradBatch:
    """Deferred split-K reduces of the weight gradients (round 3, HYRES_WGRAD_DEFER=0 turns it off).

    A weight gradient is a GEMM over the batch's pixels split into [nsplit][taps][M][N] partial slabs; the
    per-layer path launches one small deterministic reduce per layer (~130 per C2 step, 8-40 us each, mostly
    ramp and tail). Here each layer launches only its GEMM into a slab of its own, and the reduces of every
    layer issued on a stream run as ONE ``hyres_wgrad_reduce_jobs`` launch (bit-identical results: same split
    plan and per-output summation order) when the stream's gradients must be final: at a GradReady marker
    (before the all-reduce listeners), when a branch stream is left, at the end of the tape backward, when a
    new job would write a destination a pending job writes, when HYRES_WGRAD_MAX_JOBS are pending, or when the
    pending slabs would exceed ``max_bytes`` (they are caching-allocator blocks that stay alive until the flush,
    inside a captured graph's pool too: the cap bounds that extra peak memory; scripts/mem_probe.py measures it)."""

    enabled = os.environ.get("HYRES_WGRAD_DEFER", "1") == "1"
    max_bytes = 256 << 20
    _pending = {}  # stream handle -> {"jobs": [WgradJob], "keep": [tensors], "ranges": [(lo, hi)]}

    @classmethod
    def _entry(cls, handle: int) -> dict:
        ent = cls._pending.get(handle)
        if ent is None:
            ent = {"jobs": [], "keep": [], "ranges": [], "bytes": 0}
            cls._pending[handle] = ent
        return ent

    @classmethod
    def launch(cls, desc: L.WgradDesc, p_ptr: int, q_ptr: int, dst: torch.Tensor, device,
               dbias: Optional[torch.Tensor]) -> None:
        lib = L.load()
        nbytes = int(lib.hyres_wgrad_workspace_bytes(ctypes.byref(desc)))
        stream = L.stream()
        ent = cls._entry(int(stream.value or 0))
        outs = [(dst.data_ptr(), dst.data_ptr() + 4 * dst.numel())]
        if dbias is not None:
            outs.append((dbias.data_ptr(), dbias.data_ptr() + 4 * dbias.numel()))
        if any(lo < h and l < hi for lo, hi in outs for l, h in ent["ranges"]) or \
                len(ent["jobs"]) + 2 > L.WGRAD_MAX_JOBS or ent["bytes"] + nbytes > cls.max_bytes:
            cls._flush_entry(ent, stream)
        ws = torch.empty((max(nbytes, 16),), dtype=torch.uint8, device=device)
        jobs = (L.WgradJob * 2)()
        nj = ctypes.c_int(0)
        L.call("hyres_conv_wgrad_deferred", ctypes.byref(desc), p_ptr, q_ptr, dst.data_ptr(),
               None if dbias is None else dbias.data_ptr(), ws.data_ptr(), ws.numel(), jobs, ctypes.byref(nj),
               stream)
        if nj.value:
            ent["jobs"].extend(jobs[i] for i in range(nj.value))
            ent["keep"].append(ws)
            ent["ranges"].extend(outs)
            ent["bytes"] += nbytes

    @classmethod
    def _flush_entry(cls, ent: dict, stream) -> None:
        if ent["jobs"]:
            arr = (L.WgradJob * len(ent["jobs"]))(*ent["jobs"])
            L.call("hyres_wgrad_reduce_jobs", arr, len(ent["jobs"]), stream)
        ent["jobs"].clear()
        ent["keep"].clear()  # stream-ordered: the caching allocator reuses the slabs after the reduce
        ent["ranges"].clear()
        ent["bytes"] = 0

    @classmethod
    def flush(cls) -> None:
        """Run the current stream's pending reduces (its weight gradients are final after this, in stream
        order)."""
        if not cls._pending:
            return
        stream = L.stream()
        ent = cls._pending.get(int(stream.value or 0))
        if ent is not None and ent["jobs"]:
            cls._flush_entry(ent, stream)

    @classmethod
    def pending(cls) -> int:
        return sum(len(e["jobs"]) for e in cls._pending.values())


def _wgrad(desc: L.WgradDesc, p_ptr: int, q_ptr: int, dst: torch.Tensor, device,
           dbias: Optional[torch.Tensor] = None, keep=(), side: bool = False, defer: bool = True) -> None:
    """Weight gradient (+ the bias gradient = column sums of P when ``dbias`` is given, conv2d only).
    ``side``: run on the side stream (``keep`` = tensors whose memory the kernels read). ``defer``: the
    split-K reduce may be batched (WgradBatch); False when a kernel of this backward reads ``dst``."""
    side = side and SideStream.enabled and device.type == "cuda"
    if side:
        main = torch.cuda.current_stream(device)
        st = SideStream.get(device, rotate=True)
        st.wait_stream(main)
        for t in tuple(keep) + (dst,) + ((dbias,) if dbias is not None else ()):
            t.record_stream(st)
        SideStream.used = True
        with torch.cuda.stream(st):
            _wgrad_launch(desc, p_ptr, q_ptr, dst, device, dbias, slot=2)
    elif defer and WgradBatch.enabled and device.type == "cuda" and not (KernelTimer.enabled and KernelTimer.all_convs):
        WgradBatch.launch(desc, p_ptr, q_ptr, dst, device, dbias)
    else:
        _wgrad_launch(desc, p_ptr, q_ptr, dst, device, dbias, slot=7)


def _wgrad_launch(desc, p_ptr, q_ptr, dst, device, dbias, slot):
    nbytes = L.load().hyres_wgrad_workspace_bytes(ctypes.byref(desc))
    ws = _ws(nbytes, device, slot=slot)
    timed = KernelTimer.enabled and KernelTimer.all_convs
    if timed:
        s0 = torch.cuda.Event(enable_timing=True)
        s1 = torch.cuda.Event(enable_timing=True)
        s0.record()
    L.call("hyres_conv_wgrad", ctypes.byref(desc), p_ptr, q_ptr, dst.data_ptr(),
           None if dbias is None else dbias.data_ptr(), ws.data_ptr(), ws.numel(), L.stream())
    if timed:
        s1.record()
        d = desc
        q = d.B * d.Hq * d.Wq
        flops = 2.0 * q * d.ntaps * d.M * d.N
        nbytes_alg = ((2.0 if d.io_f16 & 1 else 4.0) * q * d.M + (2.0 if d.io_f16 & 2 else 4.0) * d.B * d.Hqq * d.Wqq * d.N
                      + 4.0 * d.ntaps * d.M * d.N)
        name = (f"WGRAD B{d.B} P {d.Hq}x{d.Wq}x{d.M} Q {d.Hqq}x{d.Wqq}x{d.N} taps{d.ntaps} sq{d.sq}"
                f"{' sqr' if d.square_q else ''}")
        KernelTimer.table.append((name, s0, s1, flops, nbytes_alg))


def _act_backward(y: Node, gy: torch.Tensor, gy_ld: int, act: int, pre: Optional[torch.Tensor],
                  slope: Optional[torch.Tensor]):
    """Gradient wrt the pre-activation (contiguous [P,C] buffer or the incoming view)."""
    if act == L.ACT_NONE or (act == L.ACT_RELU and y.gmasked) or (act == L.ACT_PRELU and y.pmasked):
        return gy, gy_ld
    gp = _empty((y.B, y.H, y.W, y.C), y.device, gy.dtype)
    g16 = int(gy.dtype == torch.float16)
    if act == L.ACT_RELU:
        if y.half:
            L.call("hyres_relu_bwd_2d_f16", y.ptr(), y.ld, gy.data_ptr(), gy_ld, gp.data_ptr(), y.C, y.P, y.C, g16,
                   L.stream())
        else:
            L.call("hyres_relu_bwd_2d", y.ptr(), y.ld, gy.data_ptr(), gy_ld, gp.data_ptr(), y.C, y.P, y.C, L.stream())
    else:
        ws = _ws(L.load().hyres_reduce_workspace_bytes(y.P * y.C), y.device, slot=1)
        dslope = param_grad(slope) if slope.requires_grad else _empty((1,), y.device)
        if pre.dtype == torch.float16:
            L.call("hyres_prelu_bwd_f16", pre.data_ptr(), y.C, gy.data_ptr(), gy_ld, gp.data_ptr(), y.C, y.P, y.C,
                   slope.data_ptr(), dslope.data_ptr(), ws.data_ptr(), ws.numel(), g16, L.stream())
        else:
            L.call("hyres_prelu_bwd", pre.data_ptr(), y.C, gy.data_ptr(), gy_ld, gp.data_ptr(), y.C, y.P, y.C,
                   slope.data_ptr(), dslope.data_ptr(), ws.data_ptr(), ws.numel(), L.stream())
    return gp, y.C


# --------------------------------------------------------------------------------------------------
# convolutions
# --------------------------------------------------------------------------------------------------
def conv2d(tape: Optional[Tape], x: Node, weight: torch.Tensor, bias: Optional[torch.Tensor], stride=1,
           pad=0, dil=1, act=L.ACT_NONE, slope=None, res: Optional[Node] = None, out: Optional[Node] = None,
           mask: Optional[torch.Tensor] = None, computed: bool = False,
           rowscale: Optional[torch.Tensor] = None) -> Node:
    """nn.Conv2d (+ fused bias / residual / ReLU / PReLU epilogue), NHWC, on MFMA.

    Reference call sites: models/layers/common.py:4-11, compressai conv() (k5 s2 p2),
    models/layers/enhancement.py:44-51 (dilated 3x3), :65-82; ResidualUnit's ``out += identity; relu``
    (models/layers/attention.py:26-29) and RBB's ``out + identity`` are the fused residual epilogue.
    ``mask`` implements CheckboardMaskedConv2d's weight masking (models/layers/checkerboard.py:46-47).
    A 1x1 conv may read only the first x.C of the weight's input channels (param_aggregation on
    ``cat([latent_params, zeros])``, models/checkerboard.py:115-117: the zero half contributes nothing).
    ``rowscale`` (inference, 1x1 only): conv(x * s[pixel]) formed as s[pixel] * conv_nobias(x) + bias in the
    epilogue (HYRES_EPI_ROWSCALE) — SpatialAttention's multiply ahead of MultiScaleRefine's fusion 1x1
    (enhancement.py:105-109) without writing and re-reading the scaled 192-channel map."""
    Co, Ci_w, KH, KW = weight.shape
    Ci = x.C
    assert Ci == Ci_w or (KH == 1 and KW == 1 and Ci < Ci_w and mask is None), (Ci_w, x.C)
    B, H, W = x.B, x.H, x.W
    Ho = (H + 2 * pad - dil * (KH - 1) - 1) // stride + 1
    Wo = (W + 2 * pad - dil * (KW - 1) - 1) // stride + 1
    ydt = torch.float16 if Co > 4 and act_f16(tape, Ho, Wo) else torch.float32
    y = out if out is not None else Node.new(B, Ho, Wo, Co, x.device, dtype=ydt)
    assert (y.B, y.H, y.W, y.C) == (B, Ho, Wo, Co), ((y.B, y.H, y.W, y.C), (B, Ho, Wo, Co))
    g = _filter_taps(_geom("hyres_geom_conv2d", B, H, W, Ci, x.ld, Co, y.ld, KH, KW, stride, pad, dil), mask)
    if (KH == 1 and KW == 1 and mask is None) or computed:
        w2, ldw = weight, Ci_w  # OIHW == OHWI for 1x1 (computed: no forward launch, no re-layout)
    else:
        w2, ldw = _prepped(weight, g, L.WPREP_CONV, Ci, Co, KH, KW, pad, mask), g.ntaps * Ci
    e = L.Epilogue()
    e.kind = L.EPI_BIAS
    e.act = act
    e.bias = L.ptr(bias)
    if rowscale is not None:
        assert tape is None and KH == 1 and KW == 1 and stride == 1 and rowscale.dtype == torch.float32
        assert rowscale.numel() == B * Ho * Wo and rowscale.is_contiguous()
        e.kind = L.EPI_ROWSCALE
        e.aux1, e.ld1 = rowscale.data_ptr(), 1
    if res is not None:
        assert (res.B, res.H, res.W, res.C) == (B, Ho, Wo, Co) and res.half == y.half
        e.res = res.ptr()
        e.ldres = res.ld
    e.io_f16 = _io_flags(x, y, tape)
    pre = None
    if act == L.ACT_PRELU:
        e.slope = slope.data_ptr()
        if tape is not None:
            pre = _empty((B, Ho, Wo, Co), x.device, y.v.dtype)  # stored by the epilogue in y's dtype
            e.out2 = pre.data_ptr()
            e.ldo2 = Co
    f16 = int(f16_convs())
    e.f16_operands = f16
    if computed:  # ``out`` already holds this conv's output (a fused forward): only record the backward
        assert out is not None and pre is None
    else:
        _launch_conv(g, x.ptr(), w2, ldw, y.ptr(), e)
    y.relu_out = act == L.ACT_RELU
    Trace.act(y, act, pre)
    if tape is None:
        return y
    if pre is not None:
        y.prelu = (pre, slope)
        if y.parent is not None:
            y.parent.prelu_slices = (y.parent.prelu_slices or []) + [y]

    def bwd():
        gy = y.grad()
        if gy is None:
            return
        gp, gpld = _act_backward(y, gy, y.grad_ld(), act, pre, slope)
        P = y.P
        if res is not None and res.rg and not res.defer_residual(gp, gpld):
            tgt, acc = res.grad_target()
            add2d(gp, gpld, tgt, res.grad_ld(), P, Co, acc)
        if wants_grad(bias) and not wants_grad(weight):
            _colsum_into(gp, P, Co, gpld, param_grad(bias))
        if wants_grad(weight):
            d = L.WgradDesc()
            L.call("hyres_wgrad_desc_conv2d", ctypes.byref(d), B, H, W, Ci, x.ld, Co, gpld, KH, KW, stride,
                   pad, dil)
            d.sm = Ci_w * KH * KW
            d.accumulate = 1
            d.f16_operands = f16 * AMP_WGRAD_F16
            # P = the (fp16 under AMP) gradient, Q = the saved input activation
            d.io_f16 = (1 if gp.dtype == torch.float16 else 0) | (2 if x.half else 0)
            _wgrad(d, gp.data_ptr(), x.ptr(), param_grad(weight), x.device,
                   param_grad(bias) if wants_grad(bias) else None, keep=(gp, x.v), side=True)
        if x.rg:
            ed = L.Epilogue()
            ed.kind = L.EPI_BIAS
            tgt, acc, _keep = x.grad_target_epi(ed)
            gd = _filter_taps(_geom("hyres_geom_conv2d_dgrad", B, H, W, Ci, x.grad_ld(), Co, gpld, KH, KW, stride,
                                    pad, dil), mask)
            w2d = _prepped(weight, gd, L.WPREP_CONV_DGRAD, Ci_w, Co, KH, KW, pad, mask)
            ed.accumulate = acc
            ed.f16_operands = f16
            ed.io_f16 = _dgrad_io(gp, x)
            x.relu_mask_epilogue(ed, acc)
            x.prelu_mask_epilogue(ed, acc, gd)
            _launch_conv(gd, gp.data_ptr(), w2d, gd.ntaps * Co, tgt.data_ptr(), ed)

    tape.push(bwd)
    return y


def deconv2d(tape: Optional[Tape], x: Node, weight: torch.Tensor, bias: Optional[torch.Tensor], act=L.ACT_NONE,
             out: Optional[Node] = None) -> Node:
    """compressai deconv(): nn.ConvTranspose2d(k5, s2, p2, output_padding=1) as 4 sub-pixel phases.

    Reference call sites: models/checkerboard.py:50,53,57 (g_s) and :70,72 (h_s)."""
    Ci, Co, K, _ = weight.shape
    assert Ci == x.C
    pad = K // 2
    B, H, W = x.B, x.H, x.W
    ydt = torch.float16 if Co > 4 and act_f16(tape, 2 * H, 2 * W) else torch.float32
    y = out if out is not None else Node.new(B, 2 * H, 2 * W, Co, x.device, dtype=ydt)
    g = _geom("hyres_geom_deconv2d", B, H, W, Ci, x.ld, Co, y.ld, K, pad)
    w2 = _prepped(weight, g, L.WPREP_DECONV, Ci, Co, K, K, pad)
    e = L.Epilogue()
    e.kind = L.EPI_BIAS
    e.act = act
    e.bias = L.ptr(bias)
    e.io_f16 = _io_flags(x, y, tape)
    f16 = int(f16_convs())
    e.f16_operands = f16
    _launch_conv(g, x.ptr(), w2, g.ntaps * Ci, y.ptr(), e)
    y.relu_out = act == L.ACT_RELU
    Trace.act(y, act, None)
    if tape is None:
        return y

    def bwd():
        gy = y.grad()
        if gy is None:
            return
        gp, gpld = _act_backward(y, gy, y.grad_ld(), act, None, None)
        if wants_grad(bias):
            _colsum_into(gp, y.P, Co, gpld, param_grad(bias))
        if wants_grad(weight):
            d = L.WgradDesc()
            L.call("hyres_wgrad_desc_deconv2d", ctypes.byref(d), B, H, W, Ci, x.ld, Co, gpld, K, pad)
            d.accumulate = 1
            d.f16_operands = f16 * AMP_WGRAD_F16
            # P = the saved input activation, Q = the (fp16 under AMP) gradient
            d.io_f16 = (1 if x.half else 0) | (2 if gp.dtype == torch.float16 else 0)
            _wgrad(d, x.ptr(), gp.data_ptr(), param_grad(weight), x.device, keep=(gp, x.v), side=True)
        if x.rg:
            ed = L.Epilogue()
            ed.kind = L.EPI_BIAS
            tgt, acc, _keep = x.grad_target_epi(ed)
            gd = _geom("hyres_geom_deconv2d_dgrad", B, H, W, Ci, x.grad_ld(), Co, gpld, K, pad)
            w2d = _prepped(weight, gd, L.WPREP_DECONV_DGRAD, Ci, Co, K, K, pad)
            ed.accumulate = acc
            ed.f16_operands = f16
            ed.io_f16 = _dgrad_io(gp, x)
            x.relu_mask_epilogue(ed, acc)
            x.prelu_mask_epilogue(ed, acc, gd)
            _launch_conv(gd, gp.data_ptr(), w2d, gd.ntaps * Co, tgt.data_ptr(), ed)

    tape.push(bwd)
    return y


def gdn(tape: Optional[Tape], x: Node, beta: torch.Tensor, gamma: torch.Tensor, inverse: bool) -> Node:
    """compressai GDN / IGDN: y = x * rsqrt(conv1x1(x^2, gamma') + beta')  (sqrt for IGDN).

    One MFMA GEMM with an x->x^2 A-prologue and an x*rsqrt(n) epilogue (n saved for backward);
    reparametrisation (NonNegativeParametrizer + LowerBound) in a tiny side kernel.
    Reference call sites: models/checkerboard.py:37,41 (GDN), :52,56 (IGDN)."""
    C = x.C
    assert x.contiguous
    dev = x.device
    bp = _empty((C,), dev)
    gp = _empty((C, C), dev)
    L.call("hyres_gdn_reparam_fwd", beta.data_ptr(), gamma.data_ptr(), bp.data_ptr(), gp.data_ptr(), C, L.stream())
    y = Node.new(x.B, x.H, x.W, C, dev, dtype=x.v.dtype)  # fp16 in -> fp16 out (autocast inference)
    nrm = _empty((x.B, x.H, x.W, C), dev, x.v.dtype)
    g = _geom("hyres_geom_conv2d", x.B, x.H, x.W, C, x.ld, C, C, 1, 1, 1, 0, 1)
    e = L.Epilogue()
    e.kind = L.EPI_IGDN if inverse else L.EPI_GDN
    e.io_f16 = _io_flags(x, y, tape)
    e.square_input = 1
    e.bias = bp.data_ptr()
    e.aux0 = x.ptr()
    e.ld0 = x.ld
    e.out2 = nrm.data_ptr()
    e.ldo2 = C
    f16 = int(f16_convs())
    e.f16_operands = f16
    _launch_conv(g, x.ptr(), gp, C, y.ptr(), e)
    if tape is None:
        return y

    def bwd():
        gy = y.grad()
        if gy is None:
            return
        gld = y.grad_ld()
        if gld != C:
            t = _empty((x.B, x.H, x.W, C), dev, gy.dtype)
            add2d(gy, gld, t, C, y.P, C, 0)
            gy = t
        dn = _empty((x.B, x.H, x.W, C), dev, gy.dtype)  # the norm's gradient: fp16 with y's (AMP)
        if y.half:
            L.call("hyres_gdn_dnorm_f16", gy.data_ptr(), y.ptr(), nrm.data_ptr(), dn.data_ptr(), y.P, C, int(inverse),
                   int(gy.dtype == torch.float16), L.stream())
        else:
            L.call("hyres_gdn_dnorm", gy.data_ptr(), y.ptr(), nrm.data_ptr(), dn.data_ptr(), y.P, C, int(inverse),
                   L.stream())
        if beta.requires_grad or gamma.requires_grad:
            dgp = _empty((C, C), dev)
            d = L.WgradDesc()
            L.call("hyres_wgrad_desc_conv2d", ctypes.byref(d), x.B, x.H, x.W, C, x.ld, C, C, 1, 1, 1, 0, 1)
            d.square_q = 1
            d.accumulate = 0
            d.f16_operands = f16 * AMP_WGRAD_F16
            d.io_f16 = (1 if dn.dtype == torch.float16 else 0) | (2 if x.half else 0)
            _wgrad(d, dn.data_ptr(), x.ptr(), dgp, dev, defer=False)  # read by the reparam backward below
            dbp = _empty((C,), dev)
            _colsum_into(dn, y.P, C, C, dbp, acc=0)
            L.call("hyres_gdn_reparam_bwd", beta.data_ptr(), gamma.data_ptr(), dbp.data_ptr(), dgp.data_ptr(),
                   param_grad(beta).data_ptr(), param_grad(gamma).data_ptr(), C, 1, L.stream())
        if x.rg:
            tgt, acc = x.grad_target()
            gd = _geom("hyres_geom_conv2d_dgrad", x.B, x.H, x.W, C, x.grad_ld(), C, C, 1, 1, 1, 0, 1)
            w2d = _prepped(gp, gd, L.WPREP_CONV_DGRAD, C, C, 1, 1, 0, key_extra=("gdn",))
            ed = L.Epilogue()
            ed.kind = L.EPI_IGDN_BWD if inverse else L.EPI_GDN_BWD
            ed.accumulate = acc
            ed.aux0 = x.ptr()
            ed.ld0 = x.ld
            ed.aux1 = gy.data_ptr()
            ed.ld1 = C
            ed.aux2 = nrm.data_ptr()
            ed.ld2 = C
            ed.f16_operands = f16
            ed.io_f16 = _dgrad_io(dn, x)  # x and the saved norm fp16 (AMP training), gy / dn / x's gradient with them
            _launch_conv(gd, dn.data_ptr(), w2d, C, tgt.data_ptr(), ed)

    tape.push(bwd)
    return y


# the fused ResidualUnit / RBB inference kernel (hyres_ru_fused_f16); tests and bench.py flip it for A/B
RU_FUSED = True


def residual_unit_fused(tape: Optional[Tape], x: Node, c1, c2, c3, final_relu: bool) -> Optional[Node]:
    """ResidualUnit (final_relu, models/layers/attention.py:11-30) / ResidualBottleneckBlock (compressai) forward as
    ONE launch when it applies — autocast with fp16 activations (inference, or AMP training with the fp16 region's
    activations), N = 128, W % 64 == 0 — else None (the caller runs the three convs). c1, c2, c3: the 1x1 N->N/2,
    3x3 N/2->N/2 and 1x1 N/2->N Conv2d modules. In training the launch also writes the two intermediates, and the
    three convs' backward closures are recorded on the tape exactly as the unfused chain records them."""
    if (not RU_FUSED or not x.half or not x.contiguous or x.device.type != "cuda"
            or not f16_convs() or c1.bias is None or c2.bias is None or c3.bias is None):
        return None
    if not L.load().hyres_ru_fused_f16_ok(x.B, x.H, x.W, x.C) or tuple(c2.weight.shape[2:]) != (3, 3):
        return None
    train = tape is not None
    if train and not act_f16(tape, x.H, x.W):
        return None
    y = Node.new(x.B, x.H, x.W, x.C, x.device, rg=train, dtype=torch.float16)
    t1 = t2 = None
    if train:
        t1 = Node.new(x.B, x.H, x.W, x.C // 2, x.device, dtype=torch.float16)
        t2 = Node.new(x.B, x.H, x.W, x.C // 2, x.device, dtype=torch.float16)
    L.call("hyres_ru_fused_f16", x.ptr(), y.ptr(), x.B, x.H, x.W, x.C, c1.weight.data_ptr(), c1.bias.data_ptr(),
           c2.weight.data_ptr(), c2.bias.data_ptr(), c3.weight.data_ptr(), c3.bias.data_ptr(), int(final_relu),
           None if t1 is None else t1.ptr(), None if t2 is None else t2.ptr(), L.stream())
    if not train:
        y.relu_out = final_relu
        return y
    act3 = L.ACT_RELU if final_relu else L.ACT_NONE
    conv2d(tape, x, c1.weight, c1.bias, act=L.ACT_RELU, out=t1, computed=True)
    conv2d(tape, t1, c2.weight, c2.bias, pad=1, act=L.ACT_RELU, out=t2, computed=True)
    return conv2d(tape, t2, c3.weight, c3.bias, act=act3, res=x, out=y, computed=True)


def attn_gate(tape: Optional[Tape], a: Node, b: Node, x: Node) -> Node:
    """AttentionBlock combine (models/layers/attention.py:44-47): out = a * sigmoid(b) + x."""
    assert a.contiguous and b.contiguous and x.contiguous
    n = a.P * a.C
    out = Node.new(a.B, a.H, a.W, a.C, a.device, dtype=a.v.dtype)
    if a.half:
        assert b.half and x.half
        L.call("hyres_attn_gate_fwd_f16", a.ptr(), b.ptr(), x.ptr(), out.ptr(), n, L.stream())
    else:
        L.call("hyres_attn_gate_fwd", a.ptr(), b.ptr(), x.ptr(), out.ptr(), n, L.stream())
    if tape is None:
        return out

    def bwd():
        g = out.grad()
        if g is None:
            return
        ga, acc_a = a.grad_target()
        gb, acc_b = b.grad_target()
        assert acc_a == 0 and acc_b == 0, "gate inputs are single-consumer"
        if a.half:
            assert ga.dtype == gb.dtype == g.dtype
            g16 = int(g.dtype == torch.float16)
            if a.relu_out and a.parent is None and n % 4 == 0:  # the ReLU backward folded in, as below
                L.call("hyres_attn_gate_bwd_relu_f16", a.ptr(), b.ptr(), g.data_ptr(), ga.data_ptr(), gb.data_ptr(), n,
                       g16, L.stream())
                a.gmasked = True
            else:
                L.call("hyres_attn_gate_bwd_f16", a.ptr(), b.ptr(), g.data_ptr(), ga.data_ptr(), gb.data_ptr(), n, g16,
                       L.stream())
        elif a.relu_out and a.parent is None and n % 4 == 0:
            # the last ResidualUnit's ReLU backward folded in: a's gradient leaves here masked (its producer skips it)
            L.call("hyres_attn_gate_bwd_relu", a.ptr(), b.ptr(), g.data_ptr(), ga.data_ptr(), gb.data_ptr(), n,
                   L.stream())
            a.gmasked = True
        else:
            L.call("hyres_attn_gate_bwd", a.ptr(), b.ptr(), g.data_ptr(), ga.data_ptr(), gb.data_ptr(), n, L.stream())
        if x.rg:
            x.set_grad(g)

    tape.push(bwd)
    return out


# --------------------------------------------------------------------------------------------------
# concurrent branches
# --------------------------------------------------------------------------------------------------
class BranchStreams:
    """HIP streams for independent sub-graphs (AttentionBlock's two branches, MultiScaleRefine's three
    scales): a branch's kernels run concurrently with the other branches' in forward and backward."""

    # (default stream priority: a high-priority branch or main stream measured 25-40 % slower steps, round 2;
    # limiting the branches to small grids +1.5 %; those switches were removed in round 4)
    enabled = True
    _streams = {}

    @classmethod
    def get(cls, device: torch.device, k: int) -> torch.cuda.Stream:
        key = (device.index, k)
        st = cls._streams.get(key)
        if st is None:
            st = torch.cuda.Stream(device=device)
            cls._streams[key] = st
        return st


def run_branches(tape: Optional[Tape], x: Node, fns) -> list:
    """``[fn(tape, x_k) for fn in fns]`` with branch k > 0 on its own stream.

    Branch k > 0 reads x through a proxy node with a private gradient buffer; in backward the branches'
    closures are enqueued on their streams (so their kernels overlap), and a join closure (pushed first,
    so it runs last) makes the current stream wait for them and adds the proxies' gradients into x's.
    Forward ends with the current stream waiting for every branch."""
    if not BranchStreams.enabled or x.device.type != "cuda" or len(fns) < 2:
        return [fn(tape, x) for fn in fns]
    dev = x.device
    main = torch.cuda.current_stream(dev)
    n = len(fns)
    proxies = [x] + [Node(x.v, rg=x.rg) for _ in range(n - 1)]
    streams = [main] + [BranchStreams.get(dev, k) for k in range(1, n)]
    if tape is not None:
        def join_bwd():
            cur = torch.cuda.current_stream(dev)
            for k in range(1, n):
                cur.wait_stream(streams[k])
                g = proxies[k].grad()
                if g is not None and x.rg:
                    g.record_stream(cur)
                    x.set_grad(g)
        tape.push(join_bwd)
    fork = torch.cuda.Event()
    fork.record(main)  # x is ready here; branch 0 is enqueued on main after this point
    outs = [fns[0](tape, proxies[0])]
    for k in range(1, n):
        st = streams[k]
        st.wait_event(fork)
        x.v.record_stream(st)
        cell = {}
        if tape is not None:
            def leave(cell=cell):
                WgradBatch.flush()  # the branch's weight gradients, before its stream is joined
                torch.cuda.set_stream(cell["prev"])
            tape.push(leave)
        torch.cuda.set_stream(st)
        try:
            outs.append(fns[k](tape, proxies[k]))
        finally:
            torch.cuda.set_stream(main)
        if tape is not None:
            def enter(st=st, cell=cell):
                cur = torch.cuda.current_stream(dev)
                cell["prev"] = cur
                st.wait_stream(cur)
                torch.cuda.set_stream(st)
            tape.push(enter)
        o = outs[-1]
        if isinstance(o, Node):
            o.v.record_stream(main)
    for k in range(1, n):
        main.wait_stream(streams[k])
    return outs


# --------------------------------------------------------------------------------------------------
# layout boundary
# --------------------------------------------------------------------------------------------------
def to_nhwc(x: torch.Tensor, rg: bool = False) -> Node:
    L.require_device(x)
    x = x.contiguous()
    B, C, H, W = x.shape
    y = Node.new(B, H, W, C, x.device, rg=rg)
    L.call("hyres_nchw_to_nhwc", x.data_ptr(), y.ptr(), B, C, H, W, C, L.stream())
    return y


def to_nchw(x: Node) -> torch.Tensor:
    if x.half:  # fp16 activation (autocast inference): returned as fp32 NCHW
        return x.v.permute(0, 3, 1, 2).float().contiguous()
    out = _empty((x.B, x.C, x.H, x.W), x.device)
    L.call("hyres_nhwc_to_nchw", x.ptr(), x.ld, out.data_ptr(), x.B, x.C, x.H, x.W, L.stream())
    return out


def to_nchw_grad(x: Node) -> torch.Tensor:
    g = x.grad()
    if g.dtype == torch.float16:  # AMP fp16 gradient: returned as fp32 NCHW
        return g.permute(0, 3, 1, 2).float().contiguous()
    out = _empty((x.B, x.C, x.H, x.W), x.device)
    L.call("hyres_nhwc_to_nchw", g.data_ptr(), x.grad_ld(), out.data_ptr(), x.B, x.C, x.H, x.W, L.stream())
    return out


def nchw_grad_to_nhwc(g: torch.Tensor) -> torch.Tensor:
    g = g.contiguous()
    B, C, H, W = g.shape
    y = _empty((B, H, W, C), g.device)
    L.call("hyres_nchw_to_nhwc", g.data_ptr(), y.data_ptr(), B, C, H, W, C, L.stream())
    return y
