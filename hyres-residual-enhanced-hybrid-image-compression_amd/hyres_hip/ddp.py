"""Data-parallel gradient path over RCCL (replaces the reference's nn.DataParallel,
src/training.py:211-212 / src/utils/dataset_utils.py:76-82, which is effectively disabled and broken —
SURVEY.md §5).

One process per GPU; each rank runs the full HIP step on its batch shard; the flat fp32 gradient buffer
(hyres_hip.optim.FlatParams, 41.5 MB for N=128/M=192) is all-reduced in a few large buckets (xGMI is
point-to-point: fewer, larger collectives) and averaged, which reproduces the global-batch gradient
because every loss term is a per-rank mean over equally sized shards (DDP caveats).
The aux (quantiles) loss depends only on parameters, so it is identical on every rank: no collective.
Backend "nccl" is RCCL on ROCm; the same code runs over gloo on CPU for the tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib as L


# backward-progress marker (hyres_hip.ops.GradReady, placed in models/hyres.py and models/checkerboard.py)
# -> parameter-name prefixes whose gradients are complete when it fires (backward order: refine, g_s,
# the hyperprior/context group; g_a finishes last and is reduced at the end)
HYRES_SEGMENTS = {
    "refine": ("refine.",),
    "g_s": ("residual_model.g_s.",),
    "hyper": ("residual_model.h_a.", "residual_model.h_s.", "residual_model.entropy_bottleneck.",
              "residual_model.context_prediction.", "residual_model.param_aggregation."),
}


def _split(ranges, per):
    out = []
    for a, b in ranges:
        out.extend((o, min(b, o + per)) for o in range(a, b, per))
    return out


def _merge(ranges):
    out = []
    for a, b in sorted(ranges):
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


class FlatGradReducer:
    """All-reduce (mean) of the flat gradient buffer.

    Without ``names``/``segments``, or after a graph replay: after backward, in ``bucket_bytes`` buckets (the
    default data-parallel step). With them and an EAGER backward (``overlap()``), a segment's
    buckets are launched as soon as its backward-progress marker fires (``on_marker``, a hyres_hip.ops.GradReady
    listener): the RCCL collective is enqueued behind the side stream that carries the weight gradients, so it
    runs while the rest of backward computes. ``all_reduce()`` then reduces whatever no marker covered, waits for
    every collective and scales by 1/world."""

    def __init__(self, flat, world_size: int, bucket_bytes: int = 32 << 20, group=None, names=None,
                 segments=None):
        self.flat = flat
        self.world = int(world_size)
        self.group = group
        n = flat.numel
        self.per = max(1, bucket_bytes // 4)
        self.buckets = _split([(0, n)], self.per)
        self.segments = {}
        covered = []
        if names is not None and segments:
            assert len(names) == len(flat.params)
            for mk, prefixes in segments.items():
                rs = []
                for name, p, o in zip(names, flat.params, flat.offsets):
                    if name.startswith(tuple(prefixes)):
                        rs.append((o, o + (p.numel() + 3) // 4 * 4))
                rs = _merge(rs)
                if rs:
                    self.segments[mk] = _split(rs, self.per)
                    covered.extend(rs)
        covered = _merge(covered)
        rest, cur = [], 0
        for a, b in covered:
            if a > cur:
                rest.append((cur, a))
            cur = max(cur, b)
        if cur < n:
            rest.append((cur, n))
        self.rest = _split(rest, self.per)
        self.fired = []
        self.works = []
        self.armed = True  # gradient accumulation: markers fire only on the boundary micro-batch

    def overlap(self):
        """Register ``on_marker`` as a GradReady listener (eager backward)."""
        from .ops import GradReady
        if self.on_marker not in GradReady.listeners:
            GradReady.listeners.append(self.on_marker)
        return self

    def _launch(self, ranges):
        g = self.flat.grad
        for a, b in ranges:
            self.works.append(dist.all_reduce(g[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def on_marker(self, name: str) -> None:
        ranges = self.segments.get(name)
        if not self.armed or not ranges or name in self.fired:
            return
        self.fired.append(name)
        g = self.flat.grad
        if g.is_cuda:
            from .ops import SideStream
            main = torch.cuda.current_stream(g.device)
            sides = SideStream.all(g.device)
            side = sides[0]
            side.wait_stream(main)  # gradients of this segment: main-stream (dgrad-side) writes + side wgrads
            for other in sides[1:]:
                side.wait_stream(other)
            with torch.cuda.stream(side):
                self._launch(ranges)
        else:
            self._launch(ranges)

    def launch_segments(self, names) -> None:
        """Start the all-reduce of the named segments (those not started yet) on the current stream's order: the
        split-graph step calls it between two replays (hyres_hip.graphs.CapturedStep ``between``), so the
        collectives run while the next graph computes (on an accumulation boundary only: the caller decides, as DDP's
        no_sync). ``all_reduce()`` reduces the rest and waits."""
        for name in names:
            ranges = self.segments.get(name)
            if ranges and name not in self.fired:
                self.fired.append(name)
                self._launch(ranges)

    def all_reduce(self, async_op: bool = False):
        if self.fired:
            ranges = list(self.rest)
            for mk, rs in self.segments.items():
                if mk not in self.fired:
                    ranges.extend(rs)
        else:
            ranges = self.buckets
        self._launch(ranges)
        for w in self.works:
            w.wait()
        self.works = []
        self.fired = []
        self._scale(self.flat.grad)

    def _scale(self, g: torch.Tensor):
        if self.world == 1:
            return
        if g.is_cuda:
            L.call("hyres_scale", g.data_ptr(), None, 1.0 / self.world, g.data_ptr(), g.numel(), 0, L.stream())
        else:  # gloo / CPU tests
            g.mul_(1.0 / self.world)


def broadcast_parameters(module: torch.nn.Module, src: int = 0, group=None):
    """Make every rank start from rank ``src``'s weights (buffers included)."""
    for t in list(module.parameters()) + list(module.buffers()):
        if t.numel():
            dist.broadcast(t.data, src=src, group=group)
