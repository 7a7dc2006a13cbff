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


class FlatGradReducer:
    def __init__(self, flat, world_size: int, bucket_bytes: int = 32 << 20, group=None):
        self.flat = flat
        self.world = int(world_size)
        self.group = group
        n = flat.numel
        per = max(1, bucket_bytes // 4)
        self.buckets = [(o, min(n, o + per)) for o in range(0, n, per)]

    def all_reduce(self, async_op: bool = False):
        g = self.flat.grad
        works = []
        for a, b in self.buckets:
            works.append(dist.all_reduce(g[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        for w in works:
            w.wait()
        self._scale(g)

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
