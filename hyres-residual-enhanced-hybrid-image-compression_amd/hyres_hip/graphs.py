"""HIP-graph capture of the device step.

The eager step enqueues ~1,000 kernels through Python (ctypes) per training step and ~350 per eval
forward; the host needs ~28 ms / ~13.5 ms for that at bs=16 256x256, which leaves the GPU idle between
dependent launches (eval is entirely host-bound). Capturing the step once into a HIP graph
(``torch.cuda.CUDAGraph`` = hipGraph on ROCm) and replaying it launches the whole DAG — main stream,
the AttentionBlock / MultiScaleRefine branch streams and the weight-gradient side stream, with their
event edges — in one call.

What is captured and what stays eager:
  * captured: ``forward_device`` (+ RateDistortionLoss + backward for training), i.e. every
    libhyres_hip launch of the reference's forward/backward (models/hyres.py:23-77,
    src/utils/engine.py:33-55);
  * eager: the optimiser (FusedAdam's bias correction reads the host step count), the RCCL gradient
    all-reduce (after the replay, hyres_hip.ddp.FlatGradReducer.all_reduce) and the aux (quantiles) step —
    3-10 launches per step. The graph holds no collective.
Graph-safety of the captured region:
  * weights: the conv weight re-layout cache (hyres_hip.ops._prepped) is invalidated before capture so
    every re-layout kernel is recorded and re-runs on each replay (weights change every optimiser step),
    and again after capture so eager calls never trust a buffer only the graph writes;
  * noise: training draws (EntropyBottleneck z, GaussianConditional y) read a device-resident seed that
    the graph advances (hyres_uniform_noise_dev), so each replay draws fresh U(-1/2, 1/2);
  * inputs x / jpeg_decoded / jpeg_bpp are static device buffers: ``replay(x, jpeg, bpp)`` copies new
    data into them (device-to-device) before launching.
"""
from __future__ import annotations

import contextlib
import gc
import weakref
from typing import Callable, Optional, Sequence

import torch

from . import ops as O


class GraphOutputsAlive(RuntimeError):
    """``CapturedStep.close()`` found a replay output (a tensor in the graph's private pool) still referenced by
    the caller: the graph is NOT reset. Drop every reference to the replay's outputs, then close again."""


def _tensors(obj):
    """Every tensor in a (nested) dict / list / tuple of replay outputs."""
    if isinstance(obj, torch.Tensor):
        yield obj
    elif isinstance(obj, dict):
        for v in obj.values():
            yield from _tensors(v)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            yield from _tensors(v)


# graphs whose close() found live outputs while running as a finalizer: kept here (not reset) until the process ends
_KEPT = []


def _prepare_noise(net: torch.nn.Module, device: torch.device) -> None:
    from .entropy_ops import NoiseSource
    for m in net.modules():
        ns = getattr(m, "noise", None)
        if isinstance(ns, NoiseSource):
            ns._device_seed(device)


class CapturedStep:
    """``forward_device`` (eval) or forward + RD loss + backward (train) of a ResidualJPEGCompression,
    captured once and replayed.

    ``criterion``: a RateDistortionLoss for training capture (None = eval forward under no_grad).
    ``zero_grad``: called after the warm-up runs (their backward accumulated into the gradients).
    ``split_at`` (training): backward-progress markers (hyres_hip.ops.GradReady names, e.g. ``("hyper",)``) at which
    the capture is cut into consecutive graphs sharing one memory pool. ``replay(between=f)`` replays them in order
    and calls ``f(segments)`` between two of them with the marker names whose gradients are final at that point — the
    data-parallel step starts those segments' RCCL all-reduce there, so it runs while the next graph (the rest of
    backward) computes (configs[3]: "grad all-reduce overlapped with backward"; reference src/training.py:211-212,
    src/utils/engine.py:50-56). No collective is inside any graph, and no stream is added: the collective waits on
    the replay stream.
    """

    def __init__(self, net: torch.nn.Module, x: torch.Tensor, jpeg_decoded: torch.Tensor, jpeg_bpp: float = 0.0,
                 noisequant: bool = False, criterion: Optional[Callable] = None,
                 zero_grad: Optional[Callable[[], None]] = None, warmup: int = 2,
                 capture_error_mode: str = "global", amp: bool = False,
                 loss_scale: Optional[torch.Tensor] = None, split_at: Sequence[str] = ()):
        assert x.is_cuda, "CapturedStep needs device tensors"
        self.net = net
        self.train = criterion is not None
        self.split_at = tuple(split_at) if self.train else ()
        dev = x.device
        self.x = x.detach().clone()
        self.jpeg = jpeg_decoded.detach().clone()
        self.bpp = torch.full((), float(jpeg_bpp), dtype=torch.float32, device=dev)
        self.noisequant = noisequant
        self.criterion = criterion
        _prepare_noise(net, dev)

        def run():
            # amp: the forward under torch.autocast(float16) (engine.py:32) -> fp16-operand convolutions;
            # loss_scale: the GradScaler's device scale multiplies the loss before backward (engine.py:51)
            ctx = torch.autocast("cuda", dtype=torch.float16) if amp else contextlib.nullcontext()
            if self.train:
                with ctx:
                    out = net.forward_device(self.x, self.jpeg, self.bpp, noisequant)
                    c = criterion(out, self.x)
                loss = c["loss"] if loss_scale is None else c["loss"] * loss_scale.reshape(())
                loss.backward()
                return out, c
            with torch.no_grad(), ctx:
                return net.forward_device(self.x, self.jpeg, self.bpp, noisequant), None

        # warm-up and capture run on side streams while the parameters' AccumulateGrad nodes were made on
        # the default stream; the stream waits above/below order them, so torch's mismatch warning is noise
        if self.train and hasattr(torch.autograd.graph, "set_warn_on_accumulate_grad_stream_mismatch"):
            torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                run()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        if zero_grad is not None:
            zero_grad()
        self.graphs = [torch.cuda.CUDAGraph() for _ in range(len(self.split_at) + 1)]
        self.graph = self.graphs[0]
        self.segments_done = []  # per cut: the markers whose gradients are final when the graphs before it end
        O.PrepBatch.prepare(dev)  # descriptor table uploaded now: the capture records ONE batched re-layout
        O.bump_weight_epoch()  # record every weight re-layout inside the graph
        # the graph's batched re-layout reads this descriptor table by address: keep it alive for the graph's
        # lifetime (an eager step after the capture may register new entries and rebuild the table)
        self._prep_table = O.PrepBatch.table(dev)
        # "thread_local" when an RCCL process group exists: its watchdog thread polls events while the
        # main thread captures (no collective is ever inside the graph)
        if not self.split_at:
            with torch.cuda.graph(self.graph, capture_error_mode=capture_error_mode):
                self.out, self.crit = run()
        else:
            self.out, self.crit = self._capture_split(run, dev, capture_error_mode)
        # weak references to every output the capture allocated (in the graph's private pool); the static inputs the
        # forward passes through (jpeg_decoded, jpeg_bpp_loss) belong to this object and are not tracked
        own = {t.untyped_storage().data_ptr() for t in (self.x, self.jpeg, self.bpp)}
        self._out_refs = [weakref.ref(t) for t in _tensors((self.out, self.crit))
                          if t.untyped_storage().data_ptr() not in own]
        O.bump_weight_epoch()  # eager calls must not reuse buffers only the graph writes
        # ... and the scratch buffers its kernels were recorded with: an eager call that grows a workspace slot
        # replaces the slot's tensor, and the old one must outlive the graph
        self._ws_keep = list(O.Workspace._bufs.values())
        torch.cuda.synchronize(dev)

    def _capture_split(self, run, dev, capture_error_mode):
        """Capture ``run`` as len(split_at) + 1 graphs: a GradReady listener ends the current capture and begins the
        next one (same memory pool, same capture stream) when a split marker fires in the tape backward — every
        weight-gradient reduce of the finished segments is flushed by the marker first (GradReady.mark), and the
        side stream, if used, is joined so the capture closes with no forked stream open. The markers are placed at
        module boundaries, where the branch streams are joined.

        The capture runs in "relaxed" mode: the cut happens inside the tape backward, i.e. on torch's autograd device
        thread, and a thread-local capture may only be ended by the thread that began it (HIP refuses with
        hipErrorStreamCaptureWrongThread); a global one would treat the RCCL watchdog thread's event polling as an
        unsafe call. Relaxed capture checks neither — no collective and no synchronising call is inside the graphs."""
        capture_error_mode = "relaxed"
        st = {"on": False, "idx": 0, "seen": []}

        def cut(name):
            st["seen"].append(name)
            if not st["on"] or name not in self.split_at:
                return
            O.SideStream.join()
            i = st["idx"]
            self.graphs[i].capture_end()
            self.segments_done.append(list(st["seen"]))
            st["idx"] = i + 1
            self.graphs[i + 1].capture_begin(pool=self.graphs[0].pool(), capture_error_mode=capture_error_mode)

        O.GradReady.listeners.append(cut)  # before the forward: GradReady.mark records markers only with listeners
        try:
            torch.cuda.synchronize(dev)
            gc.collect()
            torch.cuda.empty_cache()
            cap = torch.cuda.Stream(device=dev)
            cap.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(cap):
                st["on"] = True
                self.graphs[0].capture_begin(capture_error_mode=capture_error_mode)
                try:
                    out = run()
                finally:
                    st["on"] = False
                    self.graphs[st["idx"]].capture_end()
            torch.cuda.current_stream(dev).wait_stream(cap)
        finally:
            O.GradReady.listeners.remove(cut)
        if st["idx"] != len(self.split_at):
            raise RuntimeError(f"CapturedStep: split markers {self.split_at} fired {st['idx']} time(s) in the captured "
                               f"backward (markers seen: {st['seen']})")
        return out

    def live_outputs(self) -> int:
        """How many tensors the capture allocated are still alive (held by this object or by a caller)."""
        return sum(1 for r in getattr(self, "_out_refs", ()) if r() is not None)

    def close(self) -> None:
        """Wait for any replay in flight, then destroy the graph and release what it recorded.

        The outputs the capture allocated (``out``, ``crit``, returned by every ``replay()``) live in the graph's
        private memory pool. The lifetime rule: a caller drops every reference to them BEFORE ``close()``, so the pool
        is released with no block of it in use. ``close()`` enforces it: after dropping its own references it checks
        the weak references taken at capture (cycles collected first); if any output is still alive it raises
        ``GraphOutputsAlive`` and leaves the graph and its pool untouched (the step can no longer be replayed; call
        ``close()`` again once the references are gone)."""
        g = getattr(self, "graph", None)
        if g is not None:
            torch.cuda.synchronize(self.x.device)
            self.out, self.crit = None, None
            if self.live_outputs():
                gc.collect()  # an autograd cycle (output -> grad_fn -> ctx -> output) is not a caller reference
            n = self.live_outputs()
            if n:
                raise GraphOutputsAlive(
                    f"CapturedStep.close(): {n} replay output tensor(s) still referenced; drop them before close() "
                    "(the graph was not reset)")
            for gi in reversed(self.graphs):
                gi.reset()
            self.graph = None
            self.graphs = []
        self._prep_table = None
        self._ws_keep = []

    def __del__(self):
        # A finalizer may run while ANOTHER graph is being captured (garbage collection inside the capture): a
        # device synchronize there would invalidate that capture. Owners release graphs with close(); here the
        # graph is only torn down when no capture is in progress, else it is left to the process's end. If a caller
        # still holds replay outputs, the graph (and what it recorded) is parked in _KEPT instead of being reset.
        try:
            if torch.cuda.is_current_stream_capturing():
                return
            self.close()
        except GraphOutputsAlive:
            _KEPT.append((self.graphs, self._prep_table, self._ws_keep))
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def replay(self, x: Optional[torch.Tensor] = None, jpeg_decoded: Optional[torch.Tensor] = None,
               jpeg_bpp: Optional[float] = None, between: Optional[Callable[[list], None]] = None):
        """Run the captured step on the current stream; returns (outputs, loss dict or None) — static
        tensors overwritten by the next replay. A split capture replays its graphs in order and calls
        ``between(markers)`` after each graph but the last (markers: the GradReady names whose gradients are final)."""
        if x is not None:
            self.x.copy_(x, non_blocking=True)
        if jpeg_decoded is not None:
            self.jpeg.copy_(jpeg_decoded, non_blocking=True)
        if jpeg_bpp is not None:
            self.bpp.fill_(float(jpeg_bpp))
        last = len(self.graphs) - 1
        for i, g in enumerate(self.graphs):
            g.replay()
            if between is not None and i < last:
                between(self.segments_done[i])
        return self.out, self.crit
