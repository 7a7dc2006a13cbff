"""Train / test loops (src/utils/engine.py:8-202) on the HIP path.

Differences from the reference, by design:
  * the six per-step ``.item()`` host syncs (:42-47) are replaced by device-side metric buffers that are
    read back only when printing (every ``log_every`` steps) — the step itself never syncs;
  * clip_grad_norm_ + Adam are one fused HIP launch (hyres_hip.optim.FusedAdam(max_grad_norm=...));
  * with data parallelism the flat gradient is all-reduced over RCCL before the step (hyres_hip.ddp);
  * ``mixed_precision`` (train.sh:19) keeps the reference's semantics — the forward runs under
    ``torch.autocast("cuda", float16)`` (the HIP convolutions then take fp16 operands on the f16 MFMA with
    fp32 accumulation), the loss is scaled by a GradScaler (init 2^16, growth 2 / 2000 steps, backoff 0.5,
    one per epoch as engine.py:23 creates it), gradients are unscaled before clipping, a step with
    non-finite gradients is skipped and backs the scale off, and a NaN gradient also skips the aux step
    (engine.py:60-74) — with the scaler state, the skip decision and the step count all on the device
    (hyres_hip.optim.DeviceGradScaler), so there is still no per-step host sync.  The reference's NaN
    warning is printed when the metrics are drained;
  * the next batch's host JPEG round trip is started in the background before the current step
    (TurboJPEGCompression.prefetch), so the host JPEG stage overlaps the device step;
  * forward + RD loss + backward replay as a HIP graph (hyres_hip.graphs.CapturedStep, one capture per
    batch shape / noisequant / precision, taken on an accumulation boundary); the host JPEG stage, the
    H2D copies, the gradient all-reduce (after the replay in 32 MB buckets, as bench.py's N > 1 default),
    the optimiser and the aux step stay eager; with HYRES_TRAIN_GRAPH=0 the eager backward overlaps the
    all-reduce segment by segment. Every step the ranks agree over a
    host (gloo) group on the capture key and on capture success, so all ranks replay or all run eagerly and
    issue the same collectives. HYRES_TRAIN_GRAPH=0 runs every step eagerly (the reference's structure);
  * under DDP the test epoch is sharded (rank r takes images r, r + world, ...) and the meters' sums and
    counts are all-reduced, instead of every rank evaluating the whole test set.
"""
import os
import time
from contextlib import nullcontext

import torch

from src.losses import AverageMeter

__all__ = ["train_one_epoch", "test_epoch"]

_KEYS = ("loss", "bpp_loss", "residual_bpp_loss", "y_bpp_loss", "z_bpp_loss", "mse_loss")


def _metrics(out_criterion):
    """Detached device scalars of one step (keeps no reference to the step's autograd graph)."""
    return torch.stack([out_criterion[k].detach().reshape(()).float() for k in _KEYS])


def _drain(pending, meters, nan_flags=None):
    if pending:
        vals = torch.stack(pending).cpu()
        for row in vals:
            for k, v in zip(_KEYS, row.tolist()):
                meters[k].update(v)
        pending.clear()
    if nan_flags:
        for f in torch.cat(nan_flags).cpu().tolist():
            if f != f:  # sum of squares NaN <=> a NaN gradient (engine.py:62-70)
                print("Warning: NaN gradients detected, skipping update step")
        nan_flags.clear()


class _GraphedStep:
    """The drop-in training step's forward + loss + backward as replayed HIP graphs."""

    def __init__(self, model, criterion, device, mixed_precision, accumulation, scaler, zero_grad):
        self.model, self.criterion, self.device = model, criterion, device
        self.amp, self.accum, self.scaler, self.zero_grad = mixed_precision, accumulation, scaler, zero_grad
        self.caps = {}
        # loss multiplier inside the graph: 1/accumulation (x the GradScaler's device scale under AMP)
        self.ls = torch.full((1,), 1.0 / accumulation, dtype=torch.float32, device=device)
        self.enabled = os.environ.get("HYRES_TRAIN_GRAPH", "1") == "1" and device.type == "cuda"
        self.last = None
        self._host_group = host_group()

    def _agree(self, key) -> None:
        """Per-step host check under DDP: every rank must be at the same capture key (same batch shape /
        noisequant / precision), else a replaying rank and an eager or capturing rank would issue different
        collectives and hang. Ranks that agree on the key also agree on whether it still needs a capture (the
        same keys were seen in the same order). One 2-int all-reduce on a gloo group: no device sync."""
        import torch.distributed as dist
        if self._host_group is None:
            return
        h = hash(key) & 0x3FFFFFFF  # tuples of ints / bools hash identically in every process
        t = torch.tensor([h, -h], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self._host_group)
        if int(t[0]) != h or int(-t[1]) != h:
            raise RuntimeError(f"DDP ranks reached different graph-capture keys (this rank {key}); every rank must "
                               "see the same batch shapes (DistributedSampler shards are equal-length)")

    def __call__(self, d, noisequant, boundary_start, reducer, boundary_end=True):
        """Returns the static loss dict of the replayed step, or None (run this step eagerly). With a reducer the
        capture is cut at the "hyper" backward-progress marker (HYRES_DIST_SPLIT=0: one graph) and, on the
        accumulation boundary (``boundary_end``), the finished gradient segments start their all-reduce between the
        two replays, overlapping g_a's backward (bench.py's graph+overlap)."""
        if not self.enabled or d.device.type != "cpu" or not hasattr(self.model, "forward_device"):
            return None
        key = (tuple(d.shape), bool(noisequant), bool(self.amp))
        if reducer is not None:
            self._agree(key)
        cap = self.caps.get(key)
        if cap is None and not boundary_start:
            return None  # capturing zeroes the gradients: only where no partial accumulation exists
        dec, bpp = self.model.jpeg(d)  # host JPEG round trip (prefetched in the background)
        x = d.to(self.device)
        jd = dec.to(self.device)
        if self.scaler is not None:
            torch.mul(self.scaler.scale, 1.0 / self.accum, out=self.ls)
        if cap is None:
            from hyres_hip.graphs import CapturedStep
            armed = reducer.armed if reducer is not None else None
            if reducer is not None:
                reducer.armed = False  # no collective inside warm-up or capture
            err = None
            try:
                split = ("hyper",) if reducer is not None and os.environ.get("HYRES_DIST_SPLIT", "1") == "1" else ()
                cap = CapturedStep(self.model, x, jd, float(bpp), noisequant=noisequant, criterion=self.criterion,
                                   zero_grad=self.zero_grad, amp=self.amp, loss_scale=self.ls,
                                   capture_error_mode="thread_local" if reducer is not None else "global",
                                   split_at=split)
            except Exception as exc:  # noqa: BLE001 - any capture failure: stay correct, run eagerly
                err = exc
            finally:
                if reducer is not None:
                    reducer.armed = armed
            if not _all_ranks_ok(err is None, self._host_group):
                # every rank falls back together: a graphed rank and an eager rank would issue different
                # collectives (segment markers vs buckets) and hang or mix up the all-reduce
                print(f"HIP graph capture failed ({err!r} on this rank); training steps run eagerly")
                self.enabled = False
                self.zero_grad()
                return None
            self.caps[key] = cap
        self.last = cap
        between = reducer.launch_segments if (reducer is not None and boundary_end and cap.split_at) else None
        return cap.replay(x, jd, float(bpp), between=between)[1]

    def close(self) -> None:
        """Release every captured graph explicitly (end of the epoch), not from a finalizer."""
        for cap in self.caps.values():
            cap.close()
        self.caps.clear()
        self.last = None

    def reduce(self, reducer):
        """The boundary all-reduce after a replayed step: the flat gradient in buckets, after the replay."""
        reducer.all_reduce()


_HOST_GROUP = [None, None]  # (default process group it was made for, the gloo group)


def host_group():
    """The host-side (gloo) process group for the per-step agreement all-reduces, created ONCE per process group
    (``dist.new_group`` is itself a collective every rank must issue in the same order, and each group keeps its
    TCP pairs and threads for the life of the run): src/training.py creates it right after
    ``init_process_group``; later calls return the cached group. None without DDP."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return None
    world = dist.group.WORLD
    if _HOST_GROUP[0] is not world:
        _HOST_GROUP[0] = world
        _HOST_GROUP[1] = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else world
    return _HOST_GROUP[1]


def _all_ranks_ok(ok: bool, group) -> bool:
    """Capture success agreed by every rank (MIN over the host gloo group)."""
    import torch.distributed as dist
    if group is None or not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return ok
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return bool(flag.item() == 1)


def _lookahead(loader):
    """(batch, next batch or None) pairs."""
    it = iter(loader)
    cur = next(it, None)
    while cur is not None:
        nxt = next(it, None)
        yield cur, nxt
        cur = nxt


def train_one_epoch(model, criterion, train_dataloader, optimizer, aux_optimizer, epoch, clip_max_norm,
                    noisequant=True, mixed_precision=False, gradient_accumulation_steps=1, reducer=None,
                    log_every=100):
    model.train()
    if hasattr(optimizer, "max_grad_norm"):
        optimizer.max_grad_norm = float(clip_max_norm)
    meters = {k: AverageMeter() for k in _KEYS}
    pending, nan_flags = [], []
    start = time.time()
    device = next(model.parameters()).device
    scaler = None
    if mixed_precision:
        from hyres_hip.optim import DeviceGradScaler
        scaler = DeviceGradScaler(device)  # a fresh scaler per epoch, as engine.py:23
    optimizer.zero_grad()
    aux_optimizer.zero_grad()
    aux_loss = None
    amp = (lambda: torch.autocast("cuda", dtype=torch.float16)) if mixed_precision else nullcontext
    jpeg = getattr(model, "jpeg", None)
    graphed = _GraphedStep(model, criterion, device, mixed_precision, gradient_accumulation_steps, scaler,
                           optimizer.zero_grad)
    for i, (d, d_next) in enumerate(_lookahead(train_dataloader)):
        if d_next is not None and hasattr(jpeg, "prefetch"):
            jpeg.prefetch(d_next)  # the next batch's host JPEG overlaps this step's device work
        crit = graphed(d, noisequant, i % gradient_accumulation_steps == 0, reducer,
                       (i + 1) % gradient_accumulation_steps == 0)
        step_graphed = crit is not None
        if crit is not None:
            pending.append(_metrics(crit))
            n_img = len(d)
        else:
            with amp():
                out_net = model(d, noisequant)
                d = d.to(device)
                out_criterion = criterion(out_net, d)
                loss = out_criterion["loss"]
                if gradient_accumulation_steps != 1:
                    loss = loss / gradient_accumulation_steps
            if reducer is not None:  # overlapped all-reduce only on the accumulation boundary (DDP no_sync)
                reducer.armed = (i + 1) % gradient_accumulation_steps == 0
            pending.append(_metrics(out_criterion))
            if scaler is not None:
                scaler.scale_loss(loss).backward()
            else:
                loss.backward()
            n_img = len(d)
            del out_net, out_criterion, loss
        if (i + 1) % gradient_accumulation_steps == 0:
            if reducer is not None:
                if step_graphed:
                    graphed.reduce(reducer)
                else:
                    reducer.all_reduce()
            nan_src = None
            if not hasattr(optimizer, "max_grad_norm") and clip_max_norm > 0:
                torch.nn.utils.clip_grad_norm_(model.parameters(), clip_max_norm)
            if scaler is not None:
                optimizer.step(grad_scaler=scaler)  # unscale_ + clip + skip on inf/NaN (engine.py:57-80)
                scaler.update(optimizer.sumsq)
                if clip_max_norm > 0:
                    nan_src = optimizer.sumsq.clone()
                    nan_flags.append(nan_src)
            else:
                optimizer.step()
            optimizer.zero_grad()
            aux_loss = model.aux_loss()
            aux_loss.backward()
            aux_optimizer.step(skip_if_nan=nan_src)  # the reference's ``continue`` skips it on NaN
            aux_optimizer.zero_grad()
        if i % log_every == 0:
            _drain(pending, meters, nan_flags)
            print(f"Train epoch {epoch}: [{i * n_img}/{len(train_dataloader.dataset)} "
                  f"({100. * i / max(len(train_dataloader), 1):.0f}%)]"
                  f"\tLoss: {meters['loss'].val:.3f} |\tBpp loss: {meters['bpp_loss'].val:.3f} |"
                  f"\tResidual Bpp: {meters['residual_bpp_loss'].val:.3f} |"
                  f"\ty_Bpp loss: {meters['y_bpp_loss'].val:.4f} |\tz_Bpp loss: {meters['z_bpp_loss'].val:.4f} |"
                  f"\tMSE loss: {meters['mse_loss'].val:.3f} |"
                  f"\tAux loss: {float(aux_loss.detach()) if aux_loss is not None else 0.0:.2f}")
    crit = None  # the last replay's static outputs live in the graph's pool: no reference may outlive close()
    graphed.close()
    _drain(pending, meters, nan_flags)
    print(f"Train epoch {epoch}: Average losses:\tLoss: {meters['loss'].avg:.3f} |"
          f"\tBpp loss: {meters['bpp_loss'].avg:.4f} |\tResidual Bpp: {meters['residual_bpp_loss'].avg:.4f} |"
          f"\ty_Bpp loss: {meters['y_bpp_loss'].avg:.5f} |\tz_Bpp loss: {meters['z_bpp_loss'].avg:.5f} |"
          f"\tMSE loss: {meters['mse_loss'].avg:.3f} |\tTime (s) : {time.time() - start:.4f} |")
    return meters["loss"].avg, meters["bpp_loss"].avg, meters["mse_loss"].avg


def test_epoch(epoch, test_dataloader, model, criterion, save_images=False, savepath=None, all_reduce=True):
    """``all_reduce``: under DDP each rank evaluated its shard and the meters are summed over ranks (a collective:
    every rank must call it). The best-checkpoint image dump runs on rank 0 ALONE over the unsharded test set
    (src/training.py) with ``all_reduce=False``, so it joins no collective the other ranks do not issue."""
    model.eval()
    device = next(model.parameters()).device
    meters = {k: AverageMeter() for k in _KEYS}
    aux_meter = AverageMeter()
    pending = []
    with torch.no_grad():
        for i, d in enumerate(test_dataloader):
            out_net = model(d)
            d = d.to(device)
            pending.append(_metrics(criterion(out_net, d)))
            aux_meter.update(float(model.aux_loss()))
            if save_images and i < 6 and savepath:
                _save_components(out_net, d, os.path.join(savepath, "best_recon"), i)
    _drain(pending, meters)
    if all_reduce:
        _all_reduce_meters(list(meters.values()) + [aux_meter], device)
    print(f"Test epoch {epoch}: Average losses:\tLoss: {meters['loss'].avg:.3f} |"
          f"\tBpp loss: {meters['bpp_loss'].avg:.4f} |\tResidual Bpp: {meters['residual_bpp_loss'].avg:.4f} |"
          f"\ty_Bpp loss: {meters['y_bpp_loss'].avg:.4f} |\tz_Bpp loss: {meters['z_bpp_loss'].avg:.4f} |"
          f"\tMSE loss: {meters['mse_loss'].avg:.3f} |\tAux loss: {aux_meter.avg:.4f}\n")
    if save_images and savepath:
        import csv
        with open(os.path.join(savepath, "best_metrics.csv"), "w") as f:
            w = csv.writer(f)
            w.writerow(["epoch", "loss", "mse_loss", "bpp_loss", "residual_bpp", "y_bpp_loss", "z_bpp_loss",
                        "aux_loss"])
            w.writerow([epoch, meters["loss"].avg, meters["mse_loss"].avg, meters["bpp_loss"].avg,
                        meters["residual_bpp_loss"].avg, meters["y_bpp_loss"].avg, meters["z_bpp_loss"].avg,
                        aux_meter.avg])
    return meters["loss"].avg, meters["bpp_loss"].avg, meters["mse_loss"].avg


def _all_reduce_meters(meters, device) -> None:
    """DDP: each rank evaluated its shard of the test set; sum the meters' sums and counts over ranks so every
    rank reports the mean over all test batches."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    dev = device if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([[float(m.sum), float(m.count)] for m in meters], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    for m, (sm, cnt) in zip(meters, t.cpu().tolist()):
        m.sum, m.count = sm, int(cnt)
        m.avg = sm / cnt if cnt else 0.0


def _save_components(out_net, d, recon_dir, i):
    """PNG dumps (torchvision.save_image is not installed: Pillow writer)."""
    import numpy as np
    from PIL import Image
    os.makedirs(recon_dir, exist_ok=True)

    def save(t, path):
        a = (t[0].detach().clamp(0, 1).permute(1, 2, 0).cpu().numpy() * 255 + 0.5).astype(np.uint8)
        Image.fromarray(a).save(path)

    save(d, os.path.join(recon_dir, f"original_{i}.png"))
    save(out_net["x_hat"], os.path.join(recon_dir, f"recon_{i}.png"))
    save(out_net["jpeg_decoded"], os.path.join(recon_dir, f"jpeg_{i}.png"))
    save(out_net["residual"] * 0.5 + 0.5, os.path.join(recon_dir, f"residual_{i}.png"))
    save(out_net["residual_hat"] * 0.5 + 0.5, os.path.join(recon_dir, f"residual_hat_{i}.png"))
