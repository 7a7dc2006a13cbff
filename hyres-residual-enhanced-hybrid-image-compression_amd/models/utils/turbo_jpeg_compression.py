"""Host JPEG base layer (models/utils/turbo_jpeg_compression.py:8-77) — a CPU stage by design.

Semantics kept from the reference:
  * input bytes = (clamp(x, 0, 1) * 255).byte()  (truncation, :25,32);
  * ``TurboJPEG.encode(img, quality)`` with PyTurboJPEG's defaults: the RGB array is interpreted as BGR
    (TJPF_BGR) and chroma is subsampled 4:2:2 (TJSAMP_422) (:35); decode returns the same channel order;
  * bpp = total compressed bytes * 8 / (N*H*W)  (:70-73).
Backends: PyTurboJPEG if importable (bit-identical to the reference), else Pillow's bundled
libjpeg-turbo with the same effective settings (channel order reversed in/out, subsampling=1 = 4:2:2).
The hard-coded ``lib_path`` of the reference (:12) is replaced by the library's default lookup or
``HYRES_TURBOJPEG_LIB``.  Images are coded by worker processes when ``hyres_hip.jpeg_host.start()`` ran before the GPU was touched
(Pillow's coder holds the GIL, so threads do not scale), else by a thread pool (PyTurboJPEG releases the
GIL); ``prefetch`` overlaps the next batch's JPEG with the device step.  This is the host-side half of the
multi-GPU scaling story.
"""
from __future__ import annotations

import io
import os
import weakref
from collections import OrderedDict
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

import numpy as np
import torch
from torch import nn

from hyres_hip import jpeg_host

try:  # pragma: no cover - not installed in this image
    from turbojpeg import TurboJPEG as _TurboJPEG  # type: ignore
except Exception:  # noqa: BLE001
    _TurboJPEG = None


def _to_uint8_batch(x: torch.Tensor) -> np.ndarray:
    """[N,C,H,W] float -> [N,H,W,3] uint8: (clamp(x, 0, 1) * 255).byte() (truncation, :25,32), grey
    images repeated to 3 channels (:26-28); one vectorised pass over the batch."""
    t = torch.clamp(x, 0, 1)
    if t.size(1) == 1:
        t = t.repeat(1, 3, 1, 1)
    return (t * 255).byte().permute(0, 2, 3, 1).contiguous().numpy()


class _PillowTurbo:
    """PyTurboJPEG-compatible encode/decode on Pillow's libjpeg-turbo (BGR interpretation, 4:2:2)."""

    def encode(self, img_np: np.ndarray, quality: int = 85) -> bytes:
        from PIL import Image
        im = Image.fromarray(np.ascontiguousarray(img_np[..., ::-1]), "RGB")
        buf = io.BytesIO()
        im.save(buf, format="JPEG", quality=int(quality), subsampling=1)
        return buf.getvalue()

    def decode(self, data: bytes) -> np.ndarray:
        from PIL import Image
        im = Image.open(io.BytesIO(data)).convert("RGB")
        return np.asarray(im)[..., ::-1]


class TurboJPEGCompression(nn.Module):
    """Host JPEG stage.  Each image's encode -> decode round trip is ONE task on a thread pool (libjpeg-turbo
    releases the GIL); ``prefetch(x)`` starts the next batch's round trip in the background so a training
    loop overlaps the host JPEG stage with the device step (src/utils/engine.py does this)."""

    def __init__(self, quality=25, lib_path: Optional[str] = None, workers: Optional[int] = None):
        super().__init__()
        self.quality = quality
        lib_path = lib_path or os.environ.get("HYRES_TURBOJPEG_LIB")
        if _TurboJPEG is not None:
            self.jpeg = _TurboJPEG(lib_path) if lib_path else _TurboJPEG()
            self.backend = "pyturbojpeg"
        else:
            self.jpeg = _PillowTurbo()
            self.backend = "pillow-libjpeg-turbo"
        self.workers = workers or int(os.environ.get("HYRES_JPEG_WORKERS", min(16, os.cpu_count() or 1)))
        self._pool: Optional[ThreadPoolExecutor] = None
        self._bg: Optional[ThreadPoolExecutor] = None
        # prefetched round trips keyed by _key(x): a loop that prefetches batch i+1 before it reads batch i
        # (src/utils/engine.py) keeps both in flight; an entry is popped when its forward uses it
        self._pending: "OrderedDict[tuple, object]" = OrderedDict()
        self.max_pending = 4
        self.prefetch_hits = 0
        self.prefetch_misses = 0

    def _map(self, fn, items):
        if len(items) <= 1 or self.workers <= 1:
            return [fn(i) for i in items]
        if self._pool is None:
            self._pool = ThreadPoolExecutor(max_workers=self.workers, thread_name_prefix="hyres-jpeg")
        return list(self._pool.map(fn, items))

    def compress(self, x: torch.Tensor) -> List[io.BytesIO]:
        imgs = _to_uint8_batch(x.detach().cpu())
        datas = self._map(lambda im: self.jpeg.encode(im, quality=self.quality), list(imgs))
        return [io.BytesIO(d) for d in datas]

    def decompress(self, compressed_buffers, device) -> torch.Tensor:
        arrs = self._map(lambda b: self.jpeg.decode(b.getvalue()), list(compressed_buffers))
        return self._stack(arrs).to(device)

    @staticmethod
    def _stack(arrs) -> torch.Tensor:
        # torch.from_numpy(a).float().permute(2, 0, 1) / 255.0 per image (:55-58), batched
        return torch.from_numpy(np.stack(arrs)).permute(0, 3, 1, 2).float() / 255.0

    def _roundtrip(self, x: torch.Tensor):
        imgs = _to_uint8_batch(x)
        procs_pool, nprocs = jpeg_host.pool()
        if procs_pool is not None and self.backend == "pillow-libjpeg-turbo" and imgs.shape[0] > 1:
            # worker processes (Pillow's coder holds the GIL): contiguous chunks, results in order
            k = -(-imgs.shape[0] // nprocs)
            futs = [procs_pool.submit(jpeg_host.roundtrip_pillow, imgs[i:i + k], self.quality)
                    for i in range(0, imgs.shape[0], k)]
            sizes, arrs = [], []
            for f in futs:
                s_, a_ = f.result()
                sizes += s_
                arrs.append(a_)
            N, _, H, W = x.size()
            dec = torch.from_numpy(np.concatenate(arrs)).permute(0, 3, 1, 2).float() / 255.0
            return dec, sum(n * 8 for n in sizes) / (N * H * W)

        def one(im):
            data = self.jpeg.encode(im, quality=self.quality)
            return len(data), self.jpeg.decode(data)

        res = self._map(one, list(imgs))
        N, _, H, W = x.size()
        bits = sum(n * 8 for n, _ in res)
        return self._stack([a for _, a in res]), bits / (N * H * W)

    @staticmethod
    def _key(x: torch.Tensor):
        return (id(x), x.data_ptr(), x._version, tuple(x.shape))

    def prefetch(self, x: torch.Tensor) -> None:
        """Start ``forward(x)``'s host work for a CPU batch in the background.  Up to ``max_pending`` batches
        stay in flight (oldest dropped first); prefetching a batch that is already pending is a no-op."""
        if x.device.type != "cpu":
            return
        key = self._key(x)
        if key in self._pending:
            return
        if self._bg is None:
            self._bg = ThreadPoolExecutor(max_workers=1, thread_name_prefix="hyres-jpeg-prefetch")
        while len(self._pending) >= self.max_pending:
            _, (_, old) = self._pending.popitem(last=False)
            old.cancel()
        # the weak reference guards against a freed batch whose id/address a new tensor reuses
        self._pending[key] = (weakref.ref(x), self._bg.submit(self._roundtrip, x.detach()))

    def forward(self, x: torch.Tensor):
        """(decoded [N,3,H,W] on x.device, jpeg_bpp = total bytes * 8 / (N*H*W))  (:62-77)."""
        device = x.device
        ent = self._pending.pop(self._key(x), None) if x.device.type == "cpu" else None
        fut = ent[1] if ent is not None and ent[0]() is x else None
        if fut is not None:
            self.prefetch_hits += 1
            decoded, bpp = fut.result()
        else:
            self.prefetch_misses += 1
            decoded, bpp = self._roundtrip(x.detach().cpu())
        return decoded.to(device), bpp

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_pool"] = st["_bg"] = None
        st["_pending"] = OrderedDict()
        return st
