"""Host JPEG base layer (models/utils/turbo_jpeg_compression.py:8-77) — a CPU stage by design.

Semantics kept from the reference:
  * input bytes = (clamp(x, 0, 1) * 255).byte()  (truncation, :25,32);
  * ``TurboJPEG.encode(img, quality)`` with PyTurboJPEG's defaults: the RGB array is interpreted as BGR
    (TJPF_BGR) and chroma is subsampled 4:2:2 (TJSAMP_422) (:35); decode returns the same channel order;
  * bpp = total compressed bytes * 8 / (N*H*W)  (:70-73).
Backends: PyTurboJPEG if importable (bit-identical to the reference), else Pillow's bundled
libjpeg-turbo with the same effective settings (channel order reversed in/out, subsampling=1 = 4:2:2).
The hard-coded ``lib_path`` of the reference (:12) is replaced by the library's default lookup or
``HYRES_TURBOJPEG_LIB``.  Images are coded by a thread pool (libjpeg-turbo releases the GIL), which is the
host-side half of the multi-GPU scaling story.
"""
from __future__ import annotations

import io
import os
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

import numpy as np
import torch
from torch import nn

try:  # pragma: no cover - not installed in this image
    from turbojpeg import TurboJPEG as _TurboJPEG  # type: ignore
except Exception:  # noqa: BLE001
    _TurboJPEG = None


def _to_uint8_hwc(img: torch.Tensor) -> np.ndarray:
    t = torch.clamp(img, 0, 1)
    if t.size(0) == 1:
        t = t.repeat(3, 1, 1)
    return (t.permute(1, 2, 0) * 255).byte().numpy()


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
        return np.ascontiguousarray(np.asarray(im)[..., ::-1])


class TurboJPEGCompression(nn.Module):
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
        self.workers = workers or min(16, os.cpu_count() or 1)
        self._pool: Optional[ThreadPoolExecutor] = None

    def _map(self, fn, items):
        if len(items) <= 1 or self.workers <= 1:
            return [fn(i) for i in items]
        if self._pool is None:
            self._pool = ThreadPoolExecutor(max_workers=self.workers)
        return list(self._pool.map(fn, items))

    def compress(self, x: torch.Tensor) -> List[io.BytesIO]:
        x_cpu = x.detach().cpu() if x.device.type != "cpu" else x.detach()
        imgs = [_to_uint8_hwc(x_cpu[i]) for i in range(x_cpu.size(0))]
        datas = self._map(lambda im: self.jpeg.encode(im, quality=self.quality), imgs)
        return [io.BytesIO(d) for d in datas]

    def decompress(self, compressed_buffers, device) -> torch.Tensor:
        arrs = self._map(lambda b: self.jpeg.decode(b.getvalue()), list(compressed_buffers))
        imgs = [torch.from_numpy(a).float().permute(2, 0, 1) / 255.0 for a in arrs]
        return torch.stack(imgs, dim=0).to(device)

    def forward(self, x: torch.Tensor):
        device = x.device
        buffers = self.compress(x)
        N, _, H, W = x.size()
        bits = sum(len(b.getvalue()) * 8 for b in buffers)
        jpeg_bpp = bits / (N * H * W)
        return self.decompress(buffers, device), jpeg_bpp

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_pool"] = None
        return st
