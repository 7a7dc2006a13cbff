"""Process pool for the host JPEG base layer (models/utils/turbo_jpeg_compression.py).

Pillow's bundled libjpeg-turbo keeps the GIL while it codes, so a thread pool does not scale (measured: 16
images at 256x256, q50, 1 thread 3.3 ms/image, 8 threads 2.8 ms/image).  Worker *processes* do: each codes a
chunk of the batch (encode -> decode round trip, the reference's semantics) and returns the byte counts and
the decoded pixels.  The pool must be started before the process touches the GPU (``start`` is called at the
top of bench.py / src/training.py main), so the workers are plain spawned interpreters that import only
numpy and Pillow — never a GPU context, never a fork of one.
"""
from __future__ import annotations

import io
import multiprocessing as mp
import os
from concurrent.futures import ProcessPoolExecutor
from typing import List, Optional, Tuple

import numpy as np

_POOL: Optional[ProcessPoolExecutor] = None
_PROCS = 0


def _noop(i):
    return i


def default_procs(world: Optional[int] = None) -> int:
    """Worker processes per rank: HYRES_JPEG_PROCS, else min(8, cpus // world) so that the ranks of one node
    share the host cores instead of each starting 8 workers (64 processes at 8 ranks)."""
    if "HYRES_JPEG_PROCS" in os.environ:
        return int(os.environ["HYRES_JPEG_PROCS"])
    if world is None:
        world = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    try:
        cpus = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cpus = os.cpu_count() or 1
    return max(0, min(8, cpus // max(world, 1)))


def start(procs: Optional[int] = None) -> int:
    """Start ``procs`` JPEG worker processes (default ``default_procs()``); 0 or 1 disables."""
    global _POOL, _PROCS
    if _POOL is not None:
        return _PROCS
    if procs is None:
        procs = default_procs()
    if procs <= 1:
        return 0
    _POOL = ProcessPoolExecutor(max_workers=procs, mp_context=mp.get_context("spawn"))
    list(_POOL.map(_noop, range(procs)))  # bring every worker up now (before any GPU initialisation)
    _PROCS = procs
    return procs


def shutdown() -> None:
    global _POOL, _PROCS
    if _POOL is not None:
        _POOL.shutdown(wait=True)
    _POOL, _PROCS = None, 0


def pool() -> Tuple[Optional[ProcessPoolExecutor], int]:
    return _POOL, _PROCS


def roundtrip_pillow(imgs: np.ndarray, quality: int) -> Tuple[List[int], np.ndarray]:
    """PyTurboJPEG encode -> decode emulated on Pillow (RGB array read as BGR, 4:2:2): [k,H,W,3] uint8 ->
    (bytes per image, decoded [k,H,W,3] uint8 in the input's channel order)."""
    from PIL import Image
    sizes, out = [], np.empty_like(imgs)
    for i in range(imgs.shape[0]):
        im = Image.fromarray(np.ascontiguousarray(imgs[i][..., ::-1]), "RGB")
        buf = io.BytesIO()
        im.save(buf, format="JPEG", quality=int(quality), subsampling=1)
        data = buf.getvalue()
        sizes.append(len(data))
        out[i] = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))[..., ::-1]
    return sizes, out
