"""Row f2: the host JPEG base layer against the reference's own TurboJPEGCompression.

Every fixture under tests/golden was produced by tests/golden/make_golden.py running the reference's
``models/utils/turbo_jpeg_compression.py:17-77`` (its ``(clamp(x)*255).byte()`` truncation, its encode of the
RGB array with PyTurboJPEG's defaults — read as BGR, 4:2:2 — its decode and its
``bpp = bytes*8/(N*H*W)``), with the ``turbojpeg`` module emulated on Pillow's bundled libjpeg-turbo (the
PyTurboJPEG wheel is not installed).  The product's stage is byte work, so it must reproduce the stored
``jpeg_decoded`` bit for bit and ``jpeg_bpp`` exactly, through the in-process path and through the worker
process pool; and ``prefetch`` must serve a loop that prefetches the next batch before it reads the current
one (src/utils/engine.py) from the background, not recompute it.
"""
import numpy as np
import pytest
import torch

from helpers import load_npz

FIXTURES = ["hyres_eval_b2_64.npz", "hyres_train_b2_64.npz", "hyres_train_nq_b2_64.npz", "kodim01_crop64_eval.npz"]


def _check(j, g):
    dec, bpp = j(g["x"])
    assert dec.dtype == torch.float32 and dec.shape == g["jpeg_decoded"].shape
    assert torch.equal(dec, g["jpeg_decoded"]), int((dec != g["jpeg_decoded"]).sum())
    if "jpeg_bpp" in g:
        assert np.float32(bpp) == g["jpeg_bpp"].numpy(), (bpp, float(g["jpeg_bpp"]))


@pytest.mark.parametrize("fixture", FIXTURES)
def test_jpeg_stage_matches_reference_in_process(fixture):
    from hyres_hip import jpeg_host
    from models.utils.turbo_jpeg_compression import TurboJPEGCompression
    assert jpeg_host.pool()[0] is None
    g = load_npz(fixture)
    for workers in (1, 4):  # serial and thread-pool maps
        _check(TurboJPEGCompression(quality=50, workers=workers), g)


def test_jpeg_stage_matches_reference_process_pool():
    from hyres_hip import jpeg_host
    from models.utils.turbo_jpeg_compression import TurboJPEGCompression
    assert jpeg_host.start(2) == 2
    try:
        for fixture in FIXTURES:
            g = load_npz(fixture)
            _check(TurboJPEGCompression(quality=50), g)
            # a batch bigger than the pool: chunks come back in order
            x4 = torch.cat([g["x"], g["x"].flip(3), g["x"].flip(2)])
            d_pool, b_pool = TurboJPEGCompression(quality=50)(x4)
            saved = jpeg_host._POOL
            jpeg_host._POOL = None
            try:
                d_in, b_in = TurboJPEGCompression(quality=50, workers=1)(x4)
            finally:
                jpeg_host._POOL = saved
            assert torch.equal(d_pool, d_in) and b_pool == b_in
    finally:
        jpeg_host.shutdown()


def test_prefetch_serves_lookahead_loop():
    """engine.py's order: prefetch(batch i+1), then forward(batch i) — both must come from the background."""
    from models.utils.turbo_jpeg_compression import TurboJPEGCompression
    g = load_npz("hyres_eval_b2_64.npz")
    batches = [g["x"], g["x"].flip(3).contiguous(), g["x"].flip(2).contiguous(), g["x"].flip(1).contiguous()]
    j = TurboJPEGCompression(quality=50, workers=1)
    ref = [TurboJPEGCompression(quality=50, workers=1)(b) for b in batches]
    j.prefetch(batches[0])
    for i, b in enumerate(batches):
        if i + 1 < len(batches):
            j.prefetch(batches[i + 1])
        dec, bpp = j(b)
        assert torch.equal(dec, ref[i][0]) and bpp == ref[i][1]
    assert j.prefetch_hits == len(batches) and j.prefetch_misses == 0
    # a tensor that was never prefetched (or whose storage changed) is computed inline
    b = batches[0].clone()
    j.prefetch(b)
    b.add_(0.0)  # bumps the version counter: the prefetched result is stale
    dec, _ = j(b)
    assert j.prefetch_misses == 1 and torch.equal(dec, ref[0][0])
