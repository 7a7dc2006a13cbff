"""compress / decompress entropy coding with compressai 1.2.6 semantics.

* ``eb_update`` / ``gc_update``: EntropyBottleneck.update / GaussianConditional.update_scale_table —
  the quantized CDF tables (``_quantized_cdf``, ``_cdf_length``, ``_offset`` buffers, same shapes and
  dtypes as compressai, so state_dicts round-trip). The pmf -> 16-bit CDF step is the C-ABI's
  ``hyres_pmf_to_quantized_cdf``; the densities are evaluated with torch on the parameters' device (a
  one-time table build, as in the reference).
* ``eb_compress`` / ``gc_compress`` (+ decompress): the per-element work — symbol = round(v - mean),
  CDF index building over the scale table, dequantisation — runs in HIP kernels
  (``hyres_eb_symbols``, ``hyres_gc_symbols``, ``hyres_gc_dequant``) on the NHWC activations; the
  sequential rANS coder (one string per image, compressai's wire format) runs on the host
  (``hyres_rans_encode_with_indexes`` / ``hyres_rans_decode_with_indexes``).
"""
from __future__ import annotations

import ctypes
import math
from typing import List

import numpy as np
import torch

from . import _lib as L
from .ops import Node, _empty

PRECISION = 16


def _pmf_to_cdf(pmf: torch.Tensor, tail_mass: torch.Tensor, pmf_length: torch.Tensor, max_length: int):
    """compressai EntropyModel._pmf_to_cdf: row i = CDF of cat(pmf[i, :len_i], tail_i)."""
    pmf = pmf.detach().float().cpu().numpy()
    tail = tail_mass.detach().float().cpu().numpy().reshape(len(pmf), -1)
    lengths = pmf_length.detach().cpu().numpy().astype(np.int64)
    cdf = np.zeros((len(lengths), max_length + 2), dtype=np.int32)
    lib = L.load()
    for i, n in enumerate(lengths):
        prob = np.ascontiguousarray(np.concatenate([pmf[i, :n], tail[i, :1]]), dtype=np.float32)
        out = np.zeros(n + 2, dtype=np.int32)
        L.check(lib.hyres_pmf_to_quantized_cdf(prob.ctypes.data, int(n + 1), PRECISION, out.ctypes.data),
                "hyres_pmf_to_quantized_cdf")
        cdf[i, :n + 2] = out
    return torch.from_numpy(cdf)


def _logits_cumulative(eb, inputs: torch.Tensor) -> torch.Tensor:
    logits = inputs
    for i in range(len(eb.filters) + 1):
        matrix = torch.nn.functional.softplus(getattr(eb, f"_matrix{i:d}").detach().cpu())
        logits = torch.matmul(matrix, logits)
        logits = logits + getattr(eb, f"_bias{i:d}").detach().cpu()
        if i < len(eb.filters):
            logits = logits + torch.tanh(getattr(eb, f"_factor{i:d}").detach().cpu()) * torch.tanh(logits)
    return logits


@torch.no_grad()
def eb_update(eb, force: bool = False) -> bool:
    """compressai EntropyBottleneck.update (1.2.6).  Evaluated on the host in fp32, as the reference runs it
    (src/updata.py:50-53 updates a CPU-loaded model): the CDF tables are then bit-identical to the
    reference's for the same parameters, whatever device the model lives on."""
    if eb._offset.numel() > 0 and not force:
        return False
    q = eb.quantiles.detach().cpu()
    medians = q[:, 0, 1]
    minima = torch.clamp(torch.ceil(medians - q[:, 0, 0]).int(), min=0)
    maxima = torch.clamp(torch.ceil(q[:, 0, 2] - medians).int(), min=0)
    pmf_start = medians - minima
    pmf_length = maxima + minima + 1
    max_length = int(pmf_length.max().item())
    samples = torch.arange(max_length)[None, :] + pmf_start[:, None, None]
    lower = _logits_cumulative(eb, samples - 0.5)
    upper = _logits_cumulative(eb, samples + 0.5)
    sign = -torch.sign(lower + upper)
    pmf = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))[:, 0, :]
    tail_mass = torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:])
    dev = eb._offset.device
    eb._offset = (-minima).to(dev)
    eb._quantized_cdf = _pmf_to_cdf(pmf, tail_mass, pmf_length, max_length).to(dev)
    eb._cdf_length = (pmf_length + 2).to(dev)
    eb._coder_cache = None
    return True


def _standardized_quantile(q: float) -> float:
    from scipy.stats import norm
    return float(norm.ppf(q))


@torch.no_grad()
def gc_update(gc) -> None:
    """compressai GaussianConditional.update (1.2.6) over ``gc.scale_table``."""
    st = gc.scale_table.detach().float().cpu()
    multiplier = -_standardized_quantile(gc.tail_mass / 2)
    pmf_center = torch.ceil(st * multiplier).int()
    pmf_length = 2 * pmf_center + 1
    max_length = int(torch.max(pmf_length).item())
    samples = torch.abs(torch.arange(max_length).int() - pmf_center[:, None]).float()
    scale = st.unsqueeze(1)

    def cum(x):
        return 0.5 * torch.erfc(-(2 ** -0.5) * x)

    upper = cum((0.5 - samples) / scale)
    lower = cum((-0.5 - samples) / scale)
    pmf = upper - lower
    tail_mass = 2 * lower[:, :1]
    dev = gc.scale_bound.device
    gc._quantized_cdf = _pmf_to_cdf(pmf, tail_mass, pmf_length, max_length).to(dev)
    gc._offset = (-pmf_center).to(dev)
    gc._cdf_length = (pmf_length + 2).to(dev)
    gc._coder_cache = None


def _tables(model):
    """Host copies of a model's CDF tables (cached until the next update)."""
    c = getattr(model, "_coder_cache", None)
    if c is None:
        if model._offset.numel() == 0:
            raise ValueError("Entropy coder tables are not initialised: run model.update() first "
                             "(compressai: 'Uninitialized CDFs. Run update() first')")
        cdf = np.ascontiguousarray(model._quantized_cdf.cpu().numpy(), dtype=np.int32)
        c = (cdf, np.ascontiguousarray(model._cdf_length.cpu().numpy(), dtype=np.int32),
             np.ascontiguousarray(model._offset.cpu().numpy(), dtype=np.int32))
        model._coder_cache = c
    return c


def _encode(model, sym: np.ndarray, idx: np.ndarray) -> bytes:
    cdf, lengths, offsets = _tables(model)
    lib = L.load()
    n = int(sym.size)
    ln = ctypes.c_longlong(0)
    args = (sym.ctypes.data, idx.ctypes.data, n, cdf.ctypes.data, cdf.shape[1], lengths.ctypes.data,
            offsets.ctypes.data, len(lengths))
    buf = np.empty(8 * n + 64, dtype=np.uint8)  # 2 words per symbol: enough unless many bypass escapes
    if lib.hyres_rans_encode_with_indexes(*args, buf.ctypes.data, buf.size, ctypes.byref(ln)) != 0:
        buf = np.empty(ln.value, dtype=np.uint8)  # the failed call reported the exact length
        L.check(lib.hyres_rans_encode_with_indexes(*args, buf.ctypes.data, buf.size, ctypes.byref(ln)),
                "rans_encode")
    return buf[:ln.value].tobytes()


def _decode(model, data: bytes, idx: np.ndarray, out: np.ndarray = None) -> np.ndarray:
    cdf, lengths, offsets = _tables(model)
    src = np.frombuffer(data, dtype=np.uint8)
    if out is None:
        out = np.empty(idx.size, dtype=np.int32)
    assert out.dtype == np.int32 and out.flags.c_contiguous and out.size == idx.size
    L.check(L.load().hyres_rans_decode_with_indexes(src.ctypes.data, src.size, idx.ctypes.data, int(idx.size),
                                                    cdf.ctypes.data, cdf.shape[1], lengths.ctypes.data,
                                                    offsets.ctypes.data, len(lengths), out.ctypes.data),
            "rans_decode")
    return out


_POOL = None


def _pool():
    """Host threads for the rANS coder: strings are independent (per image, per pass), and the ctypes
    calls release the GIL, so anchor / non-anchor / z strings (and the images of a batch) code in parallel
    and overlap the GPU work that follows them in compress."""
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _POOL = ThreadPoolExecutor(max_workers=8, thread_name_prefix="hyres-rans")
    return _POOL


def _map(fn, items):
    items = list(items)
    if len(items) <= 1:  # one image: decode on the calling thread
        return [fn(it) for it in items]
    return list(_pool().map(fn, items))


def resolve(strings):
    """Futures -> bytes (lists of per-image strings, possibly nested)."""
    if isinstance(strings, list):
        return [resolve(v) for v in strings]
    return strings.result() if hasattr(strings, "result") else strings


def _medians(eb) -> torch.Tensor:
    return eb.quantiles.detach()[:, 0, 1].contiguous()


def _eb_indexes(C: int, H: int, W: int) -> np.ndarray:
    return np.ascontiguousarray(np.repeat(np.arange(C, dtype=np.int32), H * W))


def eb_compress(eb, z: Node) -> list:
    """EntropyBottleneck.compress(z): one string per image (futures; ``resolve`` -> bytes)."""
    B, H, W, C = z.B, z.H, z.W, z.C
    sym = torch.empty(B * C * H * W, dtype=torch.int32, device=z.device)
    L.call("hyres_eb_symbols", z.ptr(), z.ld, _medians(eb).data_ptr(), B, H, W, C, sym.data_ptr(), None, 0, 0,
           L.stream())
    sym_h = sym.cpu().numpy().reshape(B, -1)
    idx = _eb_indexes(C, H, W)
    _tables(eb)
    return [_pool().submit(_encode, eb, np.ascontiguousarray(sym_h[b]), idx) for b in range(B)]


def eb_decompress(eb, strings: List[bytes], H: int, W: int, device) -> Node:
    """EntropyBottleneck.decompress(strings, (H, W)) -> z_hat (NHWC Node)."""
    B, C = len(strings), eb.channels
    idx = _eb_indexes(C, H, W)
    _tables(eb)
    # decoded straight into pinned host memory: a pageable host->device copy of the symbols costs tens of
    # ms on this platform (measured: 4.7 MB in 21-28 ms), a pinned one well under 1 ms
    sym = torch.empty((B, C * H * W), dtype=torch.int32, pin_memory=True)
    sym_np = sym.numpy()
    _map(lambda bs: _decode(eb, bs[1], idx, sym_np[bs[0]]), enumerate(resolve(list(strings))))
    sym_d = sym.to(device, non_blocking=True)
    z_hat = Node.new(B, H, W, C, device, rg=False)
    L.call("hyres_eb_symbols", None, 0, _medians(eb).data_ptr(), B, H, W, C, sym_d.data_ptr(), z_hat.ptr(),
           z_hat.ld, 1, L.stream())
    return z_hat


def _gc_indexes(gc, params: Node, M: int, y: Node = None, parity: int = -1):
    B, H, W = params.B, params.H, params.W
    n = B * M * H * W
    idx = torch.empty(n, dtype=torch.int32, device=params.device)
    sym = torch.empty(n, dtype=torch.int32, device=params.device) if y is not None else None
    table = gc.scale_table.detach().float().contiguous()
    L.call("hyres_gc_symbols", None if y is None else y.ptr(), 0 if y is None else y.ld, params.ptr(), params.ld, M,
           B, H, W, parity, table.data_ptr(), table.numel(), L.ptr(sym), idx.data_ptr(), L.stream())
    return sym, idx


def gc_compress(gc, y: Node, params: Node, M: int, parity: int) -> list:
    """GaussianConditional.compress(y * mask(parity), build_indexes(scales), means) per image
    (models/checkerboard.py:159-161); params = [.., scales(M) | means(M)]."""
    sym, idx = _gc_indexes(gc, params, M, y, parity)
    B = params.B
    sym_h = sym.cpu().numpy().reshape(B, -1)
    idx_h = idx.cpu().numpy().reshape(B, -1)
    _tables(gc)
    return [_pool().submit(_encode, gc, np.ascontiguousarray(sym_h[b]), np.ascontiguousarray(idx_h[b]))
            for b in range(B)]


def gc_decompress(gc, strings: List[bytes], params: Node, M: int, out: Node, accumulate: bool = False) -> Node:
    """GaussianConditional.decompress(strings, build_indexes(scales), means) into ``out`` (NHWC)."""
    _, idx = _gc_indexes(gc, params, M)
    B = params.B
    idx_h = idx.cpu().numpy().reshape(B, -1)
    _tables(gc)
    sym = torch.empty(idx_h.shape, dtype=torch.int32, pin_memory=True)  # pinned: see eb_decompress
    sym_np = sym.numpy()
    _map(lambda bs: _decode(gc, bs[1], np.ascontiguousarray(idx_h[bs[0]]), sym_np[bs[0]]),
         enumerate(resolve(list(strings))))
    sym_d = sym.to(params.device, non_blocking=True)
    L.call("hyres_gc_dequant", sym_d.data_ptr(), params.ptr(), params.ld, M, B, params.H, params.W, out.ptr(), out.ld,
           int(accumulate), L.stream())
    return out


def get_scale_table(min_=0.11, max_=256, levels=64):
    """models/checkerboard.py:17-21."""
    return torch.exp(torch.linspace(math.log(min_), math.log(max_), levels))
