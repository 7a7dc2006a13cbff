"""TEST INFRASTRUCTURE ONLY — CPU restatement of compressai 1.2.6's entropy-coding primitives used by the
reference's compress/decompress (models/checkerboard.py:159-240 -> GaussianConditional /
EntropyBottleneck .compress/.decompress/.update). compressai is NOT vendored under /root/reference and is
not installed here, so this restates its published algorithm:

* ``pmf_to_quantized_cdf`` — compressai/cpp_exts/ops/ops.cpp (round to 2^precision, renormalise, fix
  zero-frequency symbols by stealing from the smallest frequency > 1);
* ``rans_encode`` / ``rans_decode`` — compressai/cpp_exts/rans/rans_interface.cpp over ryg_rans rans64.h
  (64-bit state, 32-bit words, 16-bit precision, 4-bit bypass escape for out-of-range symbols);
* ``gc_tables`` / ``eb_pmf`` — GaussianConditional.update / EntropyBottleneck.update.

No reference test or golden vector pins these ("parity unpinned" at the compressai
boundary); the HIP/C++ product is checked bit-exact against this restatement and by round trips.
Only tests/ may import this module.
"""
from __future__ import annotations

import math
from typing import List, Sequence

import numpy as np

PRECISION = 16
BYPASS_PRECISION = 4
MAX_BYPASS_VAL = (1 << BYPASS_PRECISION) - 1
RANS64_L = 1 << 31
M64 = (1 << 64) - 1


def pmf_to_quantized_cdf(pmf: Sequence[float], precision: int = PRECISION) -> List[int]:
    pmf = [float(np.float32(p)) for p in pmf]
    cdf = [0] + [int(round_half_away(p * (1 << precision))) for p in pmf]
    total = sum(cdf)
    cdf = [((1 << precision) * v) // total for v in cdf]
    for i in range(1, len(cdf)):
        cdf[i] += cdf[i - 1]
    cdf[-1] = 1 << precision
    n = len(cdf) - 1
    for i in range(n):
        if cdf[i] == cdf[i + 1]:
            best_freq, best_steal = None, -1
            for j in range(n):
                freq = cdf[j + 1] - cdf[j]
                if freq > 1 and (best_freq is None or freq < best_freq):
                    best_freq, best_steal = freq, j
            assert best_steal != -1
            if best_steal < i:
                for j in range(best_steal + 1, i + 1):
                    cdf[j] -= 1
            else:
                for j in range(i + 1, best_steal + 1):
                    cdf[j] += 1
    return cdf


def round_half_away(x: float) -> float:  # std::round
    return math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)


def _symbols(symbols, indexes, cdfs, cdf_sizes, offsets):
    syms = []
    for s, ci in zip(symbols, indexes):
        cdf = cdfs[ci]
        max_value = cdf_sizes[ci] - 2
        value = int(s) - int(offsets[ci])
        raw = 0
        if value < 0:
            raw, value = -2 * value - 1, max_value
        elif value >= max_value:
            raw, value = 2 * (value - max_value), max_value
        syms.append((cdf[value], cdf[value + 1] - cdf[value], False))
        if value == max_value:
            nb = 0
            while (raw >> (nb * BYPASS_PRECISION)) != 0:
                nb += 1
            val = nb
            while val >= MAX_BYPASS_VAL:
                syms.append((MAX_BYPASS_VAL, MAX_BYPASS_VAL + 1, True))
                val -= MAX_BYPASS_VAL
            syms.append((val, val + 1, True))
            for j in range(nb):
                v = (raw >> (j * BYPASS_PRECISION)) & MAX_BYPASS_VAL
                syms.append((v, v + 1, True))
    return syms


def rans_encode(symbols, indexes, cdfs, cdf_sizes, offsets) -> bytes:
    x = RANS64_L
    words: List[int] = []  # reverse memory order
    for start, freq, bypass in reversed(_symbols(symbols, indexes, cdfs, cdf_sizes, offsets)):
        if not bypass:
            x_max = ((RANS64_L >> PRECISION) << 32) * freq
            if x >= x_max:
                words.append(x & 0xFFFFFFFF)
                x >>= 32
            x = ((x // freq) << PRECISION) + (x % freq) + start
        else:
            freq_b = 1 << (16 - BYPASS_PRECISION)
            x_max = ((RANS64_L >> 16) << 32) * freq_b
            if x >= x_max:
                words.append(x & 0xFFFFFFFF)
                x >>= 32
            x = ((x << BYPASS_PRECISION) | start) & M64
    words.append(x >> 32)
    words.append(x & 0xFFFFFFFF)
    return np.array(words[::-1], dtype="<u4").tobytes()


def rans_decode(data: bytes, indexes, cdfs, cdf_sizes, offsets) -> List[int]:
    w = np.frombuffer(data, dtype="<u4").astype(np.uint64).tolist()
    pos = 0

    def nxt():
        nonlocal pos
        v = w[pos] if pos < len(w) else 0
        pos += 1
        return int(v)

    x = nxt() | (nxt() << 32)

    def get_bits(n):
        nonlocal x
        v = x & ((1 << n) - 1)
        x >>= n
        if x < RANS64_L:
            x = ((x << 32) | nxt()) & M64
        return v

    out = []
    for ci in indexes:
        cdf = cdfs[ci]
        max_value = cdf_sizes[ci] - 2
        cum = x & ((1 << PRECISION) - 1)
        s = 0
        while s + 1 <= max_value + 1 and cdf[s + 1] <= cum:
            s += 1
        start, freq = cdf[s], cdf[s + 1] - cdf[s]
        x = freq * (x >> PRECISION) + (x & ((1 << PRECISION) - 1)) - start
        if x < RANS64_L:
            x = ((x << 32) | nxt()) & M64
        value = s
        if value == max_value:
            val = get_bits(BYPASS_PRECISION)
            nb = val
            while val == MAX_BYPASS_VAL:
                val = get_bits(BYPASS_PRECISION)
                nb += val
            raw = 0
            for j in range(nb):
                raw |= get_bits(BYPASS_PRECISION) << (j * BYPASS_PRECISION)
            value = raw >> 1
            value = -value - 1 if raw & 1 else value + max_value
        out.append(value + int(offsets[ci]))
    return out


def standardized_cumulative(x):
    from scipy.special import erfc
    return 0.5 * erfc(-(2 ** -0.5) * np.asarray(x, dtype=np.float64))


def gc_tables(scale_table: Sequence[float], tail_mass: float = 1e-9):
    """GaussianConditional.update (compressai 1.2.6): (quantized_cdf [n, L+2], cdf_length, offset)."""
    from scipy.stats import norm
    st = np.asarray(scale_table, dtype=np.float32)
    multiplier = -norm.ppf(tail_mass / 2)
    pmf_center = np.ceil(st * np.float32(multiplier)).astype(np.int32)
    pmf_length = 2 * pmf_center + 1
    max_length = int(pmf_length.max())
    samples = np.abs(np.arange(max_length, dtype=np.int32)[None, :] - pmf_center[:, None]).astype(np.float32)
    scale = st[:, None]
    upper = standardized_cumulative((np.float32(0.5) - samples) / scale).astype(np.float32)
    lower = standardized_cumulative((np.float32(-0.5) - samples) / scale).astype(np.float32)
    pmf = upper - lower
    tail = 2 * lower[:, :1]
    cdf = np.zeros((len(st), max_length + 2), dtype=np.int32)
    for i in range(len(st)):
        prob = np.concatenate([pmf[i, :pmf_length[i]], tail[i]])
        c = pmf_to_quantized_cdf(prob)
        cdf[i, :len(c)] = c
    return cdf, pmf_length + 2, -pmf_center
