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
    """compressai GaussianConditional._standardized_cumulative: 0.5 * erfc(-(2^-0.5) x), torch fp32."""
    import torch
    return 0.5 * torch.erfc(-(2 ** -0.5) * torch.as_tensor(np.asarray(x, dtype=np.float32)))


def gc_tables(scale_table: Sequence[float], tail_mass: float = 1e-9):
    """GaussianConditional.update (compressai 1.2.6): (quantized_cdf [n, L+2], cdf_length, offset).
    compressai evaluates the pmf with torch in fp32 (the multiplier with scipy's norm.ppf)."""
    import torch
    from scipy.stats import norm
    st = torch.as_tensor(np.asarray(scale_table, dtype=np.float32))
    multiplier = -float(norm.ppf(tail_mass / 2))
    pmf_center = torch.ceil(st * multiplier).int()
    pmf_length = 2 * pmf_center + 1
    max_length = int(pmf_length.max())
    samples = torch.abs(torch.arange(max_length).int() - pmf_center[:, None]).float()
    scale = st.unsqueeze(1).float()
    upper = standardized_cumulative((0.5 - samples) / scale)
    lower = standardized_cumulative((-0.5 - samples) / scale)
    pmf = (upper - lower).numpy()
    tail = (2 * lower[:, :1]).numpy()
    return _pmf_table(pmf, tail, pmf_length.numpy(), max_length), (pmf_length + 2).numpy(), (-pmf_center).numpy()


def _pmf_table(pmf, tail, lengths, max_length):
    """compressai EntropyModel._pmf_to_cdf."""
    cdf = np.zeros((len(lengths), max_length + 2), dtype=np.int32)
    for i, n in enumerate(lengths):
        c = pmf_to_quantized_cdf(np.concatenate([pmf[i, :n], tail[i, :1]]))
        cdf[i, :len(c)] = c
    return cdf


def eb_tables(quantiles, logits_cumulative):
    """EntropyBottleneck.update (compressai 1.2.6) on the host: ``quantiles`` [C,1,3] fp32,
    ``logits_cumulative(v [C,1,L]) -> [C,1,L]`` the factorized density's cumulative logits."""
    import torch
    q = quantiles.detach().float()
    medians = q[:, 0, 1]
    minima = torch.clamp(torch.ceil(medians - q[:, 0, 0]).int(), min=0)
    maxima = torch.clamp(torch.ceil(q[:, 0, 2] - medians).int(), min=0)
    pmf_start = medians - minima
    pmf_length = maxima + minima + 1
    max_length = int(pmf_length.max())
    samples = torch.arange(max_length)[None, :] + pmf_start[:, None, None]
    with torch.no_grad():
        lower = logits_cumulative(samples - 0.5)
        upper = logits_cumulative(samples + 0.5)
    sign = -torch.sign(lower + upper)
    pmf = torch.abs(torch.sigmoid(sign * upper) - torch.sigmoid(sign * lower))[:, 0, :]
    tail = torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:])
    return (_pmf_table(pmf.numpy(), tail.numpy(), pmf_length.numpy(), max_length), (pmf_length + 2).numpy(),
            (-minima).numpy())


def build_indexes(scales, scale_table):
    """GaussianConditional.build_indexes: LowerBound(0.11) on the scales, then
    index = len(table) - 1 - #{s in table[:-1] : scales <= s}."""
    scales = np.maximum(np.asarray(scales, dtype=np.float32), np.float32(0.11))
    table = np.asarray(scale_table, dtype=np.float32)
    idx = np.full(scales.shape, len(table) - 1, dtype=np.int32)
    for s in table[:-1]:
        idx -= (scales <= s).astype(np.int32)
    return idx


def reference_compress(orc, residual, scale_table):
    """LightWeightCheckerboard.compress (models/checkerboard.py:167-198) on the functional oracle
    (oracle/hyres_oracle.py), with compressai 1.2.6's EntropyBottleneck / GaussianConditional compress:
    symbols = round(v - means) (int), one rANS string per image over the NCHW-flattened symbols,
    y_anchor_hat / z_hat obtained by decoding (= symbols + means).  Returns
    ([[anchor_strings, non_anchor_strings], z_strings], intermediates)."""
    import torch
    with torch.no_grad():
        y = orc.g_a(residual)
        z = orc.h_a(y)
        k = orc.rp + "entropy_bottleneck."
        eb_cdf, eb_len, eb_off = eb_tables(orc.p(k + "quantiles"), orc.eb_logits_cumulative)
        med = orc.eb_medians().reshape(1, -1, 1, 1)
        z_sym = torch.round(z - med).int()
        C = z.shape[1]
        z_idx = np.repeat(np.arange(C, dtype=np.int32), z.shape[2] * z.shape[3])
        z_strings = [rans_encode(z_sym[b].reshape(-1).tolist(), z_idx.tolist(), eb_cdf.tolist(), eb_len.tolist(),
                                 eb_off.tolist()) for b in range(z.shape[0])]
        z_hat = z_sym.float() + med
        latent = orc.h_s(z_hat)
        gc_cdf, gc_len, gc_off = gc_tables(scale_table)
        tables = (gc_cdf.tolist(), gc_len.tolist(), gc_off.tolist())
        H, W = y.shape[-2:]
        am = orc.anchor_mask(H, W).to(y.dtype)

        def code(v, scales, means):
            sym = torch.round(v - means).int()
            idx = build_indexes(scales.numpy(), scale_table)
            strings = [rans_encode(sym[b].reshape(-1).tolist(), idx[b].reshape(-1).tolist(), *tables)
                       for b in range(v.shape[0])]
            return strings, sym, idx

        s_a, m_a = orc.param_aggregation(torch.cat([latent, torch.zeros_like(latent)], 1)).chunk(2, 1)
        a_strings, a_sym, a_idx = code(y * am, s_a, m_a)
        y_anchor_hat = a_sym.float() + m_a
        ctx = orc.context_prediction(y_anchor_hat)
        s_n, m_n = orc.param_aggregation(torch.cat([latent, ctx], 1)).chunk(2, 1)
        n_strings, n_sym, n_idx = code(y * (1 - am), s_n, m_n)
    inter = {"y": y, "z": z, "z_sym": z_sym, "anchor_sym": a_sym, "anchor_idx": a_idx, "non_anchor_sym": n_sym,
             "non_anchor_idx": n_idx, "eb_tables": (eb_cdf, eb_len, eb_off), "gc_tables": (gc_cdf, gc_len, gc_off)}
    return [[a_strings, n_strings], z_strings], inter
