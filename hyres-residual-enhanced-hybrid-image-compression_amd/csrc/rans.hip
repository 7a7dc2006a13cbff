// Entropy coding for compress/decompress: the host side of compressai 1.2.6's
// rANS path that LightWeightCheckerboard.compress/decompress (models/checkerboard.py:159-240) and
// ResidualJPEGCompression.compress/decompress (models/hyres.py:78-131) call through
// GaussianConditional / EntropyBottleneck .compress / .decompress and .update().
//
// Restated from compressai's published algorithm (compressai/cpp_exts/rans/rans_interface.cpp,
// compressai/cpp_exts/ops/ops.cpp, ryg_rans rans64.h): 64-bit-state rANS with 32-bit words, 16-bit
// quantized CDFs, symbols outside a CDF's range escape through a bypass code of 4-bit chunks. The coder is
// inherently sequential per stream (one string per image), so it stays on the host; the per-element work
// around it (CDF index building, symbolisation, dequantisation) runs in HIP kernels (entropy.hip).
#include "common.h"

#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace hyres {
namespace rans {

constexpr uint64_t RANS64_L = 1ull << 31;  // lower bound of the normalisation interval (64-bit state)
constexpr int PRECISION = 16;
constexpr int BYPASS_PRECISION = 4;
constexpr int MAX_BYPASS_VAL = (1 << BYPASS_PRECISION) - 1;

struct Sym {
    uint16_t start, range;
    bool bypass;
};

// 64-bit state, 32-bit output words written backwards (ryg_rans rans64 as used by compressai)
struct Enc {
    uint64_t x = RANS64_L;
    std::vector<uint32_t> rev;  // words in reverse output order
    void put(uint32_t start, uint32_t freq, int scale_bits) {
        const uint64_t x_max = ((RANS64_L >> scale_bits) << 32) * freq;
        if (x >= x_max) {
            rev.push_back((uint32_t)x);
            x >>= 32;
        }
        x = ((x / freq) << scale_bits) + (x % freq) + start;
    }
    void put_bits(uint32_t val, int nbits) {  // compressai Rans64EncPutBits (nbits <= 16)
        const uint32_t freq = 1u << (16 - nbits);
        const uint64_t x_max = ((RANS64_L >> 16) << 32) * freq;
        if (x >= x_max) {
            rev.push_back((uint32_t)x);
            x >>= 32;
        }
        x = (x << nbits) | val;
    }
    void flush() {  // ptr -= 2; ptr[0] = low word, ptr[1] = high word
        rev.push_back((uint32_t)(x >> 32));
        rev.push_back((uint32_t)x);
    }
};

struct Dec {
    uint64_t x = 0;
    const uint32_t* p;
    const uint32_t* end;
    uint32_t next() { return p < end ? *p++ : 0u; }
    void init(const uint32_t* b, const uint32_t* e) {
        p = b;
        end = e;
        x = (uint64_t)next();
        x |= (uint64_t)next() << 32;
    }
    uint32_t get(int scale_bits) const { return (uint32_t)(x & ((1u << scale_bits) - 1)); }
    void advance(uint32_t start, uint32_t freq, int scale_bits) {
        const uint64_t mask = (1ull << scale_bits) - 1;
        x = freq * (x >> scale_bits) + (x & mask) - start;
        if (x < RANS64_L) x = (x << 32) | next();
    }
    uint32_t get_bits(int nbits) {
        const uint32_t v = (uint32_t)(x & ((1u << nbits) - 1));
        x >>= nbits;
        if (x < RANS64_L) x = (x << 32) | next();
        return v;
    }
};

}  // namespace rans
}  // namespace hyres

using namespace hyres;

extern "C" {

int hyres_pmf_to_quantized_cdf(const float* pmf, int n, int precision, int* cdf_out) {
    HY_REQUIRE(pmf && cdf_out && n > 0 && precision > 0 && precision <= 24, HYRES_E_ARG, "pmf_to_cdf: bad args");
    std::vector<uint32_t> cdf(n + 1);
    cdf[0] = 0;
    for (int i = 0; i < n; ++i) {
        const float p = pmf[i];
        HY_REQUIRE(p >= 0.f && std::isfinite(p), HYRES_E_ARG, "pmf_to_cdf: invalid probability %g", (double)p);
        cdf[i + 1] = (uint32_t)std::lround((double)p * (double)(1u << precision));
    }
    uint64_t total = 0;
    for (uint32_t v : cdf) total += v;
    HY_REQUIRE(total > 0, HYRES_E_ARG, "pmf_to_cdf: all probabilities round to zero");
    for (auto& v : cdf) v = (uint32_t)(((uint64_t)(1u << precision) * v) / total);
    for (int i = 1; i <= n; ++i) cdf[i] += cdf[i - 1];
    cdf[n] = 1u << precision;
    for (int i = 0; i < n; ++i) {
        if (cdf[i] == cdf[i + 1]) {  // zero-frequency symbol: steal one unit from the smallest freq > 1
            uint32_t best_freq = ~0u;
            int best_steal = -1;
            for (int j = 0; j < n; ++j) {
                const uint32_t freq = cdf[j + 1] - cdf[j];
                if (freq > 1 && freq < best_freq) {
                    best_freq = freq;
                    best_steal = j;
                }
            }
            HY_REQUIRE(best_steal != -1, HYRES_E_ARG, "pmf_to_cdf: cannot make every frequency non-zero");
            if (best_steal < i) {
                for (int j = best_steal + 1; j <= i; ++j) cdf[j]--;
            } else {
                for (int j = i + 1; j <= best_steal; ++j) cdf[j]++;
            }
        }
    }
    for (int i = 0; i <= n; ++i) cdf_out[i] = (int)cdf[i];
    return ok();
}

int hyres_rans_encode_with_indexes(const int* symbols, const int* indexes, long long n, const int* cdfs,
                                   int cdf_stride, const int* cdf_sizes, const int* offsets, int ncdf,
                                   unsigned char* out, long long out_cap, long long* out_len) {
    HY_REQUIRE(symbols && indexes && cdfs && cdf_sizes && offsets && out_len && n >= 0, HYRES_E_ARG,
               "rans_encode: NULL");
    std::vector<rans::Sym> syms;
    syms.reserve((size_t)n + 16);
    for (long long i = 0; i < n; ++i) {
        const int ci = indexes[i];
        HY_REQUIRE(ci >= 0 && ci < ncdf, HYRES_E_ARG, "rans_encode: cdf index %d out of [0,%d)", ci, ncdf);
        const int* cdf = cdfs + (long long)ci * cdf_stride;
        const int max_value = cdf_sizes[ci] - 2;
        HY_REQUIRE(max_value >= 0 && max_value + 1 < cdf_stride, HYRES_E_ARG, "rans_encode: bad cdf size");
        int value = symbols[i] - offsets[ci];
        uint32_t raw_val = 0;
        if (value < 0) {
            raw_val = (uint32_t)(-2 * value - 1);
            value = max_value;
        } else if (value >= max_value) {
            raw_val = (uint32_t)(2 * (value - max_value));
            value = max_value;
        }
        syms.push_back({(uint16_t)cdf[value], (uint16_t)(cdf[value + 1] - cdf[value]), false});
        if (value == max_value) {  // bypass: count of 4-bit chunks (itself chunked), then the chunks
            int n_bypass = 0;
            while ((raw_val >> (n_bypass * rans::BYPASS_PRECISION)) != 0) ++n_bypass;
            int val = n_bypass;
            while (val >= rans::MAX_BYPASS_VAL) {
                syms.push_back({(uint16_t)rans::MAX_BYPASS_VAL, (uint16_t)(rans::MAX_BYPASS_VAL + 1), true});
                val -= rans::MAX_BYPASS_VAL;
            }
            syms.push_back({(uint16_t)val, (uint16_t)(val + 1), true});
            for (int j = 0; j < n_bypass; ++j) {
                const int v = (int)((raw_val >> (j * rans::BYPASS_PRECISION)) & rans::MAX_BYPASS_VAL);
                syms.push_back({(uint16_t)v, (uint16_t)(v + 1), true});
            }
        }
    }
    rans::Enc enc;
    for (size_t k = syms.size(); k-- > 0;) {
        const rans::Sym& s = syms[k];
        if (!s.bypass) enc.put(s.start, s.range, rans::PRECISION);
        else enc.put_bits(s.start, rans::BYPASS_PRECISION);
    }
    enc.flush();
    const long long words = (long long)enc.rev.size();
    const long long len = 4 * words;
    *out_len = len;
    if (!out) return ok();  // size query
    HY_REQUIRE(out_cap >= len, HYRES_E_WORKSPACE, "rans_encode: output buffer %lld < %lld", out_cap, len);
    for (long long k = 0; k < words; ++k) {
        const uint32_t w = enc.rev[(size_t)(words - 1 - k)];  // little-endian words, memory order
        memcpy(out + 4 * k, &w, 4);
    }
    return ok();
}

int hyres_rans_decode_with_indexes(const unsigned char* in, long long in_len, const int* indexes, long long n,
                                   const int* cdfs, int cdf_stride, const int* cdf_sizes, const int* offsets,
                                   int ncdf, int* symbols_out) {
    HY_REQUIRE(in && indexes && cdfs && cdf_sizes && offsets && symbols_out && in_len >= 8 && in_len % 4 == 0,
               HYRES_E_ARG, "rans_decode: bad args");
    std::vector<uint32_t> words((size_t)(in_len / 4));
    memcpy(words.data(), in, (size_t)in_len);
    rans::Dec dec;
    dec.init(words.data(), words.data() + words.size());
    for (long long i = 0; i < n; ++i) {
        const int ci = indexes[i];
        HY_REQUIRE(ci >= 0 && ci < ncdf, HYRES_E_ARG, "rans_decode: cdf index %d out of [0,%d)", ci, ncdf);
        const int* cdf = cdfs + (long long)ci * cdf_stride;
        const int max_value = cdf_sizes[ci] - 2;
        const uint32_t cum = dec.get(rans::PRECISION);
        // s with cdf[s] <= cum < cdf[s+1] (compressai scans linearly; the CDF is strictly increasing, so a
        // binary search finds the same s in O(log L) — wide scales have L in the thousands)
        int lo = 0, hi = max_value;  // cdf[max_value + 1] = 2^16 > cum
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if ((uint32_t)cdf[mid] <= cum) lo = mid;
            else hi = mid - 1;
        }
        const int s = lo;
        dec.advance((uint32_t)cdf[s], (uint32_t)(cdf[s + 1] - cdf[s]), rans::PRECISION);
        int value = s;
        if (value == max_value) {
            int val = (int)dec.get_bits(rans::BYPASS_PRECISION);
            int n_bypass = val;
            while (val == rans::MAX_BYPASS_VAL) {
                val = (int)dec.get_bits(rans::BYPASS_PRECISION);
                n_bypass += val;
            }
            uint32_t raw_val = 0;
            for (int j = 0; j < n_bypass; ++j) {
                val = (int)dec.get_bits(rans::BYPASS_PRECISION);
                raw_val |= (uint32_t)val << (j * rans::BYPASS_PRECISION);
            }
            value = (int)(raw_val >> 1);
            if (raw_val & 1) value = -value - 1;
            else value += max_value;
        }
        symbols_out[i] = value + offsets[ci];
    }
    return ok();
}

}  // extern "C"
