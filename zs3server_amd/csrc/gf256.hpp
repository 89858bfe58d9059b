// gf256.hpp — host-side GF(2^8) arithmetic for the zs3gpu codec.
//
// Field and matrix construction follow klauspost/reedsolomon v1.11.8's default
// codec as used by cmd/erasure-coding.go:63 (reedsolomon.New): polynomial 0x11D,
// generator 2, systematic matrix M = Vandermonde(k+m, k) * inverse(top k x k).
// Only small matrices are built here (per (k, m) codec and per erasure pattern);
// all byte-stream arithmetic runs in the HIP kernels.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

namespace zs3 {

struct GF {
    uint8_t exp[512];
    uint8_t log[256];
    GF() {
        unsigned x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = (uint8_t)x;
            log[x] = (uint8_t)i;
            x <<= 1;
            if (x & 0x100) x ^= 0x11D;
        }
        for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
        log[0] = 0;
    }
    uint8_t mul(uint8_t a, uint8_t b) const {
        return (a && b) ? exp[log[a] + log[b]] : 0;
    }
    uint8_t div(uint8_t a, uint8_t b) const {
        if (!a) return 0;
        int d = (int)log[a] - (int)log[b];
        return exp[d < 0 ? d + 255 : d];
    }
    uint8_t pow(uint8_t a, int n) const {  // galExp
        if (n == 0) return 1;
        if (a == 0) return 0;
        return exp[((int)log[a] * n) % 255];
    }
};

inline const GF& gf() {
    static const GF g;
    return g;
}

// Gauss-Jordan inversion over GF(2^8); returns false if singular.
inline bool gf_invert(const uint8_t* in, int n, uint8_t* out) {
    const GF& g = gf();
    const int cols = 2 * n;
    std::vector<uint8_t> w((size_t)n * cols, 0);
    for (int r = 0; r < n; ++r) {
        std::memcpy(&w[(size_t)r * cols], in + (size_t)r * n, n);
        w[(size_t)r * cols + n + r] = 1;
    }
    for (int r = 0; r < n; ++r) {
        uint8_t* row = &w[(size_t)r * cols];
        if (row[r] == 0) {
            for (int rb = r + 1; rb < n; ++rb) {
                if (w[(size_t)rb * cols + r]) {
                    for (int c = 0; c < cols; ++c) std::swap(row[c], w[(size_t)rb * cols + c]);
                    break;
                }
            }
        }
        if (row[r] == 0) return false;
        if (row[r] != 1) {
            const uint8_t s = g.div(1, row[r]);
            for (int c = 0; c < cols; ++c) row[c] = g.mul(row[c], s);
        }
        for (int o = 0; o < n; ++o) {
            if (o == r) continue;
            uint8_t* ro = &w[(size_t)o * cols];
            const uint8_t s = ro[r];
            if (s)
                for (int c = 0; c < cols; ++c) ro[c] ^= g.mul(s, row[c]);
        }
    }
    for (int r = 0; r < n; ++r) std::memcpy(out + (size_t)r * n, &w[(size_t)r * cols + n], n);
    return true;
}

// (k+m) x k systematic coding matrix, row-major.
inline bool build_matrix(int k, int m, std::vector<uint8_t>& out) {
    const GF& g = gf();
    const int n = k + m;
    std::vector<uint8_t> v((size_t)n * k), inv((size_t)k * k);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) v[(size_t)r * k + c] = g.pow((uint8_t)r, c);
    if (!gf_invert(v.data(), k, inv.data())) return false;
    out.assign((size_t)n * k, 0);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) {
            uint8_t acc = 0;
            for (int t = 0; t < k; ++t) acc ^= g.mul(v[(size_t)r * k + t], inv[(size_t)t * k + c]);
            out[(size_t)r * k + c] = acc;
        }
    return true;
}

// Per-coefficient byte-permute tables for the device GF multiply.
// c*x = Ta[x & 7] ^ Tb[(x >> 3) & 7] ^ Tc[x >> 6]   (GF multiply is GF(2)-linear in x)
// Five dwords per coefficient: Ta.lo, Ta.hi, Tb.lo, Tb.hi, Tc — v_perm_b32 selects
// byte i of {hi:lo} for selector byte i in 0..7.
constexpr int kPermDwords = 5;

inline void perm_tables(uint8_t c, uint32_t out[kPermDwords]) {
    const GF& g = gf();
    uint8_t ta[8], tb[8], tc[4];
    for (int i = 0; i < 8; ++i) {
        ta[i] = g.mul(c, (uint8_t)i);
        tb[i] = g.mul(c, (uint8_t)(i << 3));
    }
    for (int i = 0; i < 4; ++i) tc[i] = g.mul(c, (uint8_t)(i << 6));
    auto pack = [](const uint8_t* b) {
        return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    };
    out[0] = pack(ta);
    out[1] = pack(ta + 4);
    out[2] = pack(tb);
    out[3] = pack(tb + 4);
    out[4] = pack(tc);
}

}  // namespace zs3
