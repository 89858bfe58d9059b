// codec_host.hpp — the host-only half of the codec: coding-matrix tables, the dyadic
// (local-ring) tables, reconstruct plans per erasure pattern, and XXH64 for the
// erasureSelfTest KAT.  No HIP: zs3gpu.hip includes it, and tests/sanitize builds it
// with g++ -fsanitize=address,undefined against the scalar oracle.
//
// Reference: NewErasure / reedsolomon.New (cmd/erasure-coding.go:42-73), the argument
// checks and inversion of reedsolomon's reconstruct() behind DecodeDataBlocks /
// DecodeDataAndParityBlocks (cmd/erasure-coding.go:96-119), erasureSelfTest's
// xxhash64 (cmd/erasure-coding.go:158-216, cespare/xxhash/v2).
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/zs3gpu.h"
#include "gf256.hpp"

namespace zs3 {

// Coding matrix + device-table images of one (k, m) codec.
struct CodecTables {
    std::vector<uint8_t> matrix;   // (k+m) x k
    std::vector<uint32_t> tables;  // m x k x 8 (parity rows), then dyadic tables if dyb
    int dyb = 0;                   // 2 or 4 when the parity block is dyadic (see below)
    size_t dyadic_off = 0;         // dword offset of the dyadic tables in `tables`
};

inline int build_codec_tables(int k, int m, CodecTables& c) {
    if (k <= 0 || m <= 0) return ZS3_ERR_INV_SHARD_NUM;  // cmd/erasure-coding.go:44-50
    if (k + m > 256) return ZS3_ERR_MAX_SHARD_NUM;
    if (!build_matrix(k, m, c.matrix)) return ZS3_ERR_SINGULAR;
    c.tables.assign((size_t)m * k * 8, 0);
    for (int r = 0; r < m; ++r)
        for (int j = 0; j < k; ++j) perm_tables(c.matrix[(size_t)(k + r) * k + j], &c.tables[((size_t)r * k + j) * 8]);
    // Dyadic structure: the Vandermonde points 0..k+m-1 make the parity block of the
    // power-of-two shapes (4+2, 8+4, 12+4, 16+4, 4+4, ...) dyadic in m x m blocks,
    // P[r][q*m + t] = D_q[r ^ t], so each block is a group-algebra product that needs
    // 3 (m = 2) or 9 (m = 4) GF multiplies instead of m*m (gf_dev.hpp).
    c.dyb = 0;
    c.dyadic_off = 0;
    if ((m == 2 || m == 4) && k % m == 0) {
        bool dy = true;
        for (int r = 0; r < m && dy; ++r)
            for (int j = 0; j < k && dy; ++j) {
                const int q = j / m, t = j % m;
                dy = c.matrix[(size_t)(k + r) * k + j] == c.matrix[(size_t)k * k + q * m + (r ^ t)];
            }
        if (dy) {
            c.dyb = m;
            c.dyadic_off = c.tables.size();
            const int per = m;  // local-ring coefficients per block (gf_dev.hpp encode_dyadic)
            c.tables.resize(c.tables.size() + (size_t)(k / m) * per * 8, 0);
            for (int q = 0; q < k / m; ++q) {
                const uint8_t* D = &c.matrix[(size_t)k * k + q * m];
                uint8_t co[4];
                if (m == 2) {
                    co[0] = D[0] ^ D[1];
                    co[1] = D[1];
                } else {
                    const uint8_t a = D[0], b = D[1], cc = D[2], d = D[3];
                    co[0] = a ^ b ^ cc ^ d;
                    co[1] = b ^ d;
                    co[2] = cc ^ d;
                    co[3] = d;
                }
                for (int i = 0; i < per; ++i)
                    perm_tables(co[i], &c.tables[c.dyadic_off + ((size_t)q * per + i) * 8]);
            }
        }
    }
    return ZS3_OK;
}

// Reconstruct plan for one erasure pattern: rows[0..k) are the k shards
// ReconstructData reads (the first k present, ascending), rows[k..k+e) the rebuilt
// ones; coef is e x k (inverted sub-matrix rows for data, M[p] * inverse for parity).
struct PlanData {
    int status = ZS3_OK;  // error for this pattern, or OK
    bool noop = false;
    int e = 0;
    std::vector<int32_t> rows;
    std::vector<uint8_t> coef;
    std::vector<uint32_t> tables;  // e x k x 8
};

inline void make_plan_data(int k, int m, const uint8_t* matrix, const uint8_t* present, int data_only, PlanData& p) {
    const int n = k + m;
    int np = 0, dp = 0;
    for (int i = 0; i < n; ++i)
        if (present[i]) {
            ++np;
            if (i < k) ++dp;
        }
    if (np == 0) {
        p.status = ZS3_ERR_SHARD_NO_DATA;
        return;
    }
    std::vector<int32_t> valid;
    for (int i = 0; i < n && (int)valid.size() < k; ++i)
        if (present[i]) valid.push_back(i);
    if (np == n || (data_only && dp == k)) {
        p.noop = true;
        p.rows = valid;  // verify-only pass (zs3_verify_reconstruct_batch)
        return;
    }
    if (np < k) {
        p.status = ZS3_ERR_TOO_FEW_SHARDS;
        return;
    }
    std::vector<uint8_t> sub((size_t)k * k), dec((size_t)k * k);
    for (int r = 0; r < k; ++r) std::memcpy(&sub[(size_t)r * k], &matrix[(size_t)valid[r] * k], (size_t)k);
    if (!gf_invert(sub.data(), k, dec.data())) {
        p.status = ZS3_ERR_SINGULAR;
        return;
    }
    const GF& g = gf();
    p.rows = valid;
    for (int d = 0; d < k; ++d) {
        if (present[d]) continue;
        p.rows.push_back(d);
        p.coef.insert(p.coef.end(), &dec[(size_t)d * k], &dec[(size_t)d * k] + k);
    }
    if (!data_only) {
        // missing parity row p = M[p] * data = (M[p] * dec) * valid rows
        for (int r = k; r < n; ++r) {
            if (present[r]) continue;
            p.rows.push_back(r);
            for (int t = 0; t < k; ++t) {
                uint8_t acc = 0;
                for (int j = 0; j < k; ++j) acc ^= g.mul(matrix[(size_t)r * k + j], dec[(size_t)j * k + t]);
                p.coef.push_back(acc);
            }
        }
    }
    p.e = (int)p.rows.size() - k;
    p.tables.assign((size_t)p.e * k * 8, 0);
    for (int i = 0; i < p.e * k; ++i) perm_tables(p.coef[(size_t)i], &p.tables[(size_t)i * 8]);
}

// One byte of c*x through the packed permute tables, as the device applies them
// (gf_dev.hpp gf_lookup: c*x = Ta[x & 7] ^ Tb[(x >> 3) & 7] ^ Tc[x >> 6]).
inline uint8_t perm_mul(const uint32_t* t, uint8_t x) {
    auto byte = [](uint32_t lo, uint32_t hi, unsigned i) {
        return (uint8_t)((i < 4 ? lo >> (8 * i) : hi >> (8 * (i - 4))) & 0xFF);
    };
    return (uint8_t)(byte(t[0], t[1], x & 7u) ^ byte(t[2], t[3], (x >> 3) & 7u) ^ byte(t[4], 0, x >> 6));
}

// ---- XXH64 (erasureSelfTest hashes with cespare/xxhash/v2) ----
namespace xxh {
constexpr uint64_t P1 = 11400714785074694791ULL, P2 = 14029467366897019727ULL, P3 = 1609587929392839161ULL,
                   P4 = 9650029242287828579ULL, P5 = 2870177450012600261ULL;
inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t rd64(const uint8_t* p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
}
inline uint32_t rd32(const uint8_t* p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}
inline uint64_t round(uint64_t acc, uint64_t in) { return rotl64(acc + in * P2, 31) * P1; }
inline uint64_t merge(uint64_t acc, uint64_t v) { return (acc ^ round(0, v)) * P1 + P4; }
}  // namespace xxh

inline uint64_t xxh64(const uint8_t* p, size_t len) {
    using namespace xxh;
    const uint8_t* end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
        const uint8_t* lim = end - 32;
        do {
            v1 = round(v1, rd64(p));
            v2 = round(v2, rd64(p + 8));
            v3 = round(v3, rd64(p + 16));
            v4 = round(v4, rd64(p + 24));
            p += 32;
        } while (p <= lim);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = merge(h, v1);
        h = merge(h, v2);
        h = merge(h, v3);
        h = merge(h, v4);
    } else {
        h = P5;
    }
    h += (uint64_t)len;
    while (p + 8 <= end) {
        h ^= round(0, rd64(p));
        h = rotl64(h, 27) * P1 + P4;
        p += 8;
    }
    if (p + 4 <= end) {
        h ^= (uint64_t)rd32(p) * P1;
        h = rotl64(h, 23) * P2 + P3;
        p += 4;
    }
    while (p < end) {
        h ^= (*p) * P5;
        h = rotl64(h, 11) * P1;
        ++p;
    }
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

// erasureSelfTest's want table (cmd/erasure-coding.go:169): xxhash64 over byte(i)||shard_i.
struct SelfTestKat {
    uint8_t k, m;
    uint64_t want;
};
inline const SelfTestKat* selftest_kats(int* n) {
    static const SelfTestKat kat[] = {
        {2, 2, 0x23fb21be2496f5d3ULL}, {2, 3, 0xa5cd5600ba0d8e7cULL}, {3, 1, 0x60ab052148b010b4ULL},
        {3, 2, 0xe64927daef76435aULL}, {3, 3, 0x672f6f242b227b21ULL}, {3, 4, 0x571e41ba23a6dc6ULL},
        {4, 1, 0x524eaa814d5d86e2ULL}, {4, 2, 0x62b9552945504fefULL}, {4, 3, 0xcbf9065ee053e518ULL},
        {4, 4, 0x9a07581dcd03da8ULL},  {4, 5, 0xbf2d27b55370113fULL}, {5, 1, 0xf71031a01d70dafULL},
        {5, 2, 0x8e5845859939d0f4ULL}, {5, 3, 0x7ad9161acbb4c325ULL}, {5, 4, 0xc446b88830b4f800ULL},
        {5, 5, 0xabf1573cc6f76165ULL}, {5, 6, 0x7b5598a85045bfb8ULL}, {6, 1, 0xe2fc1e677cc7d872ULL},
        {6, 2, 0x7ed133de5ca6a58eULL}, {6, 3, 0x39ef92d0a74cc3c0ULL}, {6, 4, 0xcfc90052bc25d20ULL},
        {6, 5, 0x71c96f6baeef9c58ULL}, {6, 6, 0x4b79056484883e4cULL}, {6, 7, 0xb1a0e2427ac2dc1aULL},
        {7, 1, 0x937ba2b7af467a22ULL}, {7, 2, 0x5fd13a734d27d37aULL}, {7, 3, 0x3be2722d9b66912fULL},
        {7, 4, 0x14c628e59011be3dULL}, {7, 5, 0xcc3b39ad4c083b9fULL}, {7, 6, 0x45af361b7de7a4ffULL},
        {7, 7, 0x456cc320cec8a6e6ULL}, {7, 8, 0x1867a9f4db315b5cULL}, {8, 1, 0xbc5756b9a9ade030ULL},
        {8, 2, 0xdfd7d9d0b3e36503ULL}, {8, 3, 0x72bb72c2cdbcf99dULL}, {8, 4, 0x3ba5e9b41bf07f0ULL},
        {8, 5, 0xd7dabc15800f9d41ULL}, {8, 6, 0xb482a6169fd270fULL},  {8, 7, 0x50748e0099d657e8ULL},
        {9, 1, 0xc77ae0144fcaeb6eULL}, {9, 2, 0x8a86c7dbebf27b68ULL}, {9, 3, 0xa64e3be6d6fe7e92ULL},
        {9, 4, 0x239b71c41745d207ULL}, {9, 5, 0x2d0803094c5a86ceULL}, {9, 6, 0xa3c2539b3af84874ULL},
        {10, 1, 0x7d30d91b89fcec21ULL}, {10, 2, 0xfa5af9aa9f1857a3ULL}, {10, 3, 0x84bc4bda8af81f90ULL},
        {10, 4, 0x6c1cba8631de994aULL}, {10, 5, 0x4383e58a086cc1acULL}, {11, 1, 0x4ed2929a2df690bULL},
        {11, 2, 0xecd6f1b1399775c0ULL}, {11, 3, 0xc78cfbfc0dc64d01ULL}, {11, 4, 0xb2643390973702d6ULL},
        {12, 1, 0x3b2a88686122d082ULL}, {12, 2, 0xfd2f30a48a8e2e9ULL}, {12, 3, 0xd5ce58368ae90b13ULL},
        {13, 1, 0x9c88e2a9d1b8fff8ULL}, {13, 2, 0xcb8460aa4cf6613ULL}, {14, 1, 0x78a28bbaec57996eULL},
    };
    *n = (int)(sizeof kat / sizeof kat[0]);
    return kat;
}

}  // namespace zs3
