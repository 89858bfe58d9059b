// host_check.cpp — host-side code under AddressSanitizer + UndefinedBehaviorSanitizer
// (the reference has Go -race; the native side gets ASan/UBSan host tests).
//
// Built by tests/test_sanitize.py with g++ -fsanitize=address,undefined together with
// oracle/zs3_oracle.c and oracle/cpu_ref.cpp.  It exercises the product's host-only
// codec half (zs3server_amd/csrc/codec_host.hpp: coding matrix, permute tables, dyadic
// tables, reconstruct plans, XXH64) and the two CPU restatements:
//   1. erasureSelfTest's 60 KATs (cmd/erasure-coding.go:158-216) computed from the
//      product's device tables applied byte by byte on the host, and from the oracle;
//   2. every erasure pattern of every (k, m) with k + m <= 8, ReconstructData and
//      Reconstruct: the product's plan (status, rows, coefficients through the permute
//      tables) against oracle_reconstruct (reedsolomon reconstruct(), erasure-coding.go:96-119);
//   3. the dyadic local-ring tables of RS(4+2), (4+4), (8+4), (12+4), (16+4): the
//      gf_dev.hpp encode_dyadic arithmetic restated on the host vs the oracle's parity;
//   4. cpu_ref's encode + HighwayHash-256 vs the oracle on ragged blocks.
// Exit status 0 = all checks passed; any sanitizer report aborts (halt_on_error).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../zs3server_amd/csrc/codec_host.hpp"

extern "C" {
int oracle_build_matrix(int k, int m, uint8_t* out);
int64_t oracle_encode_data(const uint8_t* matrix, int k, int m, const uint8_t* data, int64_t len, uint8_t* shards);
int oracle_reconstruct(const uint8_t* matrix, int k, int m, uint8_t* shards, int64_t per, const uint8_t* present,
                       int data_only);
void oracle_hh256(const uint8_t key[32], const uint8_t* msg, size_t len, uint8_t out[32]);
int64_t cpuref_encode_hash(int k, int m, const uint8_t* matrix, const uint8_t* data, int64_t block_len,
                           int64_t n_blocks, int64_t data_stride, uint8_t* parity, int64_t parity_stride,
                           uint8_t* sums, const uint8_t* key, int threads);
}

static int g_fail = 0;
#define CHECK(cond, ...)                      \
    do {                                      \
        if (!(cond)) {                        \
            std::fprintf(stderr, __VA_ARGS__); \
            std::fprintf(stderr, "\n");       \
            ++g_fail;                         \
        }                                     \
    } while (0)

static const uint8_t kKey[32] = {0x4b, 0xe7, 0x34, 0xfa, 0x8e, 0x23, 0x8a, 0xcd, 0x26, 0x3e, 0x83,
                                 0xe6, 0xbb, 0x96, 0x85, 0x52, 0x04, 0x0f, 0x93, 0x5d, 0xa3, 0x9f,
                                 0x44, 0x14, 0x97, 0xe0, 0x9d, 0x13, 0x22, 0xde, 0x36, 0xa0};

// parity of one block through the product's parity-row permute tables
static std::vector<uint8_t> encode_with_tables(const zs3::CodecTables& c, int k, int m, const uint8_t* data,
                                               int64_t len, int64_t* per_out) {
    const int64_t per = (len + k - 1) / k;
    std::vector<uint8_t> sh((size_t)(k + m) * per, 0);
    std::memcpy(sh.data(), data, (size_t)len);
    for (int r = 0; r < m; ++r)
        for (int j = 0; j < k; ++j) {
            const uint32_t* t = &c.tables[((size_t)r * k + j) * 8];
            for (int64_t b = 0; b < per; ++b) sh[(size_t)(k + r) * per + b] ^= zs3::perm_mul(t, sh[(size_t)j * per + b]);
        }
    *per_out = per;
    return sh;
}

static void check_selftest_kats() {
    int n = 0;
    const zs3::SelfTestKat* kat = zs3::selftest_kats(&n);
    CHECK(n == 60, "selftest table has %d entries", n);
    uint8_t data[256];
    for (int i = 0; i < 256; ++i) data[i] = (uint8_t)i;
    for (int i = 0; i < n; ++i) {
        const int k = kat[i].k, m = kat[i].m, R = k + m;
        zs3::CodecTables c;
        CHECK(zs3::build_codec_tables(k, m, c) == ZS3_OK, "build_codec_tables(%d,%d)", k, m);
        std::vector<uint8_t> om((size_t)R * k);
        oracle_build_matrix(k, m, om.data());
        CHECK(om == c.matrix, "matrix (%d,%d) differs from the oracle", k, m);
        int64_t per = 0;
        std::vector<uint8_t> sh = encode_with_tables(c, k, m, data, 256, &per);
        std::vector<uint8_t> osh((size_t)R * per);
        CHECK(oracle_encode_data(om.data(), k, m, data, 256, osh.data()) == per, "per (%d,%d)", k, m);
        CHECK(osh == sh, "parity (%d,%d) differs from the oracle", k, m);
        std::vector<uint8_t> stream;
        for (int r = 0; r < R; ++r) {
            stream.push_back((uint8_t)r);
            stream.insert(stream.end(), sh.begin() + (size_t)r * per, sh.begin() + (size_t)(r + 1) * per);
        }
        CHECK(zs3::xxh64(stream.data(), stream.size()) == kat[i].want, "erasureSelfTest KAT (%d,%d)", k, m);
    }
}

static void check_all_patterns(int k, int m, std::mt19937_64& rng) {
    const int R = k + m;
    const int64_t per = 37;  // odd shard size: no alignment assumptions
    zs3::CodecTables c;
    CHECK(zs3::build_codec_tables(k, m, c) == ZS3_OK, "build_codec_tables(%d,%d)", k, m);
    std::vector<uint8_t> data((size_t)k * per);
    for (auto& x : data) x = (uint8_t)rng();
    std::vector<uint8_t> full((size_t)R * per);
    oracle_encode_data(c.matrix.data(), k, m, data.data(), (int64_t)data.size(), full.data());
    for (uint32_t mask = 0; mask < (1u << R); ++mask) {
        uint8_t present[16];
        for (int i = 0; i < R; ++i) present[i] = (mask >> i) & 1u;
        for (int data_only = 0; data_only < 2; ++data_only) {
            std::vector<uint8_t> want = full;
            for (int i = 0; i < R; ++i)
                if (!present[i]) std::memset(&want[(size_t)i * per], 0xA5, (size_t)per);
            const int orc = oracle_reconstruct(c.matrix.data(), k, m, want.data(), per, present, data_only);
            zs3::PlanData p;
            zs3::make_plan_data(k, m, c.matrix.data(), present, data_only, p);
            CHECK(p.status == orc, "(%d,%d) mask %x data_only %d: plan status %d, oracle %d", k, m, mask, data_only,
                  p.status, orc);
            if (p.status || orc) continue;
            if (p.noop) continue;
            CHECK((int)p.rows.size() == k + p.e && (int)p.coef.size() == p.e * k &&
                      p.tables.size() == (size_t)p.e * k * 8,
                  "(%d,%d) mask %x: plan sizes", k, m, mask);
            std::vector<uint8_t> got = want;
            for (int i = 0; i < R; ++i)
                if (!present[i]) std::memset(&got[(size_t)i * per], 0xA5, (size_t)per);
            for (int o = 0; o < p.e; ++o) {
                const int row = p.rows[(size_t)(k + o)];
                CHECK(row >= 0 && row < R && !present[row], "(%d,%d) mask %x: output row %d", k, m, mask, row);
                std::vector<uint8_t> acc((size_t)per, 0);
                for (int t = 0; t < k; ++t) {
                    const int in = p.rows[(size_t)t];
                    const uint32_t* tab = &p.tables[((size_t)o * k + t) * 8];
                    for (int64_t b = 0; b < per; ++b) acc[(size_t)b] ^= zs3::perm_mul(tab, full[(size_t)in * per + b]);
                }
                std::memcpy(&got[(size_t)row * per], acc.data(), (size_t)per);
            }
            CHECK(got == want, "(%d,%d) mask %x data_only %d: rebuilt rows differ from the oracle", k, m, mask,
                  data_only);
        }
    }
}

// gf_dev.hpp encode_dyadic restated per byte on the host, from the dyadic tables
static void check_dyadic(int k, int m, std::mt19937_64& rng) {
    zs3::CodecTables c;
    CHECK(zs3::build_codec_tables(k, m, c) == ZS3_OK, "build_codec_tables(%d,%d)", k, m);
    CHECK(c.dyb == m, "(%d,%d) expected a dyadic parity block", k, m);
    if (c.dyb != m) return;
    const int64_t per = 64;
    std::vector<uint8_t> data((size_t)k * per);
    for (auto& x : data) x = (uint8_t)rng();
    std::vector<uint8_t> want((size_t)(k + m) * per);
    oracle_encode_data(c.matrix.data(), k, m, data.data(), (int64_t)data.size(), want.data());
    const uint32_t* dt = &c.tables[c.dyadic_off];
    auto mul = [&](int q, int i, uint8_t x) { return zs3::perm_mul(dt + ((size_t)q * m + i) * 8, x); };
    for (int64_t b = 0; b < per; ++b) {
        uint8_t Y[4] = {0, 0, 0, 0};
        for (int q = 0; q < k / m; ++q) {
            const uint8_t* x = &data[(size_t)q * m * per];
            if (m == 4) {
                const uint8_t x0 = x[b], x1 = x[per + b], x2 = x[2 * per + b], x3 = x[3 * per + b];
                const uint8_t X0 = x0 ^ x1 ^ x2 ^ x3, X1 = x1 ^ x3, X2 = x2 ^ x3, X3 = x3;
                Y[0] ^= mul(q, 0, X0);
                Y[1] ^= mul(q, 0, X1) ^ mul(q, 1, X0);
                Y[2] ^= mul(q, 0, X2) ^ mul(q, 2, X0);
                Y[3] ^= mul(q, 0, X3) ^ mul(q, 1, X2) ^ mul(q, 2, X1) ^ mul(q, 3, X0);
            } else {
                const uint8_t x0 = x[b], x1 = x[per + b];
                Y[0] ^= mul(q, 0, x0 ^ x1);
                Y[1] ^= mul(q, 0, x1) ^ mul(q, 1, x0 ^ x1);
            }
        }
        uint8_t y[4];
        if (m == 4) {
            y[0] = Y[0] ^ Y[1] ^ Y[2] ^ Y[3];
            y[1] = Y[1] ^ Y[3];
            y[2] = Y[2] ^ Y[3];
            y[3] = Y[3];
        } else {
            y[0] = Y[0] ^ Y[1];
            y[1] = Y[1];
        }
        for (int r = 0; r < m; ++r)
            CHECK(y[r] == want[(size_t)(k + r) * per + b], "(%d,%d) dyadic parity row %d byte %lld", k, m, r,
                  (long long)b);
    }
}

static void check_cpuref(int k, int m, int64_t blen, int threads, std::mt19937_64& rng) {
    const int R = k + m;
    const int64_t S = (blen + k - 1) / k;
    const int nb = 2;
    std::vector<uint8_t> mat((size_t)R * k);
    oracle_build_matrix(k, m, mat.data());
    std::vector<uint8_t> data((size_t)(nb * blen));
    for (auto& x : data) x = (uint8_t)rng();
    std::vector<uint8_t> par((size_t)(nb * m * S)), sums((size_t)nb * R * 32);
    CHECK(cpuref_encode_hash(k, m, mat.data(), data.data(), blen, nb, blen, par.data(), m * S, sums.data(), kKey,
                             threads) == S,
          "cpuref S");
    for (int b = 0; b < nb; ++b) {
        std::vector<uint8_t> sh((size_t)R * S);
        oracle_encode_data(mat.data(), k, m, &data[(size_t)(b * blen)], blen, sh.data());
        CHECK(std::memcmp(&par[(size_t)(b * m * S)], &sh[(size_t)k * S], (size_t)(m * S)) == 0,
              "cpuref parity (%d,%d) len %lld block %d", k, m, (long long)blen, b);
        for (int r = 0; r < R; ++r) {
            uint8_t h[32];
            oracle_hh256(kKey, &sh[(size_t)r * S], (size_t)S, h);
            CHECK(std::memcmp(h, &sums[((size_t)b * R + r) * 32], 32) == 0, "cpuref sum (%d,%d) len %lld row %d", k,
                  m, (long long)blen, r);
        }
    }
}

int main() {
    std::mt19937_64 rng(12345);
    check_selftest_kats();
    int shapes = 0;
    for (int k = 1; k < 8; ++k)
        for (int m = 1; k + m <= 8; ++m) {
            check_all_patterns(k, m, rng);
            ++shapes;
        }
    const int dy[][2] = {{4, 2}, {4, 4}, {8, 4}, {12, 4}, {16, 4}, {8, 2}};
    for (const auto& s : dy) check_dyadic(s[0], s[1], rng);
    const int64_t lens[] = {1, 17, 84, 4099, (1 << 16) + 3};
    for (int64_t L : lens) {
        check_cpuref(4, 2, L, 1, rng);
        check_cpuref(8, 4, L, 3, rng);
        check_cpuref(16, 4, L, 2, rng);
    }
    if (g_fail) {
        std::fprintf(stderr, "host_check: %d failures\n", g_fail);
        return 1;
    }
    std::printf("host_check: ok (60 KATs, all erasure patterns of %d shapes with k+m <= 8, 6 dyadic shapes, "
                "cpu_ref on 15 ragged cases)\n",
                shapes);
    return 0;
}
