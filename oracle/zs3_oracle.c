/*
 * zs3_oracle.c — CPU restatement of the reference's erasure-shard + bitrot-hash
 * path.  TEST INFRASTRUCTURE ONLY: linked/loaded exclusively by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
 * The product path (zs3server_amd/, libzs3gpu.so) never links or calls this.
 *
 * Parity status: PINNED.  The restatement reproduces the reference's own
 * known-answer tests (tests/test_oracle_kats.py):
 *   - erasureSelfTest golden table, cmd/erasure-coding.go:158-216 (60 (k,m)
 *     configs, xxhash64 over byte(i)||shard_i of bytes(range(256)));
 *   - bitrotSelfTest chained HighwayHash-256 digest, cmd/bitrot.go:218-249;
 *   - the magic HH-256 key derivation, cmd/bitrot.go:36-37 (HH256 under a zero
 *     key of the first 100 decimals of pi; pins the size_mod32 = 4 branch).
 * The HH remainder branches the KATs do not reach (size_mod32 & 16, and
 * size_mod4 != 0) are cross-checked against the independent Python
 * restatement in oracle/pyoracle.py.
 *
 * The arithmetic lives in two third-party Go modules that are NOT vendored in
 * /root/reference (go.mod:48, go.mod:54):
 *   - github.com/klauspost/reedsolomon v1.11.8 — default codec: GF(2^8) over
 *     x^8+x^4+x^3+x^2+1 (0x11D), generator 2, systematic matrix
 *     Vandermonde(k+m, k) * inverse(top k x k), Split (ceil, zero pad),
 *     Encode, ReconstructData, Reconstruct.
 *   - github.com/minio/highwayhash v1.0.2 — HighwayHash-256 (== Google's C
 *     reference implementation, 32-byte packets, 10 finalisation rounds).
 * Both are restated here from their published algorithms.
 *
 * Plain C99, scalar, deliberately simple.  Exported with C linkage for ctypes.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Error codes: mirror include/zs3gpu.h (reedsolomon sentinels, erasure-utils.go:52,58) */
#define OR_OK 0
#define OR_ERR_INV_SHARD_NUM -1
#define OR_ERR_MAX_SHARD_NUM -2
#define OR_ERR_TOO_FEW_SHARDS -3
#define OR_ERR_SHARD_NO_DATA -4
#define OR_ERR_SHARD_SIZE -5
#define OR_ERR_SHORT_DATA -6
#define OR_ERR_SINGULAR -11

/* ------------------------------------------------------------------------ */
/* GF(2^8), polynomial 0x11D, generator 2 (klauspost galois.go tables).     */
static uint8_t g_exp[512];
static uint8_t g_log[256];
static int g_init = 0;

static void gf_init(void) {
    if (g_init) return;
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
        g_exp[i] = (uint8_t)x;
        g_log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; i++) g_exp[i] = g_exp[i - 255];
    g_log[0] = 0; /* unused */
    g_init = 1;
}

uint8_t oracle_gf_mul(uint8_t a, uint8_t b) {
    gf_init();
    if (a == 0 || b == 0) return 0;
    return g_exp[g_log[a] + g_log[b]];
}

static uint8_t gf_div(uint8_t a, uint8_t b) { /* b != 0 */
    if (a == 0) return 0;
    int d = (int)g_log[a] - (int)g_log[b];
    if (d < 0) d += 255;
    return g_exp[d];
}

/* galExp(a, n): klauspost galois.go — 1 if n==0, 0 if a==0, else exp[(log a * n) % 255] */
static uint8_t gf_exp_pow(uint8_t a, int n) {
    if (n == 0) return 1;
    if (a == 0) return 0;
    int l = ((int)g_log[a] * n) % 255;
    return g_exp[l];
}

/* Gauss-Jordan inversion of an n x n matrix over GF(2^8) (klauspost
 * matrix.go gaussianElimination on [M | I]).  Returns 0 or OR_ERR_SINGULAR. */
int oracle_gf_invert(const uint8_t* in, int n, uint8_t* out) {
    gf_init();
    int cols = 2 * n;
    uint8_t* w = (uint8_t*)malloc((size_t)n * cols);
    for (int r = 0; r < n; r++) {
        for (int c = 0; c < n; c++) w[r * cols + c] = in[r * n + c];
        for (int c = 0; c < n; c++) w[r * cols + n + c] = (uint8_t)(r == c);
    }
    for (int r = 0; r < n; r++) {
        if (w[r * cols + r] == 0) {
            for (int rb = r + 1; rb < n; rb++) {
                if (w[rb * cols + r] != 0) {
                    for (int c = 0; c < cols; c++) {
                        uint8_t t = w[r * cols + c];
                        w[r * cols + c] = w[rb * cols + c];
                        w[rb * cols + c] = t;
                    }
                    break;
                }
            }
        }
        if (w[r * cols + r] == 0) { free(w); return OR_ERR_SINGULAR; }
        if (w[r * cols + r] != 1) {
            uint8_t s = gf_div(1, w[r * cols + r]);
            for (int c = 0; c < cols; c++) w[r * cols + c] = oracle_gf_mul(w[r * cols + c], s);
        }
        for (int rb = r + 1; rb < n; rb++) {
            uint8_t s = w[rb * cols + r];
            if (s) for (int c = 0; c < cols; c++) w[rb * cols + c] ^= oracle_gf_mul(s, w[r * cols + c]);
        }
    }
    for (int d = 0; d < n; d++) {
        for (int ra = 0; ra < d; ra++) {
            uint8_t s = w[ra * cols + d];
            if (s) for (int c = 0; c < cols; c++) w[ra * cols + c] ^= oracle_gf_mul(s, w[d * cols + c]);
        }
    }
    for (int r = 0; r < n; r++) memcpy(out + r * n, w + r * cols + n, (size_t)n);
    free(w);
    return OR_OK;
}

/* buildMatrix (klauspost reedsolomon.go): V[r][c] = galExp(byte(r), c) for
 * r < k+m, c < k; M = V * inverse(V[0:k]).  out is (k+m) x k row-major.
 * Checks mirror NewErasure, cmd/erasure-coding.go:44-50. */
int oracle_build_matrix(int k, int m, uint8_t* out) {
    gf_init();
    if (k <= 0 || m <= 0) return OR_ERR_INV_SHARD_NUM;
    if (k + m > 256) return OR_ERR_MAX_SHARD_NUM;
    int n = k + m;
    uint8_t* v = (uint8_t*)malloc((size_t)n * k);
    uint8_t* inv = (uint8_t*)malloc((size_t)k * k);
    for (int r = 0; r < n; r++)
        for (int c = 0; c < k; c++) v[r * k + c] = gf_exp_pow((uint8_t)r, c);
    int rc = oracle_gf_invert(v, k, inv);
    if (rc) { free(v); free(inv); return rc; }
    for (int r = 0; r < n; r++)
        for (int c = 0; c < k; c++) {
            uint8_t acc = 0;
            for (int t = 0; t < k; t++) acc ^= oracle_gf_mul(v[r * k + t], inv[t * k + c]);
            out[r * k + c] = acc;
        }
    free(v); free(inv);
    return OR_OK;
}

/* ShardSize, cmd/erasure-coding.go:122-124 (ceilFrac, cmd/utils.go:691). */
int64_t oracle_ceil_frac(int64_t num, int64_t den) {
    if (den == 0) return 0;
    if (den < 0) { num = -num; den = -den; }
    int64_t c = num / den;
    if (num > 0 && num % den != 0) c++;
    return c;
}

/* Split + Encode, i.e. Erasure.EncodeData (cmd/erasure-coding.go:77-91) on a
 * single block of `len` bytes.  `shards` receives (k+m) * per bytes, row i =
 * shard i (data rows zero-padded exactly like reedsolomon.Split).  Returns
 * per (shard size) or a negative error; len == 0 returns 0 (k+m empty shards). */
int64_t oracle_encode_data(const uint8_t* matrix, int k, int m, const uint8_t* data,
                           int64_t len, uint8_t* shards) {
    gf_init();
    if (len == 0) return 0;
    int64_t per = oracle_ceil_frac(len, k);
    memset(shards, 0, (size_t)((k + m) * per));
    memcpy(shards, data, (size_t)len);
    for (int r = 0; r < m; r++) {
        uint8_t* out = shards + (int64_t)(k + r) * per;
        for (int j = 0; j < k; j++) {
            uint8_t c = matrix[(k + r) * k + j];
            const uint8_t* in = shards + (int64_t)j * per;
            if (c == 0) continue;
            int lc = g_log[c];
            for (int64_t b = 0; b < per; b++) {
                uint8_t x = in[b];
                if (x) out[b] ^= g_exp[lc + g_log[x]];
            }
        }
    }
    return per;
}

/* reedsolomon.reconstruct (ReconstructData when data_only != 0, else
 * Reconstruct), called from Erasure.DecodeDataBlocks (cmd/erasure-coding.go:96)
 * and DecodeDataAndParityBlocks (:113).  shards is (k+m) x per contiguous;
 * present[i] != 0 marks shard i as present (len != 0).  Missing rows are
 * overwritten with the rebuilt shard (data rows only when data_only). */
int oracle_reconstruct(const uint8_t* matrix, int k, int m, uint8_t* shards, int64_t per,
                       const uint8_t* present, int data_only) {
    gf_init();
    int n = k + m;
    if (per <= 0) return OR_ERR_SHARD_NO_DATA;
    int np = 0, dp = 0;
    for (int i = 0; i < n; i++) if (present[i]) { np++; if (i < k) dp++; }
    if (np == 0) return OR_ERR_SHARD_NO_DATA;
    if (np == n || (data_only && dp == k)) return OR_OK;
    if (np < k) return OR_ERR_TOO_FEW_SHARDS;
    int* valid = (int*)malloc(sizeof(int) * k);
    int nv = 0;
    for (int i = 0; i < n && nv < k; i++) if (present[i]) valid[nv++] = i;
    uint8_t* sub = (uint8_t*)malloc((size_t)k * k);
    uint8_t* dec = (uint8_t*)malloc((size_t)k * k);
    for (int r = 0; r < k; r++) memcpy(sub + r * k, matrix + valid[r] * k, (size_t)k);
    int rc = oracle_gf_invert(sub, k, dec);
    if (rc) { free(valid); free(sub); free(dec); return rc; }
    for (int d = 0; d < k; d++) {
        if (present[d]) continue;
        uint8_t* out = shards + (int64_t)d * per;
        memset(out, 0, (size_t)per);
        for (int t = 0; t < k; t++) {
            uint8_t c = dec[d * k + t];
            if (!c) continue;
            const uint8_t* in = shards + (int64_t)valid[t] * per;
            for (int64_t b = 0; b < per; b++) out[b] ^= oracle_gf_mul(c, in[b]);
        }
    }
    if (!data_only) {
        for (int p = k; p < n; p++) {
            if (present[p]) continue;
            uint8_t* out = shards + (int64_t)p * per;
            memset(out, 0, (size_t)per);
            for (int j = 0; j < k; j++) {
                uint8_t c = matrix[p * k + j];
                if (!c) continue;
                const uint8_t* in = shards + (int64_t)j * per;
                for (int64_t b = 0; b < per; b++) out[b] ^= oracle_gf_mul(c, in[b]);
            }
        }
    }
    free(valid); free(sub); free(dec);
    return OR_OK;
}

/* ------------------------------------------------------------------------ */
/* HighwayHash (minio/highwayhash v1.0.2 == Google C reference).            */
typedef struct { uint64_t v0[4], v1[4], mul0[4], mul1[4]; } hh_state;

static const uint64_t HH_INIT0[4] = {0xdbe6d5d5fe4cce2fULL, 0xa4093822299f31d0ULL,
                                     0x13198a2e03707344ULL, 0x243f6a8885a308d3ULL};
static const uint64_t HH_INIT1[4] = {0x3bd39e10cb0ef593ULL, 0xc0acf169b5f18a8cULL,
                                     0xbe5466cf34e90c6cULL, 0x452821e638d01377ULL};

static uint64_t ld64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
    return v;
}

static void hh_reset(const uint8_t key[32], hh_state* s) {
    for (int i = 0; i < 4; i++) {
        uint64_t k = ld64(key + 8 * i);
        s->mul0[i] = HH_INIT0[i];
        s->mul1[i] = HH_INIT1[i];
        s->v0[i] = s->mul0[i] ^ k;
        s->v1[i] = s->mul1[i] ^ ((k >> 32) | (k << 32));
    }
}

static void zipper_merge_add(uint64_t v1, uint64_t v0, uint64_t* add1, uint64_t* add0) {
    *add0 += (((v0 & 0xff000000ULL) | (v1 & 0xff00000000ULL)) >> 24) |
             (((v0 & 0xff0000000000ULL) | (v1 & 0xff000000000000ULL)) >> 16) |
             (v0 & 0xff0000ULL) | ((v0 & 0xff00ULL) << 32) |
             ((v1 & 0xff00000000000000ULL) >> 8) | (v0 << 56);
    *add1 += (((v1 & 0xff000000ULL) | (v0 & 0xff00000000ULL)) >> 24) |
             (v1 & 0xff0000ULL) | ((v1 & 0xff0000000000ULL) >> 16) |
             ((v1 & 0xff00ULL) << 24) | ((v0 & 0xff000000000000ULL) >> 8) |
             ((v1 & 0xffULL) << 48) | (v0 & 0xff00000000000000ULL);
}

static void hh_update(const uint64_t lanes[4], hh_state* s) {
    for (int i = 0; i < 4; i++) {
        s->v1[i] += s->mul0[i] + lanes[i];
        s->mul0[i] ^= (s->v1[i] & 0xffffffffULL) * (s->v0[i] >> 32);
        s->v0[i] += s->mul1[i];
        s->mul1[i] ^= (s->v0[i] & 0xffffffffULL) * (s->v1[i] >> 32);
    }
    zipper_merge_add(s->v1[1], s->v1[0], &s->v0[1], &s->v0[0]);
    zipper_merge_add(s->v1[3], s->v1[2], &s->v0[3], &s->v0[2]);
    zipper_merge_add(s->v0[1], s->v0[0], &s->v1[1], &s->v1[0]);
    zipper_merge_add(s->v0[3], s->v0[2], &s->v1[3], &s->v1[2]);
}

static void hh_update_packet(const uint8_t* p, hh_state* s) {
    uint64_t lanes[4];
    for (int i = 0; i < 4; i++) lanes[i] = ld64(p + 8 * i);
    hh_update(lanes, s);
}

static uint32_t rotl32(uint32_t x, unsigned c) { return c ? (x << c) | (x >> (32 - c)) : x; }

static void hh_update_remainder(const uint8_t* bytes, size_t size_mod32, hh_state* s) {
    size_t size_mod4 = size_mod32 & 3;
    const uint8_t* rem = bytes + (size_mod32 & ~(size_t)3);
    uint8_t packet[32] = {0};
    for (int i = 0; i < 4; i++) {
        s->v0[i] += ((uint64_t)size_mod32 << 32) + size_mod32;
        uint32_t lo = (uint32_t)s->v1[i], hi = (uint32_t)(s->v1[i] >> 32);
        s->v1[i] = (uint64_t)rotl32(lo, (unsigned)size_mod32) |
                   ((uint64_t)rotl32(hi, (unsigned)size_mod32) << 32);
    }
    for (size_t i = 0; i < (size_t)(rem - bytes); i++) packet[i] = bytes[i];
    if (size_mod32 & 16) {
        for (int i = 0; i < 4; i++) packet[28 + i] = rem[i + size_mod4 - 4];
    } else if (size_mod4) {
        packet[16] = rem[0];
        packet[17] = rem[size_mod4 >> 1];
        packet[18] = rem[size_mod4 - 1];
    }
    hh_update_packet(packet, s);
}

static void hh_permute_update(hh_state* s) {
    uint64_t p[4];
    p[0] = (s->v0[2] >> 32) | (s->v0[2] << 32);
    p[1] = (s->v0[3] >> 32) | (s->v0[3] << 32);
    p[2] = (s->v0[0] >> 32) | (s->v0[0] << 32);
    p[3] = (s->v0[1] >> 32) | (s->v0[1] << 32);
    hh_update(p, s);
}

static void modular_reduction(uint64_t a3u, uint64_t a2, uint64_t a1, uint64_t a0,
                              uint64_t* m1, uint64_t* m0) {
    uint64_t a3 = a3u & 0x3FFFFFFFFFFFFFFFULL;
    *m1 = a1 ^ ((a3 << 1) | (a2 >> 63)) ^ ((a3 << 2) | (a2 >> 62));
    *m0 = a0 ^ (a2 << 1) ^ (a2 << 2);
}

static void hh_absorb(const uint8_t* msg, size_t len, hh_state* s) {
    size_t full = len & ~(size_t)31;
    for (size_t i = 0; i < full; i += 32) hh_update_packet(msg + i, s);
    if (len & 31) hh_update_remainder(msg + full, len & 31, s);
}

static void st64(uint8_t* p, uint64_t v) { for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i)); }

/* HighwayHash-256 digest (32 bytes, h0||h1||h2||h3 little-endian). */
void oracle_hh256(const uint8_t key[32], const uint8_t* msg, size_t len, uint8_t out[32]) {
    hh_state s;
    hh_reset(key, &s);
    hh_absorb(msg, len, &s);
    for (int i = 0; i < 10; i++) hh_permute_update(&s);
    uint64_t h[4];
    modular_reduction(s.v1[1] + s.mul1[1], s.v1[0] + s.mul1[0], s.v0[1] + s.mul0[1],
                      s.v0[0] + s.mul0[0], &h[1], &h[0]);
    modular_reduction(s.v1[3] + s.mul1[3], s.v1[2] + s.mul1[2], s.v0[3] + s.mul0[3],
                      s.v0[2] + s.mul0[2], &h[3], &h[2]);
    for (int i = 0; i < 4; i++) st64(out + 8 * i, h[i]);
}

/* HighwayHash-64 (4 finalisation rounds) — only for the public upstream vectors. */
uint64_t oracle_hh64(const uint8_t key[32], const uint8_t* msg, size_t len) {
    hh_state s;
    hh_reset(key, &s);
    hh_absorb(msg, len, &s);
    for (int i = 0; i < 4; i++) hh_permute_update(&s);
    return s.v0[0] + s.v1[0] + s.mul0[0] + s.mul1[0];
}

/* Batched HH256 over n equal-length messages at a stride (hh256 of each shard
 * chunk, cmd/bitrot-streaming.go:47-49). */
void oracle_hh256_batch(const uint8_t key[32], const uint8_t* msgs, size_t n, size_t len,
                        size_t stride, uint8_t* out) {
    for (size_t i = 0; i < n; i++) oracle_hh256(key, msgs + i * stride, len, out + 32 * i);
}

/* ------------------------------------------------------------------------ */
/* Synthetic input: counter-based splitmix64 stream (identical in
 * pyoracle.py and in the device fill kernel).  Word i of object `obj` is
 * mix(seed + obj * 2^40 + (i+1) * GAMMA); bytes are the words little-endian. */
#define SM_GAMMA 0x9e3779b97f4a7c15ULL
static uint64_t sm_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

void oracle_fill(uint64_t seed, uint64_t obj, uint8_t* out, size_t nbytes) {
    uint64_t s0 = seed + (obj << 40);
    size_t nw = nbytes / 8;
    for (size_t i = 0; i < nw; i++) st64(out + 8 * i, sm_mix(s0 + (uint64_t)(i + 1) * SM_GAMMA));
    if (nbytes & 7) {
        uint8_t tmp[8];
        st64(tmp, sm_mix(s0 + (uint64_t)(nw + 1) * SM_GAMMA));
        memcpy(out + 8 * nw, tmp, nbytes & 7);
    }
}
