// cpu_ref.cpp — CPU baseline: C++ restatement of the reference's CPU encode path.
//
// TEST / BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and tests/).  It is
// the stand-in for the Go reference, which cannot run here (no Go toolchain in the
// image; klauspost/reedsolomon v1.11.8 and minio/highwayhash v1.0.2 are not vendored).
// Label: "C++ restatement of klauspost/reedsolomon v1.11.8 + minio/highwayhash v1.0.2
// structure", never "the Go reference".
//
// Structure mirrors cmd/erasure-encode.go:83-111 per 1 MiB block, strictly sequential
// over blocks:
//   1. Split (zero pad)                           erasure-coding.go:81
//   2. Encode split by byte range over T threads  erasure-coding.go:86 (WithAutoGoroutines)
//   3. k+m HighwayHash-256 digests concurrently   erasure-encode.go:36-73 + bitrot-streaming.go:47-49
// SIMD: GF multiply via GFNI affine (AVX-512, as klauspost's GFNI kernels) when the CPU
// has avx512f+avx512bw+gfni, else AVX2 split-nibble PSHUFB (klauspost galMulAVX2);
// HighwayHash via AVX2 (as minio/highwayhash's AVX2 path).
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <functional>
#include <thread>
#include <vector>

namespace {

// ---------------- GF(2^8) tables (poly 0x11D) ----------------
struct GFT {
    uint8_t exp[512], log[256];
    GFT() {
        unsigned x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = (uint8_t)x;
            log[x] = (uint8_t)i;
            x <<= 1;
            if (x & 0x100) x ^= 0x11D;
        }
        for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
    }
    uint8_t mul(uint8_t a, uint8_t b) const { return (a && b) ? exp[log[a] + log[b]] : 0; }
};
const GFT& gft() {
    static GFT g;
    return g;
}

bool has_gfni() {
    static int v = -1;
    if (v < 0) {
        __builtin_cpu_init();
        v = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
            __builtin_cpu_supports("gfni");
    }
    return v == 1;
}

// 8x8 bit matrix for x -> c*x, in gf2p8affineqb layout: byte (7-i) of the qword
// holds row i (the bits of output bit i over input bits).
uint64_t gfni_matrix(uint8_t c) {
    const GFT& g = gft();
    uint8_t col[8];  // col[j] = c * (1 << j)
    for (int j = 0; j < 8; ++j) col[j] = g.mul(c, (uint8_t)(1u << j));
    uint64_t m = 0;
    for (int i = 0; i < 8; ++i) {
        uint8_t row = 0;
        for (int j = 0; j < 8; ++j)
            if (col[j] & (1u << i)) row |= (uint8_t)(1u << j);
        m |= (uint64_t)row << (8 * (7 - i));
    }
    return m;
}

struct Coder {
    int k, m;
    std::vector<uint8_t> coef;       // m x k parity coefficients
    std::vector<uint64_t> gfni;      // m x k affine matrices
    std::vector<uint8_t> lo, hi;     // m x k x 16 nibble tables
};

__attribute__((target("avx512f,avx512bw,gfni"))) void encode_range_gfni(const Coder& cd, uint8_t* const* in,
                                                                         uint8_t* const* out, size_t b0, size_t b1) {
    size_t b = b0;
    for (; b + 64 <= b1; b += 64) {
        __m512i acc[32];
        for (int r = 0; r < cd.m; ++r) acc[r] = _mm512_setzero_si512();
        for (int j = 0; j < cd.k; ++j) {
            const __m512i x = _mm512_loadu_si512((const void*)(in[j] + b));
            for (int r = 0; r < cd.m; ++r) {
                const __m512i A = _mm512_set1_epi64((long long)cd.gfni[r * cd.k + j]);
                acc[r] = _mm512_xor_si512(acc[r], _mm512_gf2p8affine_epi64_epi8(x, A, 0));
            }
        }
        for (int r = 0; r < cd.m; ++r) _mm512_storeu_si512((void*)(out[r] + b), acc[r]);
    }
    const GFT& g = gft();
    for (; b < b1; ++b)
        for (int r = 0; r < cd.m; ++r) {
            uint8_t a = 0;
            for (int j = 0; j < cd.k; ++j) a ^= g.mul(cd.coef[r * cd.k + j], in[j][b]);
            out[r][b] = a;
        }
}

__attribute__((target("avx2"))) void encode_range_avx2(const Coder& cd, uint8_t* const* in, uint8_t* const* out,
                                                       size_t b0, size_t b1) {
    size_t b = b0;
    const __m256i mask = _mm256_set1_epi8(0x0f);
    for (; b + 32 <= b1; b += 32) {
        __m256i acc[32];
        for (int r = 0; r < cd.m; ++r) acc[r] = _mm256_setzero_si256();
        for (int j = 0; j < cd.k; ++j) {
            const __m256i x = _mm256_loadu_si256((const __m256i*)(in[j] + b));
            const __m256i xl = _mm256_and_si256(x, mask);
            const __m256i xh = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
            for (int r = 0; r < cd.m; ++r) {
                const int ci = r * cd.k + j;
                const __m256i tl = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)&cd.lo[ci * 16]));
                const __m256i th = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)&cd.hi[ci * 16]));
                acc[r] = _mm256_xor_si256(acc[r], _mm256_xor_si256(_mm256_shuffle_epi8(tl, xl), _mm256_shuffle_epi8(th, xh)));
            }
        }
        for (int r = 0; r < cd.m; ++r) _mm256_storeu_si256((__m256i*)(out[r] + b), acc[r]);
    }
    const GFT& g = gft();
    for (; b < b1; ++b)
        for (int r = 0; r < cd.m; ++r) {
            uint8_t a = 0;
            for (int j = 0; j < cd.k; ++j) a ^= g.mul(cd.coef[r * cd.k + j], in[j][b]);
            out[r][b] = a;
        }
}

// ---------------- HighwayHash-256, AVX2 ----------------
struct HH {
    __m256i v0, v1, mul0, mul1;
};

__attribute__((target("avx2"))) inline __m256i zipper(__m256i v) {
    const __m256i msk = _mm256_setr_epi8(3, 12, 2, 5, 14, 1, 15, 0, 11, 4, 10, 13, 9, 6, 8, 7,
                                         3, 12, 2, 5, 14, 1, 15, 0, 11, 4, 10, 13, 9, 6, 8, 7);
    return _mm256_shuffle_epi8(v, msk);
}

__attribute__((target("avx2"))) inline void hh_update(HH& s, __m256i p) {
    s.v1 = _mm256_add_epi64(s.v1, _mm256_add_epi64(s.mul0, p));
    s.mul0 = _mm256_xor_si256(s.mul0, _mm256_mul_epu32(s.v1, _mm256_srli_epi64(s.v0, 32)));
    s.v0 = _mm256_add_epi64(s.v0, s.mul1);
    s.mul1 = _mm256_xor_si256(s.mul1, _mm256_mul_epu32(s.v0, _mm256_srli_epi64(s.v1, 32)));
    s.v0 = _mm256_add_epi64(s.v0, zipper(s.v1));
    s.v1 = _mm256_add_epi64(s.v1, zipper(s.v0));
}

__attribute__((target("avx2"))) void hh256_avx2(const uint8_t key[32], const uint8_t* msg, size_t len,
                                                uint8_t out[32]) {
    const __m256i init0 = _mm256_setr_epi64x((long long)0xdbe6d5d5fe4cce2fULL, (long long)0xa4093822299f31d0ULL,
                                             (long long)0x13198a2e03707344ULL, (long long)0x243f6a8885a308d3ULL);
    const __m256i init1 = _mm256_setr_epi64x((long long)0x3bd39e10cb0ef593ULL, (long long)0xc0acf169b5f18a8cULL,
                                             (long long)0xbe5466cf34e90c6cULL, (long long)0x452821e638d01377ULL);
    const __m256i k = _mm256_loadu_si256((const __m256i*)key);
    HH s;
    s.mul0 = init0;
    s.mul1 = init1;
    s.v0 = _mm256_xor_si256(init0, k);
    s.v1 = _mm256_xor_si256(init1, _mm256_shuffle_epi32(k, 0xB1));
    size_t full = len & ~(size_t)31;
    for (size_t i = 0; i < full; i += 32) hh_update(s, _mm256_loadu_si256((const __m256i*)(msg + i)));
    const size_t n = len & 31;
    if (n) {
        s.v0 = _mm256_add_epi64(s.v0, _mm256_set1_epi64x((long long)(((uint64_t)n << 32) + n)));
        s.v1 = _mm256_or_si256(_mm256_slli_epi32(s.v1, (int)n), _mm256_srli_epi32(s.v1, (int)(32 - n)));
        const uint8_t* tail = msg + full;
        alignas(32) uint8_t pkt[32] = {0};
        const size_t remain = n & ~(size_t)3, mod4 = n & 3;
        memcpy(pkt, tail, remain);
        if (n & 16) {
            memcpy(pkt + 28, tail + n - 4, 4);
        } else if (mod4) {
            pkt[16] = tail[remain];
            pkt[17] = tail[remain + (mod4 >> 1)];
            pkt[18] = tail[n - 1];
        }
        hh_update(s, _mm256_load_si256((const __m256i*)pkt));
    }
    for (int r = 0; r < 10; ++r) {
        const __m256i p = _mm256_shuffle_epi32(_mm256_permute4x64_epi64(s.v0, 0x4E), 0xB1);
        hh_update(s, p);
    }
    alignas(32) uint64_t v0[4], v1[4], m0[4], m1[4];
    _mm256_store_si256((__m256i*)v0, s.v0);
    _mm256_store_si256((__m256i*)v1, s.v1);
    _mm256_store_si256((__m256i*)m0, s.mul0);
    _mm256_store_si256((__m256i*)m1, s.mul1);
    uint64_t h[4];
    for (int p = 0; p < 2; ++p) {
        const uint64_t a3 = (v1[2 * p + 1] + m1[2 * p + 1]) & 0x3FFFFFFFFFFFFFFFULL;
        const uint64_t a2 = v1[2 * p] + m1[2 * p];
        const uint64_t a1 = v0[2 * p + 1] + m0[2 * p + 1];
        const uint64_t a0 = v0[2 * p] + m0[2 * p];
        h[2 * p + 1] = a1 ^ ((a3 << 1) | (a2 >> 63)) ^ ((a3 << 2) | (a2 >> 62));
        h[2 * p] = a0 ^ (a2 << 1) ^ (a2 << 2);
    }
    memcpy(out, h, 32);
}

// ---------------- tiny fork-join pool ----------------
class Pool {
public:
    explicit Pool(int n) : n_(n < 1 ? 1 : n) {
        for (int i = 1; i < n_; ++i) th_.emplace_back([this, i] { loop(i); });
    }
    ~Pool() {
        stop_.store(true);
        gen_.fetch_add(1);
        for (auto& t : th_) t.join();
    }
    int size() const { return n_; }
    // run f(i) for i in [0, n_) and wait
    void run(const std::function<void(int)>& f) {
        job_ = &f;
        done_.store(0);
        gen_.fetch_add(1, std::memory_order_release);
        f(0);
        for (unsigned spins = 0; done_.load(std::memory_order_acquire) != n_ - 1; ++spins) backoff(spins);
    }

private:
    static void backoff(unsigned spins) {
        if (spins < 2048)
            _mm_pause();
        else
            std::this_thread::yield();
    }
    void loop(int i) {
        uint64_t seen = 0;
        for (;;) {
            uint64_t g;
            for (unsigned spins = 0; (g = gen_.load(std::memory_order_acquire)) == seen; ++spins) backoff(spins);
            seen = g;
            if (stop_.load()) return;
            (*job_)(i);
            done_.fetch_add(1, std::memory_order_acq_rel);
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> done_{0};
    std::atomic<bool> stop_{false};
    const std::function<void(int)>* job_ = nullptr;
};

}  // namespace

extern "C" {

const char* cpuref_isa(void) { return has_gfni() ? "avx512+gfni" : "avx2"; }

// Encode + hash n_blocks blocks (block b at data + b*data_stride, block_len bytes),
// the reference way: blocks sequential, encode split by byte range over `threads`,
// then the k+m digests spread over the threads.  Parity row r of block b at
// parity + b*parity_stride + r*S; sums (may be NULL) at sums + (b*(k+m)+i)*32.
// matrix is the (k+m) x k coding matrix.  Returns S.
int64_t cpuref_encode_hash(int k, int m, const uint8_t* matrix, const uint8_t* data, int64_t block_len,
                           int64_t n_blocks, int64_t data_stride, uint8_t* parity, int64_t parity_stride,
                           uint8_t* sums, const uint8_t* key, int threads) {
    if (k <= 0 || m <= 0 || k + m > 256 || block_len <= 0 || m > 32) return -1;
    const int64_t S = (block_len + k - 1) / k;
    Coder cd;
    cd.k = k;
    cd.m = m;
    cd.coef.resize((size_t)m * k);
    cd.gfni.resize((size_t)m * k);
    cd.lo.resize((size_t)m * k * 16);
    cd.hi.resize((size_t)m * k * 16);
    const GFT& g = gft();
    for (int r = 0; r < m; ++r)
        for (int j = 0; j < k; ++j) {
            const uint8_t c = matrix[(size_t)(k + r) * k + j];
            const int ci = r * k + j;
            cd.coef[ci] = c;
            cd.gfni[ci] = gfni_matrix(c);
            for (int x = 0; x < 16; ++x) {
                cd.lo[ci * 16 + x] = g.mul(c, (uint8_t)x);
                cd.hi[ci * 16 + x] = g.mul(c, (uint8_t)(x << 4));
            }
        }
    const bool gfni = has_gfni();
    Pool pool(threads);
    const int T = pool.size();
    std::vector<uint8_t> pad((size_t)k * S);  // Split's zero-padded data rows
    std::vector<uint8_t*> in(k), out(m);
    for (int64_t b = 0; b < n_blocks; ++b) {
        const uint8_t* blk = data + b * data_stride;
        uint8_t* pb = parity + b * parity_stride;
        const uint8_t* rows;
        if (block_len == k * S) {
            rows = blk;  // in-place Split, no padding needed
        } else {
            memcpy(pad.data(), blk, (size_t)block_len);
            memset(pad.data() + block_len, 0, (size_t)(k * S - block_len));
            rows = pad.data();
        }
        for (int j = 0; j < k; ++j) in[j] = const_cast<uint8_t*>(rows) + (size_t)j * S;
        for (int r = 0; r < m; ++r) out[r] = pb + (size_t)r * S;
        // Encode split by byte range (64-byte aligned chunks)
        pool.run([&](int t) {
            const int64_t per = ((S + T - 1) / T + 63) & ~(int64_t)63;
            const int64_t b0 = t * per, b1 = (b0 + per) < S ? (b0 + per) : S;
            if (b0 >= b1) return;
            if (gfni)
                encode_range_gfni(cd, in.data(), out.data(), (size_t)b0, (size_t)b1);
            else
                encode_range_avx2(cd, in.data(), out.data(), (size_t)b0, (size_t)b1);
        });
        if (sums) {
            uint8_t* sb = sums + b * (int64_t)(k + m) * 32;
            pool.run([&](int t) {
                for (int i = t; i < k + m; i += T) {
                    const uint8_t* msg = i < k ? in[i] : out[i - k];
                    hh256_avx2(key, msg, (size_t)S, sb + (size_t)i * 32);
                }
            });
        }
    }
    return S;
}

void cpuref_hh256(const uint8_t* key, const uint8_t* msg, int64_t len, uint8_t* out) {
    hh256_avx2(key, msg, (size_t)len, out);
}

}  // extern "C"
