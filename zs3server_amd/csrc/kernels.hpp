// kernels.hpp — launch interface between the C-ABI layer (zs3gpu.hip) and the
// HIP kernels (kernels.hip).  Internal; not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zs3k {

// Batched Split+Encode(+HH256) over n_blocks independent blocks.
// Block b: data bytes at data + b*data_stride, length n (<= k*S; bytes beyond n are
// implicit zero padding, as reedsolomon.Split), parity row r at
// parity + b*parity_stride + r*S, sums (optional) at sums + (b*(k+m) + i)*32.
struct EncArgs {
    const uint8_t* data;
    int64_t data_stride;
    uint8_t* parity;
    int64_t parity_stride;
    uint8_t* sums;            // nullptr: encode only
    const uint32_t* tables;   // perm tables, 8 dwords per coefficient (r*k + j)
    const uint8_t* matrix;    // (k+m) x k coding matrix (generic path)
    int64_t S;                // shard size
    int64_t n;                // block length
    int64_t n_blocks;
    uint64_t key[4];          // HighwayHash key words (little-endian)
    int k, m;
    uint64_t* dbg;            // diagnostics build only: per-wave phase cycle sums
    int dyb;                  // 0, or 2/4: parity block is dyadic in dyb x dyb blocks
    const uint32_t* dtables;  // dyadic Karatsuba tables (3 or 9 coefficients per block)
};

// Reconstruct: out rows = coef x valid rows, per block.  Block b shard i at
// shards + b*block_stride + i*S.
struct RecArgs {
    uint8_t* shards;
    int64_t block_stride;
    int64_t S;
    int64_t n_blocks;
    const uint32_t* tables;   // perm tables, 8 dwords per (e*k + t)
    const uint8_t* coef;      // e x k coefficients (generic path)
    const int32_t* rows;      // k valid row indices then e output row indices
    int k, e;
};

// HighwayHash-256 of n equal-length messages (bitrot verify / reader path).
struct HashArgs {
    const uint8_t* msgs;
    int64_t stride;
    int64_t len;
    int64_t n;
    uint8_t* sums;            // n x 32 (at sum_stride bytes per message)
    const uint8_t* expect;    // optional n x 32 (at sum_stride); mismatch flags -> bad
    int32_t* bad;             // optional n flags at bad_stride (1 = errFileCorrupt)
    uint64_t key[4];
    int64_t sum_stride;       // 0 = 32
    int64_t bad_stride;       // 0 = 1
};

// GET / heal pass: verify the k survivor shards the decode reads
// against their stored bitrot sums and rebuild the missing shards in one pass.
struct VrArgs {
    uint8_t* shards;          // [n][k+m][S] at block_stride
    int64_t block_stride;
    int64_t S;
    int64_t n_blocks;
    const uint32_t* tables;   // perm tables, 8 dwords per (e*k + t); may be null if e == 0
    const uint8_t* coef;      // e x k coefficients (fallback path)
    const int32_t* rows;      // k survivor row indices then e rebuilt row indices
    int k, m, e;
    const uint8_t* expect;    // [n][k+m][32] stored sums; survivors are compared
    int32_t* bad;             // [n][k+m]: 1 = survivor failed bitrot (errFileCorrupt)
    uint8_t* sums_out;        // optional [n][k+m][32]: HH256 of the rebuilt rows
    uint64_t key[4];
};

// Batched MD5 / SHA-256 (digest.hip): message i of lens[i] (or len) bytes at
// msgs + i*stride; digest i at out + i*16 (MD5) or out + i*32 (SHA-256).
struct DigestArgs {
    const uint8_t* msgs;
    int64_t stride;
    int64_t len;
    const int64_t* lens;      // optional per-message lengths (device)
    int64_t n;
    uint8_t* out;
};

// Returns hipSuccess or an error from the launch.
hipError_t launch_encode(const EncArgs& a, hipStream_t s, bool* used_fast);
hipError_t launch_reconstruct(const RecArgs& a, hipStream_t s, bool* used_fast);
hipError_t launch_verify_reconstruct(const VrArgs& a, hipStream_t s, bool* used_fast);
hipError_t launch_hash(const HashArgs& a, hipStream_t s);
hipError_t launch_md5(const DigestArgs& a, hipStream_t s);
hipError_t launch_sha256(const DigestArgs& a, hipStream_t s);
hipError_t launch_fill(uint8_t* out, int64_t stride, int64_t len, int64_t n, uint64_t seed,
                       uint64_t obj0, hipStream_t s);

// Number of (k, m) pairs with a specialised fused kernel, and whether (k, m) has one.
bool has_fast_encode(int k, int m);

// Second-generation fused encode+hash kernel (fused_v2.hip), variant numbers 50+.
// Returns false when the variant does not apply to a.k/a.m (caller falls back).
bool launch_ehx(int v, const EncArgs& a, hipStream_t s);
// Warp-specialised GET / heal pass (fused_v2.hip); false if the shape has no instance.
bool launch_vr_ws(int v, const VrArgs& a, hipStream_t s);

// Tuning knob for experiments: 0 = default variant.
void set_variant(int v);
int get_variant();

}  // namespace zs3k
