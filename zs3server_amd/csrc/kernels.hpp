// kernels.hpp — launch interface between the C-ABI layer (zs3gpu.hip) and the
// HIP kernels (kernels.hip, fused_v2.hip, digest.hip).  Internal; not part of the
// public ABI.
//
// There is no process-wide tuning state: every launch carries its own `variant`
// (0 = the tuned default).  Non-zero variants exist only in the diagnostics build
// (ZS3_DIAG, libzs3gpu_diag.so); the product library compiles the defaults and the
// generic fallbacks only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef ZS3_DIAG
#define ZS3_DIAG 0
#endif

namespace zs3k {

// Which kernel family served a launch (zs3_last_path; include/zs3gpu.h ZS3_PATH_*).
enum Path : int {
    PATH_NONE = -1,
    PATH_GENERIC = 0,   // byte kernels with log/exp tables (any k, m, S)
    PATH_FIRSTGEN = 1,  // first-generation specialised kernels (kernels.hip)
    PATH_WS = 2,        // warp-specialised kernels (fused_v2.hip k_ehx_ws / k_vr_ws)
    PATH_PIPE = 3,      // mixed-wave second-generation encode (fused_v2.hip k_ehx)
    PATH_LATENCY = 4,   // small batches: k_encode_only + k_hash_lat (kernels.hip)
};

// Kernel instances a launch can name beyond its family (zs3_path_mask): bits set on the
// launching thread, read (and cleared with `reset`) by kernel_bits.
enum KernelBit : uint32_t {
    KERNEL_VR_QUAD = 1u << 16,  // k_vr_quad (vr_quad.hpp) served a GET / heal batch
};
void note_kernel(uint32_t bit);
uint32_t kernel_bits(bool reset);

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
    uint64_t* dbg;            // diagnostics build only: per-wave stamps (nullptr in the product)
    int dyb;                  // 0, or 2/4: parity block is dyadic in dyb x dyb blocks
    const uint32_t* dtables;  // dyadic local-ring tables (m coefficients per block)
    int variant;              // 0 = tuned default (the only value the product build accepts)
};

// Reconstruct: out rows = coef x valid rows, per block.  Block b shard i at
// shards + slot(b)*block_stride + i*S, slot(b) = ids ? ids[b] : b.
struct RecArgs {
    uint8_t* shards;
    int64_t block_stride;
    int64_t S;
    int64_t n_blocks;
    const uint32_t* tables;   // perm tables, 8 dwords per (e*k + t)
    const uint8_t* coef;      // e x k coefficients (generic path)
    const int32_t* rows;      // k valid row indices then e output row indices
    int k, e;
    const int32_t* ids;       // optional device block-slot list (per-block erasure patterns)
    int variant;
};

// HighwayHash-256 of n messages (bitrot writer sums / reader verify / deep scan).
// Message i: slot s = ids ? ids[i] : i.  Uniform mode: bytes at msgs + s*stride,
// length len.  Ragged mode (lens != nullptr): length lens[i]; ptrs != nullptr gives
// each message's address directly.  Chunked-file mode (chunk > 0): message i is chunk
// c = i % nchunks of file f = i / nchunks in the on-disk HighwayHash256S layout
// [32-byte sum][chunk]* (cmd/bitrot-streaming.go:43-65): bytes at
// msgs + f*stride + c*(chunk+32) + 32, expected sum 32 bytes before them, length
// chunk except the last chunk (last_len).
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
    const int32_t* ids;       // optional slot list
    const int64_t* lens;      // ragged lengths (device), or nullptr
    const uint8_t* const* ptrs;  // ragged message addresses (device), or nullptr
    int64_t chunk;            // chunked-file mode: shard size (0 = off)
    int64_t nchunks;          // chunks per file
    int64_t last_len;         // length of each file's last chunk
    int variant;              // diagnostics build only (0 = tuned default)
    // stripe mode (rps > 0): message i = shard rowmap[i % rps] of stripe i / rps (slot
    // ids[stripe] if ids); shard idx < kd at msgs + slot*stride + idx*len, else at
    // par + slot*par_stride + (idx-kd)*len; sums / expect / bad at slot*rtot + idx;
    // bytes of data shard idx at or past vlim - idx*len read as zero (Split padding)
    int rps;
    int kd;
    int rtot;
    int64_t vlim;             // valid bytes of the stripe's data (EncodeData's len); 0 = all
    const uint8_t* par;
    int64_t par_stride;
    uint8_t rowmap[64];
};

// GET / heal pass: verify the k survivor shards the decode reads
// against their stored bitrot sums and rebuild the missing shards in one pass.
// Block b lives in slot(b) = ids ? ids[b] : b of every array.
struct VrArgs {
    uint8_t* shards;          // [slots][k+m][S] at block_stride
    int64_t block_stride;
    int64_t S;
    int64_t n_blocks;
    const uint32_t* tables;   // perm tables, 8 dwords per (e*k + t); may be null if e == 0
    const uint8_t* coef;      // e x k coefficients (fallback path)
    const int32_t* rows;      // k survivor row indices then e rebuilt row indices
    int k, m, e;
    const uint8_t* expect;    // [slots][k+m][32] stored sums; survivors are compared
    int32_t* bad;             // [slots][k+m]: 1 = survivor failed bitrot (errFileCorrupt)
    uint8_t* sums_out;        // optional [slots][k+m][32]: HH256 of the rebuilt rows
    uint64_t key[4];
    const int32_t* ids;       // optional device block-slot list
    int variant;
    const int32_t* h_rows;    // host copy of `rows` (k survivors, then e rebuilt rows)
    uint64_t* dbg;            // diagnostics build only: per-wave stamps (nullptr in the product)
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
    const int64_t* offs;      // optional per-message byte offsets from msgs (device; else i*stride)
    int variant;              // diagnostics: 1 = the one-wave kernels (round 3)
};

// Launches return hipSuccess or the launch error; *path (may be null) receives the
// kernel family that ran.
hipError_t launch_encode(const EncArgs& a, hipStream_t s, int* path);
hipError_t launch_reconstruct(const RecArgs& a, hipStream_t s, int* path);
hipError_t launch_verify_reconstruct(const VrArgs& a, hipStream_t s, int* path);
hipError_t launch_hash(const HashArgs& a, hipStream_t s);
hipError_t launch_md5(const DigestArgs& a, hipStream_t s);
hipError_t launch_sha256(const DigestArgs& a, hipStream_t s);
// k_rows_copy: rows rs.row[0..n) of nb stripes (stride E, rows of S bytes), src -> dst at
// the same offsets (bases congruent mod 16; n <= 32).
struct RowSet {
    int n;
    int row[32];
};
hipError_t launch_rows_copy(const uint8_t* src, uint8_t* dst, int64_t E, int64_t S, int64_t nb, const RowSet& rs,
                            hipStream_t s);
hipError_t launch_fill(uint8_t* out, int64_t stride, int64_t len, int64_t n, uint64_t seed,
                       uint64_t obj0, hipStream_t s);
// out[r] = 1 if any of flags[r*cols .. r*cols+cols) is non-zero, else 0.
hipError_t launch_any_rows(const int32_t* flags, int64_t rows, int64_t cols, int32_t* out, hipStream_t s);

// Whether (k, m) has a specialised fused kernel.
bool has_fast_encode(int k, int m);

// Second-generation fused encode+hash kernels (fused_v2.hip).  `v` is a variant
// number; the product build knows only the defaults it dispatches to.  Returns the
// path that ran, or PATH_NONE when the variant does not apply (caller falls back).
int launch_ehx(int v, const EncArgs& a, hipStream_t s);
// Fused encode + sums for shard sizes that are not a multiple of 16 (k_ehx_ws UA mode,
// e.g. RS(12+4) on 1 MiB blocks); PATH_NONE when the shape has no such instance.
int launch_ehx_ua(const EncArgs& a, hipStream_t s);
// The same kernel for the server's non-dyadic default geometries (fused_v2_gen.hip: a
// general M x K matrix in the encode role); PATH_NONE when (k, m) has no instance or the
// layout does not fit.
int launch_ehx_gen(const EncArgs& a, hipStream_t s);
bool has_gen_encode(int k, int m);
// Warp-specialised GET / heal for the same geometries (fused_v2_get_gen.hip); false when
// (k, e) has no instance or the layout does not fit.
bool launch_vr_ws_gen(const VrArgs& a, hipStream_t s);
// Warp-specialised GET / heal pass (fused_v2.hip); false if the shape has no instance.
bool launch_vr_ws(int v, const VrArgs& a, hipStream_t s);

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device, size),
// thread-safe.
hipError_t ensure_dyn_lds(const void* kern, size_t bytes);

}  // namespace zs3k
