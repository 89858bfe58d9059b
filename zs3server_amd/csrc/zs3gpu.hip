// zs3gpu.hip — C-ABI layer (include/zs3gpu.h) over the gfx950 kernels.
//
// Host-side counterpart of the reference's Erasure value (cmd/erasure-coding.go)
// and bitrot hash factory (cmd/bitrot.go): codec construction with NewErasure's
// checks, size arithmetic, decode-matrix inversion cached per erasure pattern (as
// klauspost's inversion tree does), per-thread pinned staging for host-pointer
// calls, and the startup self-tests.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zs3gpu.h"
#if ZS3_DIAG
#include "../../include/zs3gpu_diag.h"
#endif
#include "codec_host.hpp"
#include "kernels.hpp"

namespace {

constexpr int kMajor = 0, kMinor = 1, kPatch = 0;

// cmd/bitrot.go:37 — HH-256 of the first 100 decimals of pi under a zero key.
const uint8_t kMagicKey[32] = {0x4b, 0xe7, 0x34, 0xfa, 0x8e, 0x23, 0x8a, 0xcd, 0x26, 0x3e, 0x83,
                               0xe6, 0xbb, 0x96, 0x85, 0x52, 0x04, 0x0f, 0x93, 0x5d, 0xa3, 0x9f,
                               0x44, 0x14, 0x97, 0xe0, 0x9d, 0x13, 0x22, 0xde, 0x36, 0xa0};

thread_local int t_last_path = -1;
thread_local uint32_t t_path_mask = 0;  // zs3_path_mask

void note_path(int p) {
    t_last_path = p;
    if (p >= 0) t_path_mask |= 1u << p;
}
#if ZS3_DIAG
// Diagnostics build only (libzs3gpu_diag.so): per-OS-thread experiment selection, so
// concurrent callers never see each other's settings.
thread_local int t_variant = 0;          // fused-kernel variant (0 = tuned default)
thread_local uint64_t* t_dbg = nullptr;  // stamped-variant output buffer
thread_local int t_no_dyadic = 0;        // force the plain (m*k multiply) encode
inline int call_variant() { return t_variant; }
#else
inline int call_variant() { return 0; }
#endif

void key_words(const uint8_t* key, uint64_t out[4]) {
    const uint8_t* k = key ? key : kMagicKey;
    for (int i = 0; i < 4; ++i) {
        uint64_t v = 0;
        for (int b = 7; b >= 0; --b) v = (v << 8) | k[8 * i + b];
        out[i] = v;
    }
}

int64_t ceil_frac(int64_t num, int64_t den) {  // cmd/utils.go:691
    if (den == 0) return 0;
    if (den < 0) {
        num = -num;
        den = -den;
    }
    int64_t c = num / den;
    if (num > 0 && num % den != 0) ++c;
    return c;
}

int current_device() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) return -1;
    return d;
}

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// Cached reconstruct plan for one erasure pattern (host part: codec_host.hpp).
struct RecPlan : zs3::PlanData {
    std::map<int, std::shared_ptr<DevBuf>> dev;  // device -> [tables | coef | rows]
};

}  // namespace

struct zs3_codec : zs3::CodecTables {
    int k, m;
    int64_t block_size;
    std::mutex mu;
    std::map<int, std::shared_ptr<DevBuf>> dev;  // device -> [tables | matrix]
    std::map<std::string, std::shared_ptr<RecPlan>> plans;
};

namespace {

int map_hip(hipError_t e) { return e == hipSuccess ? ZS3_OK : (e == hipErrorOutOfMemory ? ZS3_ERR_NOMEM : ZS3_ERR_DEVICE); }

// Device copy of the codec's tables + matrix on the current device.
int codec_device(zs3_codec* c, const uint32_t** tabs, const uint8_t** mat) {
    const int d = current_device();
    if (d < 0) return ZS3_ERR_DEVICE;
    std::lock_guard<std::mutex> g(c->mu);
    auto it = c->dev.find(d);
    if (it == c->dev.end()) {
        auto b = std::make_shared<DevBuf>();
        const size_t tb = c->tables.size() * 4, mb = c->matrix.size();
        if (hipMalloc(&b->p, tb + mb) != hipSuccess) return ZS3_ERR_NOMEM;
        if (hipMemcpy(b->p, c->tables.data(), tb, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy((uint8_t*)b->p + tb, c->matrix.data(), mb, hipMemcpyHostToDevice) != hipSuccess)
            return ZS3_ERR_DEVICE;
        it = c->dev.emplace(d, b).first;
    }
    *tabs = (const uint32_t*)it->second->p;
    *mat = (const uint8_t*)it->second->p + c->tables.size() * 4;
    return ZS3_OK;
}

// reedsolomon reconstruct() argument checks + inversion for one pattern.
std::shared_ptr<RecPlan> make_plan(const zs3_codec* c, const uint8_t* present, int data_only) {
    auto p = std::make_shared<RecPlan>();
    zs3::make_plan_data(c->k, c->m, c->matrix.data(), present, data_only, *p);
    return p;
}

std::shared_ptr<RecPlan> get_plan(zs3_codec* c, const uint8_t* present, int data_only) {
    std::string key((const char*)present, c->k + c->m);
    for (auto& ch : key) ch = ch ? 1 : 0;
    key.push_back(data_only ? 1 : 0);
    std::lock_guard<std::mutex> g(c->mu);
    auto it = c->plans.find(key);
    if (it != c->plans.end()) return it->second;
    auto p = make_plan(c, (const uint8_t*)key.data(), data_only);
    c->plans.emplace(key, p);
    return p;
}

int plan_device(zs3_codec* c, RecPlan* p, const uint32_t** tabs, const uint8_t** coef, const int32_t** rows) {
    const int d = current_device();
    if (d < 0) return ZS3_ERR_DEVICE;
    std::lock_guard<std::mutex> g(c->mu);
    auto it = p->dev.find(d);
    const size_t tb = p->tables.size() * 4, cb = (p->coef.size() + 15) & ~(size_t)15, rb = p->rows.size() * 4;
    if (it == p->dev.end()) {
        auto b = std::make_shared<DevBuf>();
        if (hipMalloc(&b->p, tb + cb + rb) != hipSuccess) return ZS3_ERR_NOMEM;
        uint8_t* base = (uint8_t*)b->p;
        if (hipMemcpy(base, p->tables.data(), tb, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(base + tb, p->coef.data(), p->coef.size(), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(base + tb + cb, p->rows.data(), rb, hipMemcpyHostToDevice) != hipSuccess)
            return ZS3_ERR_DEVICE;
        it = p->dev.emplace(d, b).first;
    }
    uint8_t* base = (uint8_t*)it->second->p;
    *tabs = (const uint32_t*)base;
    *coef = base + tb;
    *rows = (const int32_t*)(base + tb + cb);
    return ZS3_OK;
}

// Block-id lists of the per-block-pattern calls (zs3_*_batch_masks): every group's ids
// go into ONE pinned staging slot per call, then one stream-ordered copy into a
// hipMallocAsync'd device buffer that is freed (hipFreeAsync) behind the kernels that
// read it.  Each OS thread keeps a small ring of slots per device, so a call waits
// only for the copy out of the slot it reuses (kIdsSlots calls back), never for its
// own or the previous call's copy queued behind a large H2D on the same stream.
constexpr int kIdsSlots = 4;
struct IdsStage {
    int32_t* h[kIdsSlots] = {};
    size_t cap[kIdsSlots] = {};
    hipEvent_t ev[kIdsSlots] = {};  // last copy out of h[i]
    bool used[kIdsSlots] = {};
    int next = 0;
    ~IdsStage() {
        for (int i = 0; i < kIdsSlots; ++i) {
            if (ev[i]) (void)hipEventDestroy(ev[i]);
            if (h[i]) (void)hipHostFree(h[i]);
        }
    }
};
thread_local std::map<int, std::unique_ptr<IdsStage>> t_ids;

// Blocks of a batch grouped by erasure pattern (zs3_*_batch_masks).
struct PatternGroup {
    std::shared_ptr<RecPlan> plan;
    std::vector<int32_t> blocks;
    size_t ids_off = 0;  // offset of this group's ids in the call's device id list
    // first block when the group's blocks are one ascending run b0, b0+1, ... (-1 if not):
    // such a group launches on the shifted batch without an id list, so it takes the same
    // instances as a single-pattern call (the buffer-addressed ones need no id list)
    int64_t run0 = -1;
};

void mark_runs(std::vector<PatternGroup>& groups) {
    for (auto& g : groups) {
        g.run0 = -1;
        if (g.blocks.empty()) continue;
        bool run = true;
        for (size_t i = 1; i < g.blocks.size() && run; ++i) run = g.blocks[i] == g.blocks[0] + (int32_t)i;
        if (run) g.run0 = g.blocks[0];
    }
}

// One upload of every launched group's block ids (see IdsStage).
int upload_group_ids(std::vector<PatternGroup>& groups, bool skip_noop, hipStream_t s, int32_t** d_out) {
    *d_out = nullptr;
    size_t n = 0;
    mark_runs(groups);
    for (auto& g : groups) {
        g.ids_off = n;
        if (!g.blocks.empty() && !(skip_noop && g.plan->noop) && g.run0 < 0) n += g.blocks.size();
    }
    if (n == 0) return ZS3_OK;
    const int d = current_device();
    if (d < 0) return ZS3_ERR_DEVICE;
    auto& sp = t_ids[d];
    if (!sp) sp.reset(new IdsStage());
    const int i = sp->next;
    sp->next = (i + 1) % kIdsSlots;
    if (!sp->ev[i] && hipEventCreateWithFlags(&sp->ev[i], hipEventDisableTiming) != hipSuccess) return ZS3_ERR_DEVICE;
    if (sp->used[i] && hipEventSynchronize(sp->ev[i]) != hipSuccess) return ZS3_ERR_DEVICE;
    const size_t bytes = n * sizeof(int32_t);
    if (sp->cap[i] < bytes) {
        if (sp->h[i]) (void)hipHostFree(sp->h[i]);
        sp->h[i] = nullptr;
        sp->cap[i] = 0;
        if (hipHostMalloc((void**)&sp->h[i], bytes, hipHostMallocDefault) != hipSuccess) return ZS3_ERR_NOMEM;
        sp->cap[i] = bytes;
    }
    for (auto& g : groups)
        if (!g.blocks.empty() && !(skip_noop && g.plan->noop) && g.run0 < 0)
            std::memcpy(sp->h[i] + g.ids_off, g.blocks.data(), g.blocks.size() * sizeof(int32_t));
    if (hipMallocAsync((void**)d_out, bytes, s) != hipSuccess) return ZS3_ERR_NOMEM;
    if (hipMemcpyAsync(*d_out, sp->h[i], bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipEventRecord(sp->ev[i], s) != hipSuccess)
        return ZS3_ERR_DEVICE;
    sp->used[i] = true;
    return ZS3_OK;
}

int group_patterns(zs3_codec* c, const uint8_t* present, int64_t n, int data_only, int32_t* status,
                   std::vector<PatternGroup>& groups) {
    const int R = c->k + c->m;
    std::map<std::string, size_t> idx;
    int first = ZS3_OK;
    std::string key((size_t)R, '\0');
    for (int64_t b = 0; b < n; ++b) {
        const uint8_t* row = present + b * R;
        for (int i = 0; i < R; ++i) key[(size_t)i] = row[i] ? 1 : 0;
        auto it = idx.find(key);
        if (it == idx.end()) {
            PatternGroup g;
            g.plan = get_plan(c, (const uint8_t*)key.data(), data_only);
            it = idx.emplace(key, groups.size()).first;
            groups.push_back(std::move(g));
        }
        PatternGroup& g = groups[it->second];
        if (status) status[b] = g.plan->status;
        if (g.plan->status) {
            if (first == ZS3_OK) first = g.plan->status;
            continue;
        }
        g.blocks.push_back((int32_t)b);
    }
    return first;
}

// Per-OS-thread staging for host-pointer calls.
struct Staging {
    int dev = -1;
    hipStream_t stream = nullptr;
    uint8_t* d = nullptr;
    size_t dcap = 0;
    uint8_t* h = nullptr;
    size_t hcap = 0;
    ~Staging() {
        if (d) (void)hipFree(d);
        if (h) (void)hipHostFree(h);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

thread_local std::map<int, std::unique_ptr<Staging>> t_staging;

Staging* staging(size_t dbytes, size_t hbytes) {
    const int d = current_device();
    if (d < 0) return nullptr;
    auto& sp = t_staging[d];
    if (!sp) {
        sp.reset(new Staging());
        sp->dev = d;
        if (hipStreamCreateWithFlags(&sp->stream, hipStreamNonBlocking) != hipSuccess) return nullptr;
    }
    Staging* s = sp.get();
    if (s->dcap < dbytes) {
        if (s->d) (void)hipFree(s->d);
        s->d = nullptr;
        s->dcap = 0;
        if (hipMalloc(&s->d, dbytes) != hipSuccess) return nullptr;
        s->dcap = dbytes;
    }
    if (s->hcap < hbytes) {
        if (s->h) (void)hipHostFree(s->h);
        s->h = nullptr;
        s->hcap = 0;
        if (hipHostMalloc(&s->h, hbytes, hipHostMallocDefault) != hipSuccess) return nullptr;
        s->hcap = hbytes;
    }
    return s;
}

size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// Live zs3_host_alloc ranges (base -> bytes): the queue DMAs straight from / to a
// caller buffer that lies in one of them (the pinned bpool, internal/bpool/bpool.go:29)
struct PinnedRange {
    size_t bytes;
    uintptr_t dev;  // the allocation's device-side address (hipHostGetDevicePointer)
};
std::mutex g_pin_mu;
std::map<uintptr_t, PinnedRange> g_pinned;

}  // namespace

// [p, p+n) inside one live zs3_host_alloc allocation (queue.hip's zero-copy test); *dev
// (optional) receives the address a kernel uses for p (the mapped pinned pages)
__attribute__((visibility("hidden"))) bool zs3i_pinned_map(const void* p, size_t n, void** dev) {
    if (!p) return false;
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> g(g_pin_mu);
    auto it = g_pinned.upper_bound(a);
    if (it == g_pinned.begin()) return false;
    --it;
    const size_t sz = it->second.bytes;
    if (!(a >= it->first && a - it->first <= sz && n <= sz - (a - it->first))) return false;
    if (dev) *dev = (void*)(it->second.dev + (a - it->first));
    return true;
}
__attribute__((visibility("hidden"))) bool zs3i_pinned(const void* p, size_t n) { return zs3i_pinned_map(p, n, nullptr); }

extern "C" {

const char* zs3_strerror(int code) {
    switch (code) {
        case ZS3_OK: return "ok";
        case ZS3_ERR_INV_SHARD_NUM: return "cannot create Encoder with less than one data shard or less than zero parity shards";
        case ZS3_ERR_MAX_SHARD_NUM: return "cannot create Encoder with more than 256 data+parity shards";
        case ZS3_ERR_TOO_FEW_SHARDS: return "too few shards given";
        case ZS3_ERR_SHARD_NO_DATA: return "no shard data";
        case ZS3_ERR_SHARD_SIZE: return "shard sizes do not match";
        case ZS3_ERR_SHORT_DATA: return "not enough data to fill the number of requested shards";
        case ZS3_ERR_FILE_CORRUPT: return "file is corrupted";
        case ZS3_ERR_INVALID_ARG: return "invalid arguments specified";
        case ZS3_ERR_DEVICE: return "device error";
        case ZS3_ERR_NOMEM: return "out of memory";
        case ZS3_ERR_SINGULAR: return "matrix is singular";
        default: return "unknown error";
    }
}

int zs3_version(void) { return (kMajor << 16) | (kMinor << 8) | kPatch; }

int zs3_device_count(int* count) {
    if (!count) return ZS3_ERR_INVALID_ARG;
    return map_hip(hipGetDeviceCount(count));
}
int zs3_set_device(int device) { return map_hip(hipSetDevice(device)); }
int zs3_dev_alloc(void** d_ptr, size_t bytes) {
    if (!d_ptr) return ZS3_ERR_INVALID_ARG;
    return map_hip(hipMalloc(d_ptr, bytes));
}
int zs3_dev_free(void* d_ptr) { return map_hip(hipFree(d_ptr)); }
int zs3_host_alloc(void** h_ptr, size_t bytes) {
    if (!h_ptr) return ZS3_ERR_INVALID_ARG;
    int rc = map_hip(hipHostMalloc(h_ptr, bytes, hipHostMallocMapped | hipHostMallocPortable));
    if (rc == ZS3_OK && *h_ptr) {
        void* dev = nullptr;
        if (hipHostGetDevicePointer(&dev, *h_ptr, 0) != hipSuccess || !dev) dev = *h_ptr;  // unified addressing
        std::lock_guard<std::mutex> g(g_pin_mu);
        g_pinned[(uintptr_t)*h_ptr] = PinnedRange{bytes, (uintptr_t)dev};
    }
    return rc;
}
int zs3_host_free(void* h_ptr) {
    {
        // only what zs3_host_alloc returned: the pinned bpool's Go-heap fallback buffers
        // (and any other pointer) are refused untouched, so a pool may call this on every
        // buffer it drops
        std::lock_guard<std::mutex> g(g_pin_mu);
        if (g_pinned.erase((uintptr_t)h_ptr) == 0) return ZS3_ERR_INVALID_ARG;
    }
    return map_hip(hipHostFree(h_ptr));
}
int zs3_memcpy_h2d(void* d, const void* h, size_t bytes, void* stream) {
    return map_hip(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
}
int zs3_memcpy_d2h(void* h, const void* d, size_t bytes, void* stream) {
    return map_hip(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
}
int zs3_stream_sync(void* stream) { return map_hip(hipStreamSynchronize((hipStream_t)stream)); }

int zs3_codec_new(int k, int m, int64_t block_size, zs3_codec** out) {
    if (!out) return ZS3_ERR_INVALID_ARG;
    *out = nullptr;
    // NewErasure, cmd/erasure-coding.go:44-50
    if (k <= 0 || m <= 0) return ZS3_ERR_INV_SHARD_NUM;
    if (k + m > 256) return ZS3_ERR_MAX_SHARD_NUM;
    std::unique_ptr<zs3_codec> c(new zs3_codec());
    c->k = k;
    c->m = m;
    c->block_size = block_size;
    const int rc = zs3::build_codec_tables(k, m, *c);
    if (rc) return rc;
    *out = c.release();
    return ZS3_OK;
}

void zs3_codec_free(zs3_codec* c) { delete c; }

int zs3_codec_matrix(const zs3_codec* c, uint8_t* out) {
    if (!c || !out) return ZS3_ERR_INVALID_ARG;
    std::memcpy(out, c->matrix.data(), c->matrix.size());
    return ZS3_OK;
}

int zs3_codec_params(const zs3_codec* c, int* k, int* m, int64_t* block_size) {
    if (!c) return ZS3_ERR_INVALID_ARG;
    if (k) *k = c->k;
    if (m) *m = c->m;
    if (block_size) *block_size = c->block_size;
    return ZS3_OK;
}

int64_t zs3_shard_size(const zs3_codec* c) { return c ? ceil_frac(c->block_size, c->k) : 0; }

int64_t zs3_shard_file_size(const zs3_codec* c, int64_t total) {
    if (!c) return 0;
    if (total == 0) return 0;
    if (total == -1) return -1;
    const int64_t num = total / c->block_size;
    const int64_t last = total % c->block_size;
    return num * zs3_shard_size(c) + ceil_frac(last, c->k);
}

int64_t zs3_shard_file_offset(const zs3_codec* c, int64_t start, int64_t length, int64_t total) {
    if (!c) return 0;
    const int64_t ss = zs3_shard_size(c);
    const int64_t sfs = zs3_shard_file_size(c, total);
    const int64_t end_shard = (start + length) / c->block_size;
    int64_t till = end_shard * ss + ss;
    if (till > sfs) till = sfs;
    return till;
}

int64_t zs3_bitrot_shard_file_size(int64_t size, int64_t shard_size) {
    return ceil_frac(size, shard_size) * 32 + size;
}

// Batch layout checks: a caller's layout error comes back as
// ZS3_ERR_INVALID_ARG instead of becoming an out-of-bounds or overlapping device access.
// Encode: block b reads d_data + b*ds + [0, len) and writes d_parity + b*ps + [0, m*S);
// blocks must not overlap (ds >= len, ps >= m*S when n > 1) and no parity row may land
// on a data byte (the kernels read a tile's data rows before its parity rows are
// written, but a later tile's data must survive).  Disjoint data and parity spans
// (separate regions, as the queue's slots — whatever the strides, so k == m slots with
// equal strides pass) are accepted first; overlapping spans only with equal strides (the
// reference's in-place Split layout, parity = data + k*S), checked per period.  The
// diagnostics build also accepts ds = ps = 0: every block aliased onto block 0
// (timing-only L2-resident runs, scripts/sweep_variants.py SWEEP_ALIAS).
static bool encode_layout_ok(const uint8_t* data, int64_t ds, int64_t len, int64_t n, const uint8_t* parity,
                             int64_t ps, int64_t mS) {
#if ZS3_DIAG
    if (ds == 0 && ps == 0) return true;
#endif
    if (ds < 0 || ps < 0) return false;
    if (n > 1 && (ds < len || ps < mS)) return false;
    const int64_t off = (int64_t)((uintptr_t)parity - (uintptr_t)data);
    const int64_t d_end = (n - 1) * ds + len, p_end = off + (n - 1) * ps + mS;
    if (p_end <= 0 || off >= d_end) return true;  // disjoint spans
    if (n == 1 || ds != ps) return false;
    // equal strides, interleaved spans: the parity rows of every block sit in the gap of one period
    const int64_t r = ((off % ds) + ds) % ds;
    return r >= len && r + mS <= ds;
}

// Reconstruct / verify: block b's k+m shard rows at d_shards + b*stride + i*S.
static bool stripe_layout_ok(int64_t stride, int64_t n, int64_t RS) { return stride >= 0 && (n <= 1 || stride >= RS); }

int zs3_encode_batch(const zs3_codec* cc, const uint8_t* d_data, int64_t data_stride, int64_t block_len,
                     int64_t n_blocks, uint8_t* d_parity, int64_t parity_stride, uint8_t* d_sums,
                     void* stream) {
    zs3_codec* c = const_cast<zs3_codec*>(cc);
    if (!c || block_len < 0 || n_blocks < 0) return ZS3_ERR_INVALID_ARG;
    if (block_len == 0 || n_blocks == 0) return ZS3_OK;  // EncodeData len 0: k+m empty shards
    if (!d_data || !d_parity) return ZS3_ERR_INVALID_ARG;
    const int64_t S = ceil_frac(block_len, c->k);
    if (!encode_layout_ok(d_data, data_stride, block_len, n_blocks, d_parity, parity_stride, (int64_t)c->m * S))
        return ZS3_ERR_INVALID_ARG;
    zs3k::EncArgs a{};
    int rc = codec_device(c, &a.tables, &a.matrix);
    if (rc) return rc;
    a.data = d_data;
    a.data_stride = data_stride;
    a.parity = d_parity;
    a.parity_stride = parity_stride;
    a.sums = d_sums;
    a.S = S;
    a.n = block_len;
    a.n_blocks = n_blocks;
    a.k = c->k;
    a.m = c->m;
    a.dyb = c->dyb;
    a.dtables = a.tables + c->dyadic_off;
    key_words(nullptr, a.key);
    a.variant = call_variant();
#if ZS3_DIAG
    if (t_no_dyadic) a.dyb = 0;
    a.dbg = t_dbg;
#endif
    int path = zs3k::PATH_NONE;
    rc = map_hip(zs3k::launch_encode(a, (hipStream_t)stream, &path));
    note_path(path);
    return rc;
}

int zs3_reconstruct_batch(const zs3_codec* cc, uint8_t* d_shards, int64_t block_stride, int64_t shard_len,
                          int64_t n_blocks, const uint8_t* present, int data_only, void* stream) {
    zs3_codec* c = const_cast<zs3_codec*>(cc);
    if (!c || !present || shard_len < 0 || n_blocks < 0) return ZS3_ERR_INVALID_ARG;
    auto plan = get_plan(c, present, data_only);
    if (plan->status) return plan->status;
    if (shard_len == 0) return ZS3_ERR_SHARD_NO_DATA;
    if (plan->noop || n_blocks == 0) return ZS3_OK;
    if (!d_shards || !stripe_layout_ok(block_stride, n_blocks, (int64_t)(c->k + c->m) * shard_len))
        return ZS3_ERR_INVALID_ARG;
    zs3k::RecArgs a{};
    int rc = plan_device(c, plan.get(), &a.tables, &a.coef, &a.rows);
    if (rc) return rc;
    a.shards = d_shards;
    a.block_stride = block_stride;
    a.S = shard_len;
    a.n_blocks = n_blocks;
    a.k = c->k;
    a.e = plan->e;
    a.variant = call_variant();
    int path = zs3k::PATH_NONE;
    rc = map_hip(zs3k::launch_reconstruct(a, (hipStream_t)stream, &path));
    note_path(path);
    return rc;
}

int zs3_verify_reconstruct_batch(const zs3_codec* cc, uint8_t* d_shards, int64_t block_stride, int64_t shard_len,
                                 int64_t n_blocks, const uint8_t* present, int data_only, const uint8_t* d_expect,
                                 int32_t* d_bad, uint8_t* d_sums_out, void* stream) {
    zs3_codec* c = const_cast<zs3_codec*>(cc);
    if (!c || !present || shard_len < 0 || n_blocks < 0) return ZS3_ERR_INVALID_ARG;
    auto plan = get_plan(c, present, data_only);
    if (plan->status) return plan->status;
    if (shard_len == 0) return ZS3_ERR_SHARD_NO_DATA;
    if (n_blocks == 0) return ZS3_OK;
    if (!d_shards || !d_expect || !d_bad) return ZS3_ERR_INVALID_ARG;
    const int R = c->k + c->m;
    if (!stripe_layout_ok(block_stride, n_blocks, (int64_t)R * shard_len)) return ZS3_ERR_INVALID_ARG;
    int rc = map_hip(hipMemsetAsync(d_bad, 0, (size_t)n_blocks * R * 4, (hipStream_t)stream));
    if (rc) return rc;
    zs3k::VrArgs a{};
    rc = plan_device(c, plan.get(), &a.tables, &a.coef, &a.rows);
    if (rc) return rc;
    a.shards = d_shards;
    a.block_stride = block_stride;
    a.S = shard_len;
    a.n_blocks = n_blocks;
    a.k = c->k;
    a.m = c->m;
    a.e = plan->noop ? 0 : plan->e;
    a.expect = d_expect;
    a.bad = d_bad;
    a.sums_out = a.e > 0 ? d_sums_out : nullptr;
    a.h_rows = plan->rows.data();
    key_words(nullptr, a.key);
    a.variant = call_variant();
#if ZS3_DIAG
    a.dbg = t_dbg;
#endif
    int path = zs3k::PATH_NONE;
    rc = map_hip(zs3k::launch_verify_reconstruct(a, (hipStream_t)stream, &path));
    note_path(path);
    return rc;
}

static int digest_batch(bool sha, const uint8_t* d_msgs, int64_t stride, int64_t len, const int64_t* d_lens,
                        const int64_t* d_offs, int64_t n, uint8_t* d_out, void* stream) {
    if (n < 0 || (n > 0 && (!d_out || !d_msgs)) || (!d_lens && len < 0)) return ZS3_ERR_INVALID_ARG;
    // one message's block count is kept in 32 bits by the kernels
    if (!d_lens && len >= ((int64_t)1 << 36)) return ZS3_ERR_INVALID_ARG;
    zs3k::DigestArgs a{};
    a.msgs = d_msgs;
    a.stride = stride;
    a.len = len;
    a.lens = d_lens;
    a.offs = d_offs;
    a.n = n;
    a.out = d_out;
    a.variant = call_variant();
    return map_hip(sha ? zs3k::launch_sha256(a, (hipStream_t)stream) : zs3k::launch_md5(a, (hipStream_t)stream));
}

int zs3_md5_batch(const uint8_t* d_msgs, int64_t stride, int64_t len, const int64_t* d_lens, int64_t n,
                  uint8_t* d_out, void* stream) {
    return digest_batch(false, d_msgs, stride, len, d_lens, nullptr, n, d_out, stream);
}

int zs3_sha256_batch(const uint8_t* d_msgs, int64_t stride, int64_t len, const int64_t* d_lens, int64_t n,
                     uint8_t* d_out, void* stream) {
    return digest_batch(true, d_msgs, stride, len, d_lens, nullptr, n, d_out, stream);
}

int zs3_md5_parts(const uint8_t* d_base, const int64_t* d_offsets, const int64_t* d_lens, int64_t n,
                  uint8_t* d_out, void* stream) {
    if (n > 0 && (!d_offsets || !d_lens)) return ZS3_ERR_INVALID_ARG;
    return digest_batch(false, d_base, 0, 0, d_lens, d_offsets, n, d_out, stream);
}

int zs3_sha256_parts(const uint8_t* d_base, const int64_t* d_offsets, const int64_t* d_lens, int64_t n,
                     uint8_t* d_out, void* stream) {
    if (n > 0 && (!d_offsets || !d_lens)) return ZS3_ERR_INVALID_ARG;
    return digest_batch(true, d_base, 0, 0, d_lens, d_offsets, n, d_out, stream);
}

// etag.Multipart (internal/etag/etag.go:211-226): skip multipart ("-N") and encrypted
// (longer than 16 bytes, no '-') ETags, MD5 the concatenation of the rest on the device,
// append '-' and the decimal count.
int zs3_etag_multipart(const uint8_t* h_etags, const int64_t* offsets, const int64_t* lens, int64_t n,
                       uint8_t* h_out) {
    if (n < 0 || (n > 0 && (!h_etags || !offsets || !lens)) || !h_out) return ZS3_ERR_INVALID_ARG;
    if (n == 0) return 0;
    std::vector<uint8_t> cat;
    int64_t count = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (lens[i] < 0) return ZS3_ERR_INVALID_ARG;
        if (lens[i] > 16) continue;  // IsMultipart or IsEncrypted (etag.go:145-155)
        cat.insert(cat.end(), h_etags + offsets[i], h_etags + offsets[i] + lens[i]);
        ++count;
    }
    uint8_t* d = nullptr;
    const size_t bytes = cat.size() + 16;
    if (hipMalloc(&d, bytes) != hipSuccess) return ZS3_ERR_NOMEM;
    int rc = ZS3_OK;
    if (!cat.empty()) rc = map_hip(hipMemcpy(d, cat.data(), cat.size(), hipMemcpyHostToDevice));
    if (!rc) rc = zs3_md5_batch(d, 0, (int64_t)cat.size(), nullptr, 1, d + cat.size(), nullptr);
    if (!rc) rc = map_hip(hipMemcpy(h_out, d + cat.size(), 16, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    if (rc) return rc;
    char suffix[24];
    const int ns = snprintf(suffix, sizeof suffix, "-%lld", (long long)count);
    memcpy(h_out + 16, suffix, (size_t)ns);
    return 16 + ns;
}

int zs3_hh256_batch(const uint8_t* key, const uint8_t* d_msgs, int64_t stride, int64_t len, int64_t n,
                    uint8_t* d_sums, void* stream) {
    if (len < 0 || n < 0 || (n > 0 && !d_sums)) return ZS3_ERR_INVALID_ARG;
    zs3k::HashArgs a{};
    a.variant = call_variant();
    a.msgs = d_msgs;
    a.stride = stride;
    a.len = len;
    a.n = n;
    a.sums = d_sums;
    key_words(key, a.key);
    return map_hip(zs3k::launch_hash(a, (hipStream_t)stream));
}

int zs3_hh256_verify_batch(const uint8_t* key, const uint8_t* d_msgs, int64_t stride, int64_t len, int64_t n,
                           const uint8_t* d_want, int32_t* d_bad, void* stream) {
    if (len < 0 || n < 0 || (n > 0 && (!d_want || !d_bad))) return ZS3_ERR_INVALID_ARG;
    zs3k::HashArgs a{};
    a.variant = call_variant();
    a.msgs = d_msgs;
    a.stride = stride;
    a.len = len;
    a.n = n;
    a.expect = d_want;
    a.bad = d_bad;
    key_words(key, a.key);
    return map_hip(zs3k::launch_hash(a, (hipStream_t)stream));
}

int zs3_reconstruct_batch_masks(const zs3_codec* cc, uint8_t* d_shards, int64_t block_stride, int64_t shard_len,
                                int64_t n_blocks, const uint8_t* present, int data_only, int32_t* status,
                                void* stream) {
    zs3_codec* c = const_cast<zs3_codec*>(cc);
    if (!c || !present || shard_len < 0 || n_blocks < 0) return ZS3_ERR_INVALID_ARG;
    std::vector<PatternGroup> groups;
    const int first = group_patterns(c, present, n_blocks, data_only, status, groups);
    if (shard_len == 0) return first ? first : (n_blocks ? ZS3_ERR_SHARD_NO_DATA : ZS3_OK);
    if (n_blocks > 0 && (!d_shards || !stripe_layout_ok(block_stride, n_blocks, (int64_t)(c->k + c->m) * shard_len)))
        return ZS3_ERR_INVALID_ARG;
    hipStream_t s = (hipStream_t)stream;
    int last = zs3k::PATH_NONE;
    int32_t* d_ids = nullptr;
    int rc = upload_group_ids(groups, true, s, &d_ids);
    if (rc) return rc;
    for (auto& g : groups) {
        if (g.blocks.empty() || g.plan->noop) continue;
        zs3k::RecArgs a{};
        rc = plan_device(c, g.plan.get(), &a.tables, &a.coef, &a.rows);
        if (rc) break;
        a.shards = g.run0 >= 0 ? d_shards + g.run0 * block_stride : d_shards;
        a.block_stride = block_stride;
        a.S = shard_len;
        a.n_blocks = (int64_t)g.blocks.size();
        a.k = c->k;
        a.e = g.plan->e;
        a.ids = g.run0 >= 0 ? nullptr : d_ids + g.ids_off;
        a.variant = call_variant();
        rc = map_hip(zs3k::launch_reconstruct(a, s, &last));
        if (rc) break;
    }
    if (d_ids) (void)hipFreeAsync(d_ids, s);
    if (rc) return rc;
    note_path(last);
    return first;
}

int zs3_verify_reconstruct_batch_masks(const zs3_codec* cc, uint8_t* d_shards, int64_t block_stride,
                                       int64_t shard_len, int64_t n_blocks, const uint8_t* present, int data_only,
                                       const uint8_t* d_expect, int32_t* d_bad, uint8_t* d_sums_out,
                                       int32_t* status, void* stream) {
    zs3_codec* c = const_cast<zs3_codec*>(cc);
    if (!c || !present || shard_len < 0 || n_blocks < 0) return ZS3_ERR_INVALID_ARG;
    std::vector<PatternGroup> groups;
    const int first = group_patterns(c, present, n_blocks, data_only, status, groups);
    if (shard_len == 0) return first ? first : (n_blocks ? ZS3_ERR_SHARD_NO_DATA : ZS3_OK);
    if (n_blocks == 0) return first;
    if (!d_shards || !d_expect || !d_bad) return ZS3_ERR_INVALID_ARG;
    hipStream_t s = (hipStream_t)stream;
    const int R = c->k + c->m;
    if (!stripe_layout_ok(block_stride, n_blocks, (int64_t)R * shard_len)) return ZS3_ERR_INVALID_ARG;
    int rc = map_hip(hipMemsetAsync(d_bad, 0, (size_t)n_blocks * R * 4, s));
    if (rc) return rc;
    int last = zs3k::PATH_NONE;
    int32_t* d_ids = nullptr;
    rc = upload_group_ids(groups, false, s, &d_ids);
    if (rc) return rc;
    for (auto& g : groups) {
        if (g.blocks.empty()) continue;
        zs3k::VrArgs a{};
        rc = plan_device(c, g.plan.get(), &a.tables, &a.coef, &a.rows);
        if (rc) break;
        const int64_t b0 = g.run0 >= 0 ? g.run0 : 0;
        a.shards = d_shards + b0 * block_stride;
        a.block_stride = block_stride;
        a.S = shard_len;
        a.n_blocks = (int64_t)g.blocks.size();
        a.k = c->k;
        a.m = c->m;
        a.e = g.plan->noop ? 0 : g.plan->e;
        a.expect = d_expect + b0 * R * 32;
        a.bad = d_bad + b0 * R;
        a.sums_out = a.e > 0 && d_sums_out ? d_sums_out + b0 * R * 32 : nullptr;
        a.h_rows = g.plan->rows.data();
        a.ids = g.run0 >= 0 ? nullptr : d_ids + g.ids_off;
        key_words(nullptr, a.key);
        a.variant = call_variant();
        rc = map_hip(zs3k::launch_verify_reconstruct(a, s, &last));
        if (rc) break;
    }
    if (d_ids) (void)hipFreeAsync(d_ids, s);
    if (rc) return rc;
    note_path(last);
    return first;
}

int zs3_hh256_batch_ragged(const uint8_t* key, const uint8_t* const* d_ptrs, const int64_t* d_lens, int64_t n,
                           uint8_t* d_sums, void* stream) {
    if (n < 0 || (n > 0 && (!d_ptrs || !d_lens || !d_sums))) return ZS3_ERR_INVALID_ARG;
    zs3k::HashArgs a{};
    a.variant = call_variant();
    a.ptrs = d_ptrs;
    a.lens = d_lens;
    a.n = n;
    a.sums = d_sums;
    key_words(key, a.key);
    return map_hip(zs3k::launch_hash(a, (hipStream_t)stream));
}

int zs3_bitrot_verify_file_batch(const uint8_t* key, const uint8_t* d_files, int64_t file_stride, int64_t n_files,
                                 int64_t want_size, int64_t part_size, int64_t shard_size, int32_t* d_bad,
                                 int32_t* d_file_bad, int64_t* chunks_out, void* stream) {
    if (n_files < 0 || part_size < 0 || shard_size <= 0) return ZS3_ERR_INVALID_ARG;
    // bitrot.go:159-162: the stream must be exactly bitrotShardFileSize(partSize, shardSize)
    if (want_size != zs3_bitrot_shard_file_size(part_size, shard_size)) return ZS3_ERR_FILE_CORRUPT;
    const int64_t chunks = ceil_frac(part_size, shard_size);
    if (chunks_out) *chunks_out = chunks;
    hipStream_t s = (hipStream_t)stream;
    if (n_files == 0) return ZS3_OK;
    if (chunks == 0) {
        return d_file_bad ? map_hip(hipMemsetAsync(d_file_bad, 0, (size_t)n_files * 4, s)) : ZS3_OK;
    }
    if (!d_files || !d_bad || file_stride < want_size) return ZS3_ERR_INVALID_ARG;
    zs3k::HashArgs a{};
    a.variant = call_variant();
    a.msgs = d_files;
    a.stride = file_stride;
    a.n = n_files * chunks;
    a.bad = d_bad;
    a.chunk = shard_size;
    a.nchunks = chunks;
    a.last_len = part_size - (chunks - 1) * shard_size;
    key_words(key, a.key);
    int rc = map_hip(zs3k::launch_hash(a, s));
    if (rc || !d_file_bad) return rc;
    return map_hip(zs3k::launch_any_rows(d_bad, n_files, chunks, d_file_bad, s));
}

int zs3_fill_batch(uint8_t* d_out, int64_t stride, int64_t len, int64_t n, uint64_t seed, uint64_t obj0,
                   void* stream) {
    if (len < 0 || n < 0) return ZS3_ERR_INVALID_ARG;
    return map_hip(zs3k::launch_fill(d_out, stride, len, n, seed, obj0, (hipStream_t)stream));
}

int64_t zs3_encode_data(const zs3_codec* c, uint8_t* buf, int64_t len, int64_t cap, uint8_t* h_sums) {
    if (!c || len < 0) return ZS3_ERR_INVALID_ARG;
    if (len == 0) return 0;
    if (!buf) return ZS3_ERR_INVALID_ARG;
    const int k = c->k, m = c->m, R = k + m;
    const int64_t S = ceil_frac(len, k);
    if (cap < (int64_t)R * S) return ZS3_ERR_INVALID_ARG;
    std::memset(buf + len, 0, (size_t)(k * S - len));  // reedsolomon.Split zero-fill
    const size_t dbytes = align16((size_t)R * S) + (size_t)R * 32;
    Staging* st = staging(dbytes, dbytes);
    if (!st) return ZS3_ERR_NOMEM;
    std::memcpy(st->h, buf, (size_t)(k * S));
    uint8_t* d_sums = st->d + align16((size_t)R * S);
    int rc = map_hip(hipMemcpyAsync(st->d, st->h, (size_t)(k * S), hipMemcpyHostToDevice, st->stream));
    if (rc) return rc;
    rc = zs3_encode_batch(c, st->d, (int64_t)R * S, len, 1, st->d + (size_t)k * S, (int64_t)R * S,
                          h_sums ? d_sums : nullptr, st->stream);
    if (rc) return rc;
    rc = map_hip(hipMemcpyAsync(st->h + (size_t)k * S, st->d + (size_t)k * S, (size_t)(m * S),
                                hipMemcpyDeviceToHost, st->stream));
    if (rc) return rc;
    if (h_sums) {
        rc = map_hip(hipMemcpyAsync(st->h + align16((size_t)R * S), d_sums, (size_t)R * 32,
                                    hipMemcpyDeviceToHost, st->stream));
        if (rc) return rc;
    }
    rc = map_hip(hipStreamSynchronize(st->stream));
    if (rc) return rc;
    std::memcpy(buf + (size_t)k * S, st->h + (size_t)k * S, (size_t)(m * S));
    if (h_sums) std::memcpy(h_sums, st->h + align16((size_t)R * S), (size_t)R * 32);
    return S;
}

int zs3_decode_data_blocks(const zs3_codec* cc, uint8_t* shards, int64_t S, const uint8_t* present, int data_only) {
    zs3_codec* c = const_cast<zs3_codec*>(cc);
    if (!c || !present || S < 0) return ZS3_ERR_INVALID_ARG;
    auto plan = get_plan(c, present, data_only);
    if (plan->status) return plan->status;
    if (S == 0) return ZS3_ERR_SHARD_NO_DATA;
    if (plan->noop) return ZS3_OK;
    const int R = c->k + c->m;
    const size_t bytes = (size_t)R * S;
    Staging* st = staging(bytes, bytes);
    if (!st) return ZS3_ERR_NOMEM;
    std::memcpy(st->h, shards, bytes);
    int rc = map_hip(hipMemcpyAsync(st->d, st->h, bytes, hipMemcpyHostToDevice, st->stream));
    if (rc) return rc;
    rc = zs3_reconstruct_batch(c, st->d, (int64_t)bytes, S, 1, present, data_only, st->stream);
    if (rc) return rc;
    rc = map_hip(hipMemcpyAsync(st->h, st->d, bytes, hipMemcpyDeviceToHost, st->stream));
    if (rc) return rc;
    rc = map_hip(hipStreamSynchronize(st->stream));
    if (rc) return rc;
    for (size_t i = plan->rows.size() - plan->e; i < plan->rows.size(); ++i) {
        const int r = plan->rows[i];
        std::memcpy(shards + (size_t)r * S, st->h + (size_t)r * S, (size_t)S);
    }
    return ZS3_OK;
}

int zs3_hh256(const uint8_t* key, const uint8_t* msg, int64_t len, uint8_t* out32) {
    if (len < 0 || !out32 || (len > 0 && !msg)) return ZS3_ERR_INVALID_ARG;
    const size_t mb = align16((size_t)len > 0 ? (size_t)len : 1);
    Staging* st = staging(mb + 32, mb + 32);
    if (!st) return ZS3_ERR_NOMEM;
    if (len) std::memcpy(st->h, msg, (size_t)len);
    int rc = map_hip(hipMemcpyAsync(st->d, st->h, mb, hipMemcpyHostToDevice, st->stream));
    if (rc) return rc;
    rc = zs3_hh256_batch(key, st->d, (int64_t)mb, len, 1, st->d + mb, st->stream);
    if (rc) return rc;
    rc = map_hip(hipMemcpyAsync(st->h + mb, st->d + mb, 32, hipMemcpyDeviceToHost, st->stream));
    if (rc) return rc;
    rc = map_hip(hipStreamSynchronize(st->stream));
    if (rc) return rc;
    std::memcpy(out32, st->h + mb, 32);
    return ZS3_OK;
}

}  // extern "C"

namespace {

// Parallel memcpy for pageable <-> pinned staging (one PCIe Gen5 x16 link needs
// more than one CPU core of memcpy bandwidth).
void par_memcpy(uint8_t* dst, const uint8_t* src, size_t n, int threads) {
    if (n < (8u << 20) || threads <= 1) {
        std::memcpy(dst, src, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = ((n + threads - 1) / threads + 4095) & ~(size_t)4095;
    for (int t = 0; t < threads; ++t) {
        const size_t lo = (size_t)t * per;
        if (lo >= n) break;
        const size_t len = std::min(per, n - lo);
        th.emplace_back([=] { std::memcpy(dst + lo, src + lo, len); });
    }
    for (auto& x : th) x.join();
}

// Staging buffers of the stream drivers (stream_range, stream_vr_range), kept across
// calls: pinning hundreds of MiB of host memory and allocating the device slots cost more
// than a 4 GiB stream's own transfers (a 4 GiB pageable RS(16+4) stream: 0.35 s, most of
// it hipHostMalloc; profiles/r05/stream.jsonl).  Idle buffers are reused by the next call
// on the same device (first fit of at most twice the size asked for); at most g_pool_max
// bytes stay idle (6 GiB unless the process sets another cap with zs3_pool_limit, which
// also trims at once), the oldest idle buffers are freed first.
struct PoolBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool host = false;
    int dev = -1;
};
std::mutex g_pool_mu;
std::vector<PoolBuf> g_pool;  // idle
size_t g_pool_idle = 0;
size_t g_pool_max = (size_t)6 << 30;

hipError_t pool_get(bool host, size_t bytes, void** out) {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (size_t i = 0; i < g_pool.size(); ++i) {
            const PoolBuf& b = g_pool[i];
            if (b.host == host && (host || b.dev == dev) && b.cap >= bytes && b.cap <= 2 * bytes + (1 << 20)) {
                *out = b.p;
                g_pool_idle -= b.cap;
                g_pool.erase(g_pool.begin() + (std::ptrdiff_t)i);
                return hipSuccess;
            }
        }
    }
    return host ? hipHostMalloc(out, bytes, hipHostMallocDefault) : hipMalloc(out, bytes);
}

// with g_pool_mu held: move idle buffers past the cap (oldest first) into `drop`
void pool_evict_locked(std::vector<PoolBuf>& drop) {
    while (g_pool_idle > g_pool_max && !g_pool.empty()) {
        drop.push_back(g_pool.front());
        g_pool_idle -= g_pool.front().cap;
        g_pool.erase(g_pool.begin());
    }
}

size_t pool_free(const std::vector<PoolBuf>& drop) {
    size_t n = 0;
    for (auto& b : drop) {
        n += b.cap;
        if (b.host) {
            (void)hipHostFree(b.p);
        } else {
            int cur = -1;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(b.dev);
            (void)hipFree(b.p);
            (void)hipSetDevice(cur);
        }
    }
    return n;
}

void pool_put(bool host, void* p, size_t bytes) {
    if (!p) return;
    int dev = -1;
    (void)hipGetDevice(&dev);
    std::vector<PoolBuf> drop;
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        g_pool.push_back(PoolBuf{p, bytes, host, dev});
        g_pool_idle += bytes;
        pool_evict_locked(drop);
    }
    (void)pool_free(drop);
}

// The device-side address of pinned host memory (a kernel's view of it), or nullptr.
uint8_t* host_dev_ptr(void* p) {
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || !d) {
        (void)hipGetLastError();
        return nullptr;
    }
    return (uint8_t*)d;
}

bool is_pinned(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeHost;
}

}  // namespace

extern "C" {

int64_t zs3_pool_limit(uint64_t max_idle_bytes) {
    std::vector<PoolBuf> drop;
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        g_pool_max = (size_t)max_idle_bytes;
        pool_evict_locked(drop);
    }
    return (int64_t)pool_free(drop);
}

}  // extern "C"

namespace {

// One device's share of an end-to-end stream (blocks [b0, b1) of full size B): a
// 3-slot pipeline.  For pageable caller buffers the host copies run on helper tasks —
// pageable -> pinned for batch i+1 while batch i is in flight, pinned -> pageable for
// batch i once its D2H event fires — so the submitting thread only enqueues
// H2D -> fused kernel -> D2H (three streams, cross-stream events) and never copies.
int stream_range(zs3_codec* c, int device, const uint8_t* src, int64_t b0, int64_t b1, uint8_t* h_parity,
                 uint8_t* h_sums, int64_t NB, bool src_pinned, bool out_pinned, int cpu_threads) {
    if (b1 <= b0) return ZS3_OK;
    NB = std::min(NB, b1 - b0);
    if (hipSetDevice(device) != hipSuccess) return ZS3_ERR_DEVICE;
    const int k = c->k, m = c->m, R = k + m;
    const int64_t B = c->block_size;
    const int64_t S = ceil_frac(B, k);
    const int64_t stride = (int64_t)R * S;
    constexpr int NS = 3;
    struct Slot {
        uint8_t* d = nullptr;     // NB stripes [k*S data | m*S parity] + sums
        uint8_t* hin = nullptr;   // pinned input staging (pageable src)
        uint8_t* hout = nullptr;  // pinned parity+sums staging (pageable outputs)
        hipEvent_t in_done = nullptr, out_done = nullptr;
        bool used = false;
        std::future<int> fill, drain;
    };
    Slot sl[NS];
    hipStream_t s_in = nullptr, s_comp = nullptr, s_out = nullptr;
    hipEvent_t ev_in = nullptr, ev_comp = nullptr;
    int rc = ZS3_OK;
    auto chk = [&](hipError_t e) {
        if (e != hipSuccess && rc == ZS3_OK) rc = map_hip(e);
        return e == hipSuccess;
    };
    chk(hipStreamCreateWithFlags(&s_in, hipStreamNonBlocking));
    chk(hipStreamCreateWithFlags(&s_comp, hipStreamNonBlocking));
    chk(hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking));
    chk(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
    chk(hipEventCreateWithFlags(&ev_comp, hipEventDisableTiming));
    const size_t dbytes = (size_t)NB * stride + (size_t)NB * R * 32;
    const size_t obytes = (size_t)NB * m * S + (size_t)NB * R * 32;
    for (auto& x : sl) {
        chk(pool_get(false, dbytes, (void**)&x.d));
        if (!src_pinned) chk(pool_get(true, (size_t)NB * B, (void**)&x.hin));
        if (!out_pinned) chk(pool_get(true, obytes, (void**)&x.hout));
        chk(hipEventCreateWithFlags(&x.in_done, hipEventDisableTiming));
        chk(hipEventCreateWithFlags(&x.out_done, hipEventDisableTiming));
    }
    const int64_t nbatch = (b1 - b0 + NB - 1) / NB;
    const int th = std::max(1, cpu_threads / 2);  // half for the fill side, half for the drain side
    auto range = [&](int64_t i, int64_t& bb, int64_t& nb) {
        bb = b0 + i * NB;
        nb = std::min(NB, b1 - bb);
    };
    auto start_fill = [&](int64_t i) {
        Slot& x = sl[i % NS];
        int64_t bb, nb;
        range(i, bb, nb);
        const bool wait_prev = x.used;
        hipEvent_t prev = x.in_done;
        uint8_t* hin = x.hin;
        x.fill = std::async(std::launch::async, [=]() -> int {
            // the slot's previous H2D must have read hin before it is refilled
            if (wait_prev && hipEventSynchronize(prev) != hipSuccess) return ZS3_ERR_DEVICE;
            par_memcpy(hin, src + bb * B, (size_t)nb * B, th);
            return ZS3_OK;
        });
    };
    if (!src_pinned && rc == ZS3_OK) start_fill(0);
    for (int64_t i = 0; i < nbatch && rc == ZS3_OK; ++i) {
        Slot& x = sl[i % NS];
        int64_t bb, nb;
        range(i, bb, nb);
        if (x.drain.valid()) {  // the slot's previous outputs are back in the caller's buffers
            const int e = x.drain.get();
            if (e && rc == ZS3_OK) rc = e;
        }
        const uint8_t* in = src + bb * B;
        if (!src_pinned) {
            const int e = x.fill.get();
            if (e && rc == ZS3_OK) rc = e;
            in = x.hin;
        }
        if (rc) break;
        if (!src_pinned && i + 1 < nbatch) {
            Slot& y = sl[(i + 1) % NS];
            if (y.drain.valid()) {
                const int e = y.drain.get();
                if (e && rc == ZS3_OK) rc = e;
            }
            start_fill(i + 1);
        }
        // the previous use of x.d (its D2H) must be done before the H2D overwrites it
        if (x.used) chk(hipStreamWaitEvent(s_in, x.out_done, 0));
        chk(hipMemcpy2DAsync(x.d, (size_t)stride, in, (size_t)B, (size_t)B, (size_t)nb, hipMemcpyHostToDevice, s_in));
        chk(hipEventRecord(x.in_done, s_in));
        chk(hipEventRecord(ev_in, s_in));
        chk(hipStreamWaitEvent(s_comp, ev_in, 0));
        uint8_t* dsums = x.d + (size_t)NB * stride;
        const int e = zs3_encode_batch(c, x.d, stride, B, nb, x.d + (size_t)k * S, stride, dsums, s_comp);
        if (e && rc == ZS3_OK) rc = e;
        chk(hipEventRecord(ev_comp, s_comp));
        chk(hipStreamWaitEvent(s_out, ev_comp, 0));
        uint8_t* po = out_pinned ? h_parity + bb * m * S : x.hout;
        uint8_t* so = out_pinned ? h_sums + bb * R * 32 : x.hout + (size_t)NB * m * S;
        chk(hipMemcpy2DAsync(po, (size_t)m * S, x.d + (size_t)k * S, (size_t)stride, (size_t)m * S, (size_t)nb,
                             hipMemcpyDeviceToHost, s_out));
        chk(hipMemcpyAsync(so, dsums, (size_t)nb * R * 32, hipMemcpyDeviceToHost, s_out));
        chk(hipEventRecord(x.out_done, s_out));
        x.used = true;
        if (!out_pinned) {
            hipEvent_t done = x.out_done;
            uint8_t* hout = x.hout;
            x.drain = std::async(std::launch::async, [=]() -> int {
                if (hipEventSynchronize(done) != hipSuccess) return ZS3_ERR_DEVICE;
                par_memcpy(h_parity + bb * m * S, hout, (size_t)nb * m * S, th);
                std::memcpy(h_sums + bb * R * 32, hout + (size_t)NB * m * S, (size_t)nb * R * 32);
                return ZS3_OK;
            });
        }
    }
    for (auto& x : sl) {
        if (x.fill.valid()) (void)x.fill.get();
        if (x.drain.valid()) {
            const int e = x.drain.get();
            if (e && rc == ZS3_OK) rc = e;
        }
    }
    chk(hipStreamSynchronize(s_out));
    for (auto& x : sl) {
        pool_put(false, x.d, dbytes);
        pool_put(true, x.hin, (size_t)NB * B);
        pool_put(true, x.hout, obytes);
        if (x.in_done) (void)hipEventDestroy(x.in_done);
        if (x.out_done) (void)hipEventDestroy(x.out_done);
    }
    if (ev_in) (void)hipEventDestroy(ev_in);
    if (ev_comp) (void)hipEventDestroy(ev_comp);
    if (s_in) (void)hipStreamDestroy(s_in);
    if (s_comp) (void)hipStreamDestroy(s_comp);
    if (s_out) (void)hipStreamDestroy(s_out);
    return rc;
}

// Streamed GET / heal of one object's blocks on one device (zs3_stream_decode): the
// Erasure.Decode / Erasure.Heal block loops (erasure-decode.go:230-276, :287-332) as a
// 3-slot pipeline of batches: H2D of batch i+1's survivor rows || the fused verify +
// rebuild (+ heal sums) of batch i || D2H of batch i-1's rebuilt rows, flags and sums.
// Stripe b is at h + b*E (E = (k+m)*S), row j at + j*S.  Pinned caller buffers move by
// DMA, row by row across the batch (only rows some block of the batch has); pageable ones
// are staged whole-stripe by helper threads, as stream_range does.
int stream_vr_range(zs3_codec* c, uint8_t* h, int64_t nblk, const uint8_t* present, int data_only,
                    const uint8_t* h_expect, int32_t* h_bad, uint8_t* h_sums_out, int32_t* status, int64_t NB,
                    bool pinned, int cpu_threads) {
    if (nblk <= 0) return ZS3_OK;
    const int k = c->k, m = c->m, R = k + m;
    const int64_t S = ceil_frac(c->block_size, k);
    const int64_t E = (int64_t)R * S;
    const bool heal = !data_only;
    const bool hash_out = heal && h_sums_out;
    NB = std::min(NB, nblk);  // a 2-block object does not size (and pool) 128-block slots
    constexpr int NS = 3;
    struct Slot {
        uint8_t* d = nullptr;    // NB stripes | NB*R*32 expected sums | NB*R int32 flags | NB*R*32 heal sums
        uint8_t* hs = nullptr;   // pinned staging of NB stripes (pageable caller)
        uint8_t* hsm = nullptr;  // pinned staging: NB*R*32 expected sums | NB*R int32 flags | NB*R*32 heal sums
        uint8_t* hs_dev = nullptr;  // hs as a kernel addresses it (k_rows_copy)
        hipEvent_t in_done = nullptr, out_done = nullptr;
        bool used = false;
        std::future<int> fill, drain;
    };
    Slot sl[NS];
    hipStream_t s_in = nullptr, s_comp = nullptr, s_out = nullptr;
    hipEvent_t ev_in = nullptr, ev_comp = nullptr;
    int rc = ZS3_OK, first_block_err = ZS3_OK;
    auto chk = [&](hipError_t e) {
        if (e != hipSuccess && rc == ZS3_OK) rc = map_hip(e);
        return e == hipSuccess;
    };
    chk(hipStreamCreateWithFlags(&s_in, hipStreamNonBlocking));
    chk(hipStreamCreateWithFlags(&s_comp, hipStreamNonBlocking));
    chk(hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking));
    chk(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
    chk(hipEventCreateWithFlags(&ev_comp, hipEventDisableTiming));
    const size_t off_exp = (size_t)NB * E, off_bad = off_exp + (size_t)NB * R * 32, off_out = off_bad + (size_t)NB * R * 4;
    const size_t dbytes = off_out + (size_t)NB * R * 32;
    // The per-block arrays (expected sums in, flags and heal sums out) are the caller's
    // own, usually pageable, memory: an async copy to or from pageable memory makes the
    // host wait for the stream to drain first, which serialised every batch's H2D behind
    // the previous batch's D2H (rocprofv3 DMA trace, profiles/r06/dma_sg).  They move
    // through this pinned staging instead; the drain copies the outputs out.
    const size_t sm_bad = (size_t)NB * R * 32, sm_out = sm_bad + (size_t)NB * R * 4;
    const size_t smbytes = sm_out + (size_t)NB * R * 32;
    for (auto& x : sl) {
        chk(pool_get(false, dbytes, (void**)&x.d));
        chk(pool_get(true, smbytes, (void**)&x.hsm));
        if (!pinned) chk(pool_get(true, (size_t)NB * E, (void**)&x.hs));
        if (x.hs) x.hs_dev = host_dev_ptr(x.hs);
        chk(hipEventCreateWithFlags(&x.in_done, hipEventDisableTiming));
        chk(hipEventCreateWithFlags(&x.out_done, hipEventDisableTiming));
    }
    const int th = std::max(1, cpu_threads / 2);
    const int64_t nbatch = (nblk + NB - 1) / NB;
    const bool rows2d = (S % 256) == 0;  // per-row strided DMA only for aligned rows
    uint8_t* const h_dev = pinned && !rows2d ? host_dev_ptr(h) : nullptr;
    // rows of a batch: `any_present` to upload, `any_rebuilt` to bring back
    auto rows_of = [&](int64_t bb, int64_t nb, std::vector<uint8_t>& any_present, std::vector<uint8_t>& any_rebuilt) {
        any_present.assign((size_t)R, 0);
        any_rebuilt.assign((size_t)R, 0);
        for (int64_t b = bb; b < bb + nb; ++b)
            for (int j = 0; j < R; ++j) {
                if (present[b * R + j]) any_present[(size_t)j] = 1;
                else if (j < k || heal) any_rebuilt[(size_t)j] = 1;
            }
    };
    auto start_fill = [&](int64_t i) {
        Slot& x = sl[i % NS];
        const int64_t bb = i * NB, nb = std::min(NB, nblk - bb);
        const bool wait_prev = x.used;
        hipEvent_t prev = x.in_done;
        uint8_t* hs = x.hs;
        x.fill = std::async(std::launch::async, [=]() -> int {
            if (wait_prev && hipEventSynchronize(prev) != hipSuccess) return ZS3_ERR_DEVICE;
            par_memcpy(hs, h + bb * E, (size_t)(nb * E), th);
            return ZS3_OK;
        });
    };
    if (!pinned && rc == ZS3_OK) start_fill(0);
    std::vector<uint8_t> anyp, anyr;
    std::vector<int32_t> stat((size_t)NB);               // block status when the caller passes none
    std::vector<std::pair<int64_t, int64_t>> runs;        // (first block, count) served
    for (int64_t i = 0; i < nbatch && rc == ZS3_OK; ++i) {
        Slot& x = sl[i % NS];
        const int64_t bb = i * NB, nb = std::min(NB, nblk - bb);
        if (x.drain.valid()) {
            const int e = x.drain.get();
            if (e && rc == ZS3_OK) rc = e;
        }
        if (!pinned) {
            const int e = x.fill.get();
            if (e && rc == ZS3_OK) rc = e;
        }
        if (rc) break;
        if (!pinned && i + 1 < nbatch) {
            Slot& y = sl[(i + 1) % NS];
            if (y.drain.valid()) {
                const int e = y.drain.get();
                if (e && rc == ZS3_OK) rc = e;
            }
            start_fill(i + 1);
        }
        rows_of(bb, nb, anyp, anyr);
        if (x.used) chk(hipStreamWaitEvent(s_in, x.out_done, 0));
        if (pinned && rows2d) {
            for (int j = 0; j < R; ++j)
                if (anyp[(size_t)j])
                    chk(hipMemcpy2DAsync(x.d + (size_t)j * S, (size_t)E, h + bb * E + (size_t)j * S, (size_t)E, (size_t)S,
                                         (size_t)nb, hipMemcpyHostToDevice, s_in));
        } else if (pinned) {
            chk(hipMemcpyAsync(x.d, h + bb * E, (size_t)(nb * E), hipMemcpyHostToDevice, s_in));
        } else {
            chk(hipMemcpyAsync(x.d, x.hs, (size_t)(nb * E), hipMemcpyHostToDevice, s_in));
        }
        if (hash_out) chk(hipMemsetAsync(x.d + off_out, 0, (size_t)nb * R * 32, s_in));  // no stale sums
        if (h_expect) {
            std::memcpy(x.hsm, h_expect + bb * R * 32, (size_t)nb * R * 32);  // the slot's last D2H is done
            chk(hipMemcpyAsync(x.d + off_exp, x.hsm, (size_t)nb * R * 32, hipMemcpyHostToDevice, s_in));
        } else
            chk(hipMemsetAsync(x.d + off_exp, 0, (size_t)nb * R * 32, s_in));
        chk(hipEventRecord(x.in_done, s_in));
        chk(hipEventRecord(ev_in, s_in));
        chk(hipStreamWaitEvent(s_comp, ev_in, 0));
        int32_t* st_b = status ? status + bb : stat.data();
        const int e = zs3_verify_reconstruct_batch_masks(c, x.d, E, S, nb, present + bb * R, data_only, x.d + off_exp,
                                                         (int32_t*)(x.d + off_bad), hash_out ? x.d + off_out : nullptr,
                                                         st_b, s_comp);
        // runs of blocks that were served: a block with too few shards gets nothing back
        // (its rows that were never uploaded hold whatever the pooled slot last held — bytes
        // of another call — so they must not reach the caller's buffer)
        runs.clear();
        for (int64_t b = 0; b < nb;) {
            if (st_b[b] != 0) {
                ++b;
                continue;
            }
            int64_t b2 = b;
            while (b2 < nb && st_b[b2] == 0) ++b2;
            runs.emplace_back(b, b2 - b);
            b = b2;
        }
        if (e == ZS3_ERR_TOO_FEW_SHARDS || e == ZS3_ERR_SHARD_NO_DATA) {
            if (first_block_err == ZS3_OK) first_block_err = e;
        } else if (e && rc == ZS3_OK) {
            rc = e;
        }
        chk(hipEventRecord(ev_comp, s_comp));
        chk(hipStreamWaitEvent(s_out, ev_comp, 0));
        // rebuilt rows back into the caller's stripes (pinned) or the slot's staging: one
        // strided copy per rebuilt row index, or — for rows that are not 256-byte aligned,
        // which the DMA engine copies strided at a fraction of its rate (RS(12+4) on 1 MiB
        // blocks: 7.2 vs 30 GiB/s, profiles/r05/stream.jsonl) — one k_rows_copy launch per
        // run of served blocks (round 6: the whole stripes before, 8x the bytes for two
        // rebuilt rows of RS(12+4); the whole stripes still when the two bases are not
        // congruent mod 16)
        uint8_t* dst = pinned ? h + bb * E : x.hs;
        zs3k::RowSet rset{};
        int nrb = 0;  // rebuilt row indices of the batch (k_rows_copy takes up to 32)
        for (int j = 0; j < R; ++j) nrb += anyr[(size_t)j] ? 1 : 0;
        if (nrb <= 32)
            for (int j = 0; j < R; ++j)
                if (anyr[(size_t)j]) rset.row[rset.n++] = j;
        uint8_t* ddst = nullptr;  // dst as the kernel addresses it
        if (!rows2d && nrb <= 32) {
            uint8_t* base = pinned ? h_dev : x.hs_dev;
            if (base) ddst = base + (pinned ? bb * E : 0);
        }
        const bool rows_kernel = ddst && ((((uintptr_t)ddst - (uintptr_t)x.d)) & 15) == 0;
        for (const auto& rn : runs) {
            const int64_t r0 = rn.first, rl = rn.second;
            if (rows2d) {
                for (int j = 0; j < R; ++j)
                    if (anyr[(size_t)j])
                        chk(hipMemcpy2DAsync(dst + r0 * E + (size_t)j * S, (size_t)E, x.d + r0 * E + (size_t)j * S,
                                             (size_t)E, (size_t)S, (size_t)rl, hipMemcpyDeviceToHost, s_out));
            } else if (rows_kernel) {
                chk(zs3k::launch_rows_copy(x.d + r0 * E, ddst + r0 * E, E, S, rl, rset, s_out));
            } else {
                chk(hipMemcpyAsync(dst + r0 * E, x.d + r0 * E, (size_t)(rl * E), hipMemcpyDeviceToHost, s_out));
            }
        }
        if (h_bad) chk(hipMemcpyAsync(x.hsm + sm_bad, x.d + off_bad, (size_t)nb * R * 4, hipMemcpyDeviceToHost, s_out));
        if (hash_out)
            chk(hipMemcpyAsync(x.hsm + sm_out, x.d + off_out, (size_t)nb * R * 32, hipMemcpyDeviceToHost, s_out));
        chk(hipEventRecord(x.out_done, s_out));
        x.used = true;
        {
            // after the batch's D2H: flags and heal sums to the caller's arrays, and (pageable
            // stripes) the rebuilt rows of each served block from the staging
            hipEvent_t done = x.out_done;
            uint8_t* hs = pinned ? nullptr : x.hs;
            const uint8_t* hsm = x.hsm;
            std::vector<uint8_t> pres, served;
            if (!pinned) {
                pres.assign(present + bb * R, present + (bb + nb) * R);
                served.resize((size_t)nb);
                for (int64_t b = 0; b < nb; ++b) served[(size_t)b] = st_b[b] == 0;
            }
            x.drain = std::async(std::launch::async, [=]() -> int {
                if (hipEventSynchronize(done) != hipSuccess) return ZS3_ERR_DEVICE;
                if (h_bad) std::memcpy(h_bad + bb * R, hsm + sm_bad, (size_t)nb * R * 4);
                if (hash_out) std::memcpy(h_sums_out + bb * R * 32, hsm + sm_out, (size_t)nb * R * 32);
                if (hs)
                    for (int64_t b = 0; b < nb; ++b)
                        for (int j = 0; j < R; ++j)
                            if (served[(size_t)b] && !pres[(size_t)(b * R + j)] && (j < k || heal))
                                std::memcpy(h + (bb + b) * E + (size_t)j * S, hs + b * E + (size_t)j * S, (size_t)S);
                return ZS3_OK;
            });
        }
    }
    for (auto& x : sl) {
        if (x.fill.valid()) (void)x.fill.get();
        if (x.drain.valid()) {
            const int e = x.drain.get();
            if (e && rc == ZS3_OK) rc = e;
        }
    }
    chk(hipStreamSynchronize(s_out));
    for (auto& x : sl) {
        pool_put(false, x.d, dbytes);
        pool_put(true, x.hs, (size_t)NB * E);
        pool_put(true, x.hsm, smbytes);
        if (x.in_done) (void)hipEventDestroy(x.in_done);
        if (x.out_done) (void)hipEventDestroy(x.out_done);
    }
    if (ev_in) (void)hipEventDestroy(ev_in);
    if (ev_comp) (void)hipEventDestroy(ev_comp);
    if (s_in) (void)hipStreamDestroy(s_in);
    if (s_comp) (void)hipStreamDestroy(s_comp);
    if (s_out) (void)hipStreamDestroy(s_out);
    return rc ? rc : first_block_err;
}

}  // namespace

extern "C" {

void zs3_split_range(int64_t total, int world, int rank, int64_t* lo, int64_t* hi) {
    // contiguous near-equal ranges, the first total % world ranks one longer
    // (zs3server_amd/dist.py split_range)
    if (world <= 0 || rank < 0 || rank >= world || total < 0) {
        if (lo) *lo = 0;
        if (hi) *hi = 0;
        return;
    }
    const int64_t base = total / world, extra = total % world;
    const int64_t l = (int64_t)rank * base + std::min<int64_t>(rank, extra);
    if (lo) *lo = l;
    if (hi) *hi = l + base + (rank < extra ? 1 : 0);
}

int64_t zs3_stream_encode_multi(const zs3_codec* cc, const int* devices, int n_devices, const uint8_t* src,
                                int64_t total_len, uint8_t* h_parity, uint8_t* h_sums, int64_t batch_blocks) {
    zs3_codec* c = const_cast<zs3_codec*>(cc);
    if (!c || total_len < 0 || batch_blocks <= 0 || n_devices <= 0 || !devices ||
        (total_len > 0 && (!src || !h_parity || !h_sums)))
        return ZS3_ERR_INVALID_ARG;
    if (total_len == 0) return 0;
    const int k = c->k, m = c->m, R = k + m;
    const int64_t B = c->block_size;
    const int64_t S = ceil_frac(B, k);
    const int64_t nfull = total_len / B;
    const int64_t tail = total_len % B;
    const int64_t nblocks = nfull + (tail ? 1 : 0);
    const bool src_pinned = is_pinned(src);
    const bool out_pinned = is_pinned(h_parity) && is_pinned(h_sums);
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    const int cpu_threads = std::max(2, std::min(16, hw / n_devices));
    int caller_dev = 0;
    (void)hipGetDevice(&caller_dev);
    std::vector<int> rcs((size_t)n_devices, ZS3_OK);
    std::vector<std::thread> th;
    for (int r = 0; r < n_devices; ++r) {
        int64_t lo, hi;
        zs3_split_range(nfull, n_devices, r, &lo, &hi);
        th.emplace_back([&, r, lo, hi] {
            // select the device first: an empty range still encodes the tail on devices[r]
            if (hipSetDevice(devices[r]) != hipSuccess) {
                rcs[(size_t)r] = ZS3_ERR_DEVICE;
                return;
            }
            rcs[(size_t)r] = stream_range(c, devices[r], src, lo, hi, h_parity, h_sums, batch_blocks, src_pinned,
                                          out_pinned, cpu_threads);
            if (r == n_devices - 1 && tail && rcs[(size_t)r] == ZS3_OK) {
                // last partial block: EncodeData on its own shard size (erasure-encode.go:85-96)
                std::vector<uint8_t> buf((size_t)R * ceil_frac(tail, k), 0);
                std::memcpy(buf.data(), src + nfull * B, (size_t)tail);
                uint8_t sums[32 * 256];
                const int64_t St = zs3_encode_data(c, buf.data(), tail, (int64_t)buf.size(), sums);
                if (St < 0) {
                    rcs[(size_t)r] = (int)St;
                } else {
                    std::memcpy(h_parity + nfull * m * S, buf.data() + (size_t)k * St, (size_t)m * St);
                    std::memcpy(h_sums + nfull * R * 32, sums, (size_t)R * 32);
                }
            }
        });
    }
    for (auto& t : th) t.join();
    (void)hipSetDevice(caller_dev);
    for (int e : rcs)
        if (e) return e;
    return nblocks;
}

int64_t zs3_stream_encode(const zs3_codec* c, const uint8_t* src, int64_t total_len, uint8_t* h_parity,
                          uint8_t* h_sums, int64_t batch_blocks) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return ZS3_ERR_DEVICE;
    return zs3_stream_encode_multi(c, &dev, 1, src, total_len, h_parity, h_sums, batch_blocks);
}

int64_t zs3_stream_decode(const zs3_codec* cc, uint8_t* h_stripes, int64_t total_len, const uint8_t* h_present,
                          int data_only, const uint8_t* h_expect, int32_t* h_bad, uint8_t* h_sums_out,
                          int32_t* h_status, int64_t batch_blocks) {
    zs3_codec* c = const_cast<zs3_codec*>(cc);
    if (!c || total_len < 0 || batch_blocks <= 0 || (total_len > 0 && (!h_stripes || !h_present)))
        return ZS3_ERR_INVALID_ARG;
    if (total_len == 0) return 0;
    const int k = c->k, R = c->k + c->m;
    const int64_t B = c->block_size;
    const int64_t S = ceil_frac(B, k);
    const int64_t E = (int64_t)R * S;
    const int64_t nfull = total_len / B, tail = total_len % B;
    const int64_t nblocks = nfull + (tail ? 1 : 0);
    const size_t bytes = (size_t)(nblocks * E);
    const bool pinned = zs3i_pinned(h_stripes, bytes) || is_pinned(h_stripes);
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    int rc = stream_vr_range(c, h_stripes, nfull, h_present, data_only, h_expect, h_bad, h_sums_out, h_status,
                             batch_blocks, pinned, std::max(2, std::min(16, hw)));
    if (rc && rc != ZS3_ERR_TOO_FEW_SHARDS && rc != ZS3_ERR_SHARD_NO_DATA) return rc;
    if (tail) {
        // the short last block on its own shard size (erasure-decode.go:112-114): rows at
        // j*S' inside its stripe slot
        const int64_t St = ceil_frac(tail, k);
        uint8_t* stripe = h_stripes + nfull * E;
        uint8_t* d = nullptr;
        const size_t db = (size_t)R * St + (size_t)R * 32 + (size_t)R * 4 + (size_t)R * 32;
        hipStream_t s = nullptr;
        int e = map_hip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        if (!e) e = map_hip(hipMalloc(&d, db));
        const uint8_t* pres = h_present + nfull * R;
        if (!e) e = map_hip(hipMemcpyAsync(d, stripe, (size_t)R * St, hipMemcpyHostToDevice, s));
        if (!e) {
            if (h_expect)
                e = map_hip(hipMemcpyAsync(d + (size_t)R * St, h_expect + nfull * R * 32, (size_t)R * 32,
                                           hipMemcpyHostToDevice, s));
            else
                e = map_hip(hipMemsetAsync(d + (size_t)R * St, 0, (size_t)R * 32, s));
        }
        int32_t one = ZS3_OK;
        uint8_t* dbad = d + (size_t)R * St + (size_t)R * 32;
        uint8_t* dout = dbad + (size_t)R * 4;
        if (!e) {
            const int ee = zs3_verify_reconstruct_batch_masks(c, d, (int64_t)R * St, St, 1, pres, data_only,
                                                              d + (size_t)R * St, (int32_t*)dbad,
                                                              !data_only && h_sums_out ? dout : nullptr, &one, s);
            if (ee && ee != ZS3_ERR_TOO_FEW_SHARDS && ee != ZS3_ERR_SHARD_NO_DATA) e = ee;
        }
        if (h_status) h_status[nfull] = one;
        if (!e && one == ZS3_OK) {
            for (int j = 0; j < R && !e; ++j)
                if (!pres[j] && (j < k || !data_only))
                    e = map_hip(hipMemcpyAsync(stripe + (size_t)j * St, d + (size_t)j * St, (size_t)St,
                                               hipMemcpyDeviceToHost, s));
        }
        if (!e && h_bad) e = map_hip(hipMemcpyAsync(h_bad + nfull * R, dbad, (size_t)R * 4, hipMemcpyDeviceToHost, s));
        if (!e && !data_only && h_sums_out)
            e = map_hip(hipMemcpyAsync(h_sums_out + nfull * R * 32, dout, (size_t)R * 32, hipMemcpyDeviceToHost, s));
        if (s) {
            if (!e) e = map_hip(hipStreamSynchronize(s));
            (void)hipStreamDestroy(s);
        }
        if (d) (void)hipFree(d);
        if (e) return e;
        if (one != ZS3_OK && rc == ZS3_OK) rc = one;
    }
    return rc ? rc : nblocks;
}

int zs3_selftest(void) {
    // erasureSelfTest, cmd/erasure-coding.go:158-216 (want table from :169)
    int nkat = 0;
    const zs3::SelfTestKat* kat = zs3::selftest_kats(&nkat);
    int ok = 1;
    for (int ik = 0; ik < nkat; ++ik) {
        const zs3::SelfTestKat& t = kat[ik];
        zs3_codec* c = nullptr;
        if (zs3_codec_new(t.k, t.m, 1 << 20, &c)) return ZS3_ERR_FILE_CORRUPT;
        const int R = t.k + t.m;
        std::vector<uint8_t> buf(512 * 2, 0);
        for (int i = 0; i < 256; ++i) buf[i] = (uint8_t)i;
        const int64_t S = zs3_encode_data(c, buf.data(), 256, (int64_t)buf.size(), nullptr);
        if (S <= 0) {
            zs3_codec_free(c);
            return S < 0 ? (int)S : ZS3_ERR_FILE_CORRUPT;
        }
        std::vector<uint8_t> stream;
        for (int i = 0; i < R; ++i) {
            stream.push_back((uint8_t)i);
            stream.insert(stream.end(), buf.begin() + (size_t)i * S, buf.begin() + (size_t)(i + 1) * S);
        }
        if (zs3::xxh64(stream.data(), stream.size()) != t.want) ok = 0;
        // delete first shard, DecodeDataBlocks (:201-209)
        std::vector<uint8_t> first(buf.begin(), buf.begin() + S);
        std::vector<uint8_t> pres(R, 1);
        pres[0] = 0;
        std::memset(buf.data(), 0, (size_t)S);
        if (zs3_decode_data_blocks(c, buf.data(), S, pres.data(), 1) != ZS3_OK) ok = 0;
        if (std::memcmp(first.data(), buf.data(), (size_t)S) != 0) ok = 0;
        zs3_codec_free(c);
    }
    // bitrotSelfTest, cmd/bitrot.go:218-249 (HighwayHash256S)
    static const uint8_t want_hh[32] = {0x39, 0xc0, 0x40, 0x7e, 0xd3, 0xf0, 0x1b, 0x18, 0xd2, 0x2c, 0x85,
                                        0xdb, 0x4a, 0xef, 0xf1, 0x1e, 0x06, 0x0c, 0xa5, 0xf4, 0x31, 0x31,
                                        0xb0, 0x12, 0x67, 0x31, 0xca, 0x19, 0x7c, 0xd4, 0x23, 0x13};
    std::vector<uint8_t> msg;
    uint8_t sum[32] = {0};
    for (int i = 0; i < 32 * 32; i += 32) {
        if (zs3_hh256(nullptr, msg.data(), (int64_t)msg.size(), sum) != ZS3_OK) return ZS3_ERR_DEVICE;
        msg.insert(msg.end(), sum, sum + 32);
    }
    if (std::memcmp(sum, want_hh, 32) != 0) ok = 0;
    return ok ? ZS3_OK : ZS3_ERR_FILE_CORRUPT;
}

int zs3_last_path(void) { return t_last_path; }

uint32_t zs3_path_mask(int reset) {
    const uint32_t m = t_path_mask | zs3k::kernel_bits(reset != 0);
    if (reset) t_path_mask = 0;
    return m;
}

#if ZS3_DIAG
int zs3_debug_set_variant(int variant) {
    // variant >= 1000: same variant with the plain (non-dyadic) GF encode
    t_no_dyadic = variant >= 1000;
    t_variant = variant % 1000;
    return ZS3_OK;
}

int zs3_debug_set_buffer(void* d_dbg) {
    t_dbg = (uint64_t*)d_dbg;
    return ZS3_OK;
}

int zs3_debug_encode_layout_ok(const void* d_data, int64_t data_stride, int64_t block_len, int64_t n_blocks,
                               const void* d_parity, int64_t parity_stride, int64_t parity_bytes) {
    return encode_layout_ok((const uint8_t*)d_data, data_stride, block_len, n_blocks, (const uint8_t*)d_parity,
                            parity_stride, parity_bytes) ? 1 : 0;
}
#endif

}  // extern "C"
