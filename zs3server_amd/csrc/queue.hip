// queue.hip — cross-request batching submission queue (SURVEY.md §8b "Threading",
// §7 hard part iv).
//
// The reference encodes ONE 1 MiB block per request, strictly sequentially per object
// (cmd/erasure-encode.go:83-111 -> Erasure.EncodeData, cmd/erasure-coding.go:77-91),
// and decodes one block per parallelReader round (cmd/erasure-decode.go:230-276 ->
// DecodeDataBlocks :96).  One block is ~0.2 us of HBM work against tens of us of
// fixed launch + PCIe cost, so a drop-in that calls the device once per block loses to
// the CPU.  This queue gathers the blocks of all concurrent requests (every Go
// goroutine that calls EncodeData / DecodeDataBlocks sits in its own OS thread inside
// cgo) into device batches:
//
//   submitter thread:  reserve a position in the lane's open slot (pinned staging),
//                      copy its block in (in parallel with other submitters), return a
//                      zs3_req handle
//   dispatcher thread: close the open slot when it is full, when nothing is in flight
//                      (batch-while-busy: an idle device gets work at once, a busy
//                      one lets the next batch grow), when the oldest block has waited
//                      max_wait_us, or on flush; then H2D -> kernels -> D2H on the
//                      lane's stream, all asynchronous
//   completer thread:  waits for each launched slot's event, marks the slot ready and
//                      wakes the waiters, then copies out every block nobody claimed
//   zs3_req_wait:      once its slot is ready the submitter claims its own block and
//                      copies the results into its buffers itself (as each goroutine
//                      encodes its own block in the reference), in parallel with the
//                      other waiters; if the completer claimed it first, it waits
// Each block is claimed exactly once (an atomic flag per slot position); whoever
// finishes the slot's last block frees the slot.  Slot reuse never depends on a
// waiter (the completer claims what is not being waited for), so a thread may hold any
// number of un-waited requests.
//
// Lanes: ENCODE (EncodeData + the k+m bitrot sums), GET (ReconstructData of the
// missing data shards, with the survivors' bitrot sums verified in the same pass when
// given — parallelReader + DecodeDataBlocks), HEAL (Reconstruct of data and parity plus
// the rebuilt shards' sums — Erasure.Heal, cmd/erasure-decode.go:287-332).  Every block
// in a batch keeps its own erasure pattern (zs3_verify_reconstruct_batch_masks).
// Blocks of the full shard size fill a slot from the front and go in one launch; the
// short last block of an object (its own shard size, erasure-encode.go:85-96) fills
// from the back and is launched on its own.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/zs3gpu.h"
#include "queue_policy.hpp"

bool zs3i_pinned(const void* p, size_t n);  // zs3gpu.hip: inside a live zs3_host_alloc range
bool zs3i_pinned_map(const void* p, size_t n, void** dev);  // ... and its device-side address

namespace {

enum Lane { ENC = 0, GET = 1, HEAL = 2, NLANE = 3 };
using Clock = std::chrono::steady_clock;

struct Slot;

}  // namespace

struct DevQ;

struct zs3_req {
    DevQ* q = nullptr;
    Slot* slot = nullptr;
    int lane = ENC;
    int pos = 0;
    int64_t S = 0;  // shard size of this block
    // encode
    uint8_t* h_buf = nullptr;
    int64_t len = 0;
    uint8_t* h_sums = nullptr;
    // decode
    uint8_t* h_shards = nullptr;
    uint8_t present[256];
    const uint8_t* h_expect = nullptr;
    int32_t* h_bad = nullptr;
    uint8_t* h_sums_out = nullptr;
    int status = ZS3_OK;   // the block's status at launch (its pattern's reedsolomon error)
    bool zc = false;       // zero-copy: the caller's buffer is pinned (zs3_host_alloc), so its
                           // bytes move to / from the device slot without host staging
    uint8_t* d_map = nullptr;  // zc (copy-list mode): the caller's buffer as a kernel addresses it
    bool done = false;     // results copied out (completer)
    int64_t result = 0;    // zs3_req_wait's return value
};

namespace {

struct Slot {
    int lane = ENC;
    uint8_t* h = nullptr;  // pinned, same layout as d
    uint8_t* d = nullptr;
    enum State { FREE, OPEN, LAUNCHED } state = FREE;
    int front = 0;         // next full-size position
    int back = 0;          // short blocks placed at cap-1, cap-2, ...
    int copying = 0;       // submitters still copying in
    std::vector<zs3_req*> reqs;
    Clock::time_point opened;
    hipEvent_t done_ev = nullptr;
    hipEvent_t start_ev = nullptr;  // diagnostics build: the batch's first stream op (timing)
    hipStream_t stream = nullptr;  // per slot: batches overlap each other's kernels
    hipEvent_t ev_in = nullptr;    // split streams: the batch's H2D copies are done
    hipEvent_t ev_comp = nullptr;  // split streams: the batch's kernels are done
    int launch_status = ZS3_OK;
    bool ready = false;                          // results are in the pinned slot
    int nblocks = 0;                             // blocks at launch (inflight_blocks)
    std::unique_ptr<std::atomic<uint8_t>[]> claimed;  // [cap] block copied out by one thread
    std::atomic<int> pending{0};                 // blocks not yet finished (+1 completer)
};

}  // namespace

#if ZS3_DIAG
enum QTimer {
    QT_SUB_LOCK,    // submitters: lock + slot reservation (incl. backpressure waits)
    QT_SUB_COPY,    // submitters: copy-in (memcpy into the pinned slot / zero-copy DMA call)
    QT_DISP_LAUNCH, // dispatcher: launch_slot (HIP enqueue calls)
    QT_COMP_SYNC,   // completer: waiting for a batch's done event
    QT_WAIT_READY,  // waiters: zs3_req_wait until the batch's results are in the slot
    QT_COPY_OUT,    // waiters / completer: copy-out (finish_req)
    QT_GPU_SUM,     // sum of the batches' stream intervals (first copy in .. done), us*1000
    QT_GPU_UNION,   // union of those intervals (device busy time), us*1000
    QT_N
};
inline int64_t qt_now() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}
#endif

// One device's part of a queue: its lanes, staging slots, streams and threads.  A queue
// (zs3_queue, below) holds one per listed device and assigns every submitted block to
// one of them (zs3q::pick_device); each device batches its own blocks.
struct DevQ {
    const zs3_codec* c = nullptr;
    int k = 0, m = 0, R = 0;
    int64_t B = 0, S = 0, E = 0;  // block size, full shard size, bytes per position
    int device = 0;
    int cap = 64;                 // positions per slot = the largest batch (zs3q::slot_blocks)
    int max_wait_us = 200;
    int nslots = 4;
    // Pinned callers (round 4; ZS3_QUEUE_ZC=<mode> selects another for A/B measurements,
    // profiles/r04/queue_ab*.jsonl):
    //   0 staged like pageable callers (memcpy into the pinned slot, one DMA per batch);
    //   1 (default) zero-copy only for a lone caller: the first block of a batch while no
    //     other batch of its lane is in flight is DMA'd by its submitter (the slot is still
    //     empty), everything else staged — under concurrency the extra per-batch DMA call
    //     cost more than the memcpy it saves (16 submitters 18-20 vs 20-22 GiB/s,
    //     profiles/r04/queue_ab4.jsonl);
    //   2 every block zero-copy by a DMA of its own (round 3): the per-block DMA calls of
    //     many submitters serialise in the runtime (256 submitters 26.3 vs staged 32.8
    //     GiB/s);
    //   3 zero-copy by one copy-list kernel per batch and direction over the mapped
    //     pinned pages: GPU-initiated PCIe reads are slower than the DMA engine (256
    //     submitters 16.6 GiB/s).
    int zc_mode = 1;
    // Copy streams (round 6).  1 (default): every lane has one H2D and one D2H stream
    // shared by its slots, the slot's own stream runs only the kernels (events chain the
    // three), so one batch's D2H runs beside the next one's H2D on the other DMA
    // direction; 0: each slot's stream carries its H2D, kernels and D2H in order
    // (rounds 2-5).  tools/queue_bench_diag, profiles/r06/queue_split.jsonl.
    int split = 1;
    hipStream_t s_in[NLANE] = {nullptr, nullptr, nullptr};
    hipStream_t s_out[NLANE] = {nullptr, nullptr, nullptr};

    std::mutex mu;
    std::condition_variable cv_space;   // a slot became free / open
    std::condition_variable cv_disp;    // dispatcher: new work, copies finished, flush, stop
    std::condition_variable cv_done;    // a slot finished
    std::condition_variable cv_comp;    // completer: a slot was launched
    std::vector<Slot> slots[NLANE];
    enum { LANE_NONE, LANE_INIT, LANE_READY };
    int lane_state[NLANE] = {LANE_NONE, LANE_NONE, LANE_NONE};
    Slot* open[NLANE] = {nullptr, nullptr, nullptr};
    int inflight[NLANE] = {0, 0, 0};
    int inflight_blocks[NLANE] = {0, 0, 0};  // blocks of the launched, unfinished slots
    std::vector<Slot*> sealed[NLANE];         // closed to new blocks, waiting for copiers
    // Seal point (ready_to_close): the open slot closes at pipe_pct % of the live blocks.
    // Round 6 (profiles/r06/queue_pipe.jsonl, queue_pipe_live.jsonl, split copy streams):
    // 33 % keeps three batches in flight (64 submitters 34.6-35.9 -> 37.8-39.4 GiB/s), and
    // the live count includes submitters parked on backpressure (pipe_live 1) — counting
    // only the open + launched blocks shrinks the seal point whenever every slot is busy,
    // down to 8-block batches at 25 % (256 submitters 10-11 GiB/s).  Diagnostics build:
    // ZS3_QUEUE_PIPE_PCT, ZS3_QUEUE_PIPE_LIVE (0 = rounds 4-5).
    int pipe_pct = 33;
    int pipe_live = 1;
    std::atomic<int> live[NLANE]{};           // blocks assigned to this device, not yet finished
    std::deque<Slot*> launched;
    bool flush = false;
    bool stop = false;       // dispatcher: drain the open slots and exit
    bool comp_stop = false;  // completer: exit once every launched slot is done
    std::thread disp, comp;
    std::atomic<int64_t> n_batches{0}, n_blocks{0}, n_zc{0};
#if ZS3_DIAG
    // Host-side phase timers (zs3_debug_queue_timers, tools/queue_bench_diag): thread-ns
    // summed over the threads that spent them, and the device's busy time (the union of
    // the launched batches' stream intervals, from timing events).
    std::atomic<int64_t> tm[QT_N] = {};
    hipEvent_t ref_ev = nullptr;  // time origin of the stream intervals
    double last_end_ms = -1.0;    // completer: end of the union so far
#endif

    // region offsets inside a slot (bytes).  ENCODE: [cap][k*S] data rows, then
    // [cap][m*S] parity rows (each direction one contiguous DMA copy of the bytes that
    // cross PCIe); GET / HEAL: [cap][(k+m)*S] stripes
    size_t off_par() const { return (size_t)cap * k * S; }                     // ENCODE parity rows
    size_t off_sums() const { return (size_t)cap * E; }                       // [cap][R][32] sums / expect
    size_t off_bad() const { return off_sums() + (size_t)cap * R * 32; }      // [cap][R] int32
    size_t off_out() const { return off_bad() + (size_t)cap * R * 4; }        // [cap][R][32] heal sums
    size_t slot_bytes(int lane) const {
        return lane == ENC ? off_bad() : lane == GET ? off_out() : off_out() + (size_t)cap * R * 32;
    }
};

namespace {

int map_hip(hipError_t e) { return e == hipSuccess ? ZS3_OK : (e == hipErrorOutOfMemory ? ZS3_ERR_NOMEM : ZS3_ERR_DEVICE); }

// Allocate a lane's slots on first use (runs on a submitter; lk is held on entry and
// on return, but the allocation itself runs unlocked so the dispatcher and completer
// keep serving the other lanes; other submitters of this lane wait for it).  A failed
// allocation leaves the lane unallocated, so a later submit retries.
int ensure_lane(DevQ* q, std::unique_lock<std::mutex>& lk, int lane) {
    for (;;) {
        if (q->lane_state[lane] == DevQ::LANE_READY) return ZS3_OK;
        if (q->lane_state[lane] == DevQ::LANE_NONE) break;
        q->cv_space.wait(lk);
    }
    q->lane_state[lane] = DevQ::LANE_INIT;
    const size_t bytes = q->slot_bytes(lane);
    const int nslots = q->nslots, cap = q->cap, device = q->device;
    lk.unlock();
    int prev = 0;
    (void)hipGetDevice(&prev);
    std::vector<Slot> v((size_t)nslots);
    int rc = map_hip(hipSetDevice(device));
    hipStream_t si = nullptr, so = nullptr;
    if (q->split && rc == ZS3_OK) rc = map_hip(hipStreamCreateWithFlags(&si, hipStreamNonBlocking));
    if (q->split && rc == ZS3_OK) rc = map_hip(hipStreamCreateWithFlags(&so, hipStreamNonBlocking));
    for (auto& s : v) {
        s.lane = lane;
        if (rc == ZS3_OK) rc = map_hip(hipHostMalloc((void**)&s.h, bytes, hipHostMallocDefault));
        if (rc == ZS3_OK) rc = map_hip(hipMalloc((void**)&s.d, bytes));
#if ZS3_DIAG
        if (rc == ZS3_OK) rc = map_hip(hipEventCreate(&s.done_ev));  // timed: the device busy time
        if (rc == ZS3_OK) rc = map_hip(hipEventCreate(&s.start_ev));
#else
        if (rc == ZS3_OK) rc = map_hip(hipEventCreateWithFlags(&s.done_ev, hipEventDisableTiming));
#endif
        if (rc == ZS3_OK) rc = map_hip(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
        if (q->split && rc == ZS3_OK) rc = map_hip(hipEventCreateWithFlags(&s.ev_in, hipEventDisableTiming));
        if (q->split && rc == ZS3_OK) rc = map_hip(hipEventCreateWithFlags(&s.ev_comp, hipEventDisableTiming));
        s.claimed.reset(new std::atomic<uint8_t>[(size_t)cap]);
    }
    if (rc != ZS3_OK) {
        for (auto& s : v) {
            if (s.h) (void)hipHostFree(s.h);
            if (s.d) (void)hipFree(s.d);
            if (s.done_ev) (void)hipEventDestroy(s.done_ev);
            if (s.start_ev) (void)hipEventDestroy(s.start_ev);
            if (s.stream) (void)hipStreamDestroy(s.stream);
            if (s.ev_in) (void)hipEventDestroy(s.ev_in);
            if (s.ev_comp) (void)hipEventDestroy(s.ev_comp);
        }
        if (si) (void)hipStreamDestroy(si);
        if (so) (void)hipStreamDestroy(so);
    }
    (void)hipSetDevice(prev);
    lk.lock();
    if (rc == ZS3_OK) {
        q->slots[lane] = std::move(v);
        q->s_in[lane] = si;
        q->s_out[lane] = so;
    }
    q->lane_state[lane] = rc == ZS3_OK ? DevQ::LANE_READY : DevQ::LANE_NONE;
    q->cv_space.notify_all();
    return rc;
}

// ---- zero-copy transport: a copy-list kernel ---------------------------------------
// Up to CL_MAX (src, dst, len) entries per launch, passed by value (kernel arguments);
// grid.y = entry, grid.x strides the entry's bytes in W-byte words (W = the widest
// alignment every entry allows).  Reads of the callers' mapped pinned pages and writes
// to them cross PCIe as the GPU's own requests: one launch per batch and direction
// instead of one DMA call per block (64 submitters each calling hipMemcpyAsync on the
// slot's stream serialised in the runtime: pinned 17.7 vs pageable 20.8 GiB/s,
// profiles/r03/queue_native_zero_copy_first.jsonl).
constexpr int CL_MAX = 80;
struct CopyList {
    const uint8_t* src[CL_MAX];
    uint8_t* dst[CL_MAX];
    int64_t len[CL_MAX];
    int n;
};

template <typename W>
__global__ void __launch_bounds__(256) k_copy_list(CopyList L) {
    const int e = blockIdx.y;
    const W* src = reinterpret_cast<const W*>(L.src[e]);
    W* dst = reinterpret_cast<W*>(L.dst[e]);
    const int64_t nw = L.len[e] / (int64_t)sizeof(W);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nw; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x < (int)(L.len[e] % (int64_t)sizeof(W))) {
        const int64_t b = nw * (int64_t)sizeof(W) + threadIdx.x;
        L.dst[e][b] = L.src[e][b];
    }
    __threadfence_system();  // host-visible before the batch's completion event
}

struct CopyEntry {
    const uint8_t* src;
    uint8_t* dst;
    int64_t len;
};

int run_copy_list(const std::vector<CopyEntry>& v, hipStream_t st) {
    for (size_t i0 = 0; i0 < v.size(); i0 += CL_MAX) {
        CopyList L{};
        L.n = (int)std::min<size_t>(CL_MAX, v.size() - i0);
        uintptr_t al = 0;
        int64_t mx = 0;
        for (int j = 0; j < L.n; ++j) {
            const CopyEntry& c = v[i0 + (size_t)j];
            L.src[j] = c.src;
            L.dst[j] = c.dst;
            L.len[j] = c.len;
            al |= (uintptr_t)c.src | (uintptr_t)c.dst;
            mx = std::max(mx, c.len);
        }
        const int w = (al & 15) == 0 ? 16 : (al & 7) == 0 ? 8 : (al & 3) == 0 ? 4 : 1;
        const int64_t words = mx / w;
        const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(64, (words + 1023) / 1024));
        const dim3 grid(gx, (unsigned)L.n);
        if (w == 16)
            hipLaunchKernelGGL(k_copy_list<uint4>, grid, dim3(256), 0, st, L);
        else if (w == 8)
            hipLaunchKernelGGL(k_copy_list<uint2>, grid, dim3(256), 0, st, L);
        else if (w == 4)
            hipLaunchKernelGGL(k_copy_list<uint32_t>, grid, dim3(256), 0, st, L);
        else
            hipLaunchKernelGGL(k_copy_list<uint8_t>, grid, dim3(256), 0, st, L);
        if (hipGetLastError() != hipSuccess) return ZS3_ERR_DEVICE;
    }
    return ZS3_OK;
}

// Calls f(a, b) for every maximal run [a, b) of positions < n with skip[pos] == 0.
template <class F>
void for_runs(const std::vector<uint8_t>& skip, int n, F f) {
    for (int i = 0; i < n;) {
        if (skip[(size_t)i]) {
            ++i;
            continue;
        }
        int j = i;
        while (j < n && !skip[(size_t)j]) ++j;
        f(i, j);
        i = j;
    }
}

int pipe_size(const DevQ* q, const Slot* s, int lane);

// Reserve a position for one block in the lane's open slot (caller holds lk).
int reserve(DevQ* q, std::unique_lock<std::mutex>& lk, zs3_req* r, bool full) {
    int rc = ensure_lane(q, lk, r->lane);
    if (rc) return rc;
    for (;;) {
        if (q->stop) return ZS3_ERR_INVALID_ARG;
        Slot* s = q->open[r->lane];
        if (s && s->front + s->back < q->cap) {
            r->slot = s;
            r->pos = full ? s->front++ : q->cap - 1 - s->back++;
            s->copying++;
            s->reqs.push_back(r);
            if (s->front + s->back == q->cap || s->front + s->back >= pipe_size(q, s, r->lane)) {
                // sealed: later submitters open the next slot at once instead of growing this
                // one while its copiers are still busy (the dispatcher launches it when the
                // last copier is done)
                q->sealed[r->lane].push_back(s);
                q->open[r->lane] = nullptr;
                q->cv_disp.notify_one();
            }
            return ZS3_OK;
        }
        if (!s) {
            for (auto& x : q->slots[r->lane])
                if (x.state == Slot::FREE) {
                    x.state = Slot::OPEN;
                    x.front = x.back = x.copying = 0;
                    x.reqs.clear();
                    x.launch_status = ZS3_OK;
                    x.ready = false;
                    x.opened = Clock::now();
                    q->open[r->lane] = &x;
                    break;
                }
            if (q->open[r->lane]) continue;
        }
        q->cv_space.wait(lk);  // every slot busy (or the open one full): backpressure
    }
}

void copy_in_done(DevQ* q, Slot* s) {
    std::lock_guard<std::mutex> g(q->mu);
    if (--s->copying == 0) q->cv_disp.notify_one();
}

// ---- launch of a closed slot (dispatcher thread, no lock held) ----------------------
// Three phases: every H2D copy of the batch (stream si), its kernels (the slot's stream
// sc), every D2H copy (so); with split streams events hand the batch from one to the
// next, otherwise all three are the slot's stream.
void launch_slot(DevQ* q, Slot* s) {
    const hipStream_t sc = s->stream;
    const hipStream_t si = q->split ? q->s_in[s->lane] : sc, so = q->split ? q->s_out[s->lane] : sc;
    const int k = q->k, m = q->m, R = q->R;
    const int64_t E = q->E, S = q->S;
    const int nf = s->front;
    int rc = ZS3_OK;
    auto chk = [&](int e) {
        if (e != ZS3_OK && rc == ZS3_OK) rc = e;
    };
    auto hand = [&](hipStream_t from, hipEvent_t ev, hipStream_t to) {
        if (from == to) return;
        chk(map_hip(hipEventRecord(ev, from)));
        chk(map_hip(hipStreamWaitEvent(to, ev, 0)));
    };
    uint8_t* dsum = s->d + q->off_sums();
    uint8_t* hsum = s->h + q->off_sums();
#if ZS3_DIAG
    if (s->start_ev) chk(map_hip(hipEventRecord(s->start_ev, si)));
#endif
    if (s->lane == ENC) {
        // full-size blocks: data rows in, one fused launch, parity rows + sums out;
        // staged blocks move by one DMA per run of staged positions each way; zero-copy
        // blocks were copied in by their submitter (on sc) and get their parity rows
        // straight back into the caller's buffer.  Short blocks: one launch each.
        const size_t KS = (size_t)k * S, MS = (size_t)m * S, po = q->off_par();
        std::vector<uint8_t> zc((size_t)nf, 0);
        std::vector<CopyEntry> gin, gout;
        for (zs3_req* r : s->reqs)
            if (r->pos < nf && r->zc) {
                zc[(size_t)r->pos] = 1;
                if (r->d_map) {
                    gin.push_back({r->d_map, s->d + r->pos * KS, r->len});
                    gout.push_back({s->d + po + r->pos * MS, r->d_map + KS, (int64_t)MS});
                }
            }
        for_runs(zc, nf, [&](int a, int b) {
            chk(map_hip(hipMemcpyAsync(s->d + a * KS, s->h + a * KS, (size_t)(b - a) * KS, hipMemcpyHostToDevice, si)));
        });
        for (zs3_req* r : s->reqs)
            if (r->pos >= nf) {
                const size_t o = (size_t)r->pos * KS;
                chk(map_hip(hipMemcpyAsync(s->d + o, s->h + o, (size_t)(k * r->S), hipMemcpyHostToDevice, si)));
            }
        hand(si, s->ev_in, sc);
        if (!gin.empty()) chk(run_copy_list(gin, sc));
        if (nf > 0) chk(zs3_encode_batch(q->c, s->d, (int64_t)KS, q->B, nf, s->d + po, (int64_t)MS, dsum, sc));
        for (zs3_req* r : s->reqs)
            if (r->pos >= nf) {
                const size_t o = (size_t)r->pos * KS, op = po + (size_t)r->pos * MS;
                chk(zs3_encode_batch(q->c, s->d + o, (int64_t)KS, r->len, 1, s->d + op, (int64_t)MS,
                                     dsum + (size_t)r->pos * R * 32, sc));
            }
        if (!gout.empty()) chk(run_copy_list(gout, sc));
        hand(sc, s->ev_comp, so);
        for_runs(zc, nf, [&](int a, int b) {
            chk(map_hip(hipMemcpyAsync(s->h + po + a * MS, s->d + po + a * MS, (size_t)(b - a) * MS,
                                       hipMemcpyDeviceToHost, so)));
        });
        for (zs3_req* r : s->reqs)
            if (r->pos < nf && r->zc && !r->d_map)
                chk(map_hip(hipMemcpyAsync(r->h_buf + KS, s->d + po + r->pos * MS, MS, hipMemcpyDeviceToHost, so)));
        if (nf > 0) chk(map_hip(hipMemcpyAsync(hsum, dsum, (size_t)nf * R * 32, hipMemcpyDeviceToHost, so)));
        for (zs3_req* r : s->reqs)
            if (r->pos >= nf) {
                const size_t op = po + (size_t)r->pos * MS, so_ = (size_t)r->pos * R * 32;
                chk(map_hip(hipMemcpyAsync(s->h + op, s->d + op, (size_t)(m * r->S), hipMemcpyDeviceToHost, so)));
                chk(map_hip(hipMemcpyAsync(hsum + so_, dsum + so_, (size_t)R * 32, hipMemcpyDeviceToHost, so)));
            }
    } else {
        const int data_only = s->lane == GET ? 1 : 0;
        int32_t* dbad = (int32_t*)(s->d + q->off_bad());
        uint8_t* hbad = s->h + q->off_bad();
        uint8_t* dout = s->lane == HEAL ? s->d + q->off_out() : nullptr;
        uint8_t* hout = s->h + q->off_out();
        std::vector<uint8_t> zc((size_t)nf, 0);
        std::vector<CopyEntry> gin;
        for (zs3_req* r : s->reqs)
            if (r->pos < nf && r->zc) {
                zc[(size_t)r->pos] = 1;
                if (r->d_map) {
                    // the survivors, one entry per run of present rows
                    std::vector<uint8_t> absent((size_t)R);
                    for (int i = 0; i < R; ++i) absent[(size_t)i] = !r->present[i];
                    for_runs(absent, R, [&](int a, int b) {
                        gin.push_back({r->d_map + (size_t)a * S, s->d + (size_t)r->pos * E + (size_t)a * S,
                                       (int64_t)(b - a) * S});
                    });
                }
            }
        for_runs(zc, nf, [&](int a, int b) {
            chk(map_hip(hipMemcpyAsync(s->d + (size_t)a * E, s->h + (size_t)a * E, (size_t)(b - a) * E,
                                       hipMemcpyHostToDevice, si)));
        });
        if (nf > 0) chk(map_hip(hipMemcpyAsync(dsum, hsum, (size_t)nf * R * 32, hipMemcpyHostToDevice, si)));
        for (zs3_req* r : s->reqs)
            if (r->pos >= nf) {
                const size_t o = (size_t)r->pos * E, so_ = (size_t)r->pos * R * 32;
                chk(map_hip(hipMemcpyAsync(s->d + o, s->h + o, (size_t)(R * r->S), hipMemcpyHostToDevice, si)));
                chk(map_hip(hipMemcpyAsync(dsum + so_, hsum + so_, (size_t)R * 32, hipMemcpyHostToDevice, si)));
            }
        hand(si, s->ev_in, sc);
        if (nf > 0) {
            if (!gin.empty()) chk(run_copy_list(gin, sc));
            std::vector<uint8_t> pres((size_t)nf * R, 0);
            std::vector<int32_t> status((size_t)nf, ZS3_OK);
            for (zs3_req* r : s->reqs)
                if (r->pos < nf) std::memcpy(&pres[(size_t)r->pos * R], r->present, (size_t)R);
            const int e = zs3_verify_reconstruct_batch_masks(q->c, s->d, E, S, nf, pres.data(), data_only, dsum, dbad,
                                                             dout, status.data(), sc);
            if (e != ZS3_OK && e != ZS3_ERR_TOO_FEW_SHARDS && e != ZS3_ERR_SHARD_NO_DATA) chk(e);
            for (zs3_req* r : s->reqs)
                if (r->pos < nf) r->status = status[(size_t)r->pos];
        }
        for (zs3_req* r : s->reqs) {
            if (r->pos < nf) continue;
            const size_t o = (size_t)r->pos * E;
            const size_t so_ = (size_t)r->pos * R * 32, bo = (size_t)r->pos * R * 4;
            int32_t one = ZS3_OK;
            const int e = zs3_verify_reconstruct_batch_masks(q->c, s->d + o, E, r->S, 1, r->present, data_only,
                                                             dsum + so_, (int32_t*)((uint8_t*)dbad + bo),
                                                             dout ? dout + so_ : nullptr, &one, sc);
            if (e != ZS3_OK && e != ZS3_ERR_TOO_FEW_SHARDS && e != ZS3_ERR_SHARD_NO_DATA) chk(e);
            r->status = one;
        }
        // rebuilt rows to zero-copy callers in copy-list mode: one launch for the batch
        std::vector<CopyEntry> gout;
        for (zs3_req* r : s->reqs) {
            if (r->status != ZS3_OK || !r->zc || !r->d_map) continue;
            const size_t o = (size_t)r->pos * E;
            for (int i = 0; i < R; ++i)
                if (!r->present[i] && (i < k || !data_only))
                    gout.push_back({s->d + o + (size_t)i * r->S, r->d_map + (size_t)i * r->S, r->S});
        }
        if (!gout.empty()) chk(run_copy_list(gout, sc));
        hand(sc, s->ev_comp, so);
        if (nf > 0) {
            chk(map_hip(hipMemcpyAsync(hbad, dbad, (size_t)nf * R * 4, hipMemcpyDeviceToHost, so)));
            if (dout) chk(map_hip(hipMemcpyAsync(hout, dout, (size_t)nf * R * 32, hipMemcpyDeviceToHost, so)));
        }
        for (zs3_req* r : s->reqs) {
            if (r->pos < nf) continue;
            const size_t so_ = (size_t)r->pos * R * 32, bo = (size_t)r->pos * R * 4;
            chk(map_hip(hipMemcpyAsync(hbad + bo, (uint8_t*)dbad + bo, (size_t)R * 4, hipMemcpyDeviceToHost, so)));
            if (dout) chk(map_hip(hipMemcpyAsync(hout + so_, dout + so_, (size_t)R * 32, hipMemcpyDeviceToHost, so)));
        }
        // rebuilt rows back to the pinned slot (only those, per block), or straight into
        // a zero-copy caller's shard rows
        for (zs3_req* r : s->reqs) {
            if (r->status != ZS3_OK || (r->zc && r->d_map)) continue;
            const size_t o = (size_t)r->pos * E;
            uint8_t* hdst = r->zc ? r->h_shards : s->h + o;
            for (int i = 0; i < R; ++i)
                if (!r->present[i] && (i < k || !data_only))
                    chk(map_hip(hipMemcpyAsync(hdst + (size_t)i * r->S, s->d + o + (size_t)i * r->S, (size_t)r->S,
                                               hipMemcpyDeviceToHost, so)));
        }
    }
    chk(map_hip(hipEventRecord(s->done_ev, so)));
    s->launch_status = rc;
    q->n_batches.fetch_add(1);
    q->n_blocks.fetch_add((int64_t)s->reqs.size());
}

// Blocks at which the open slot closes for pipelining (ready_to_close); caller holds mu.
int pipe_size(const DevQ* q, const Slot* s, int lane) {
    int live = (int)s->reqs.size() + q->inflight_blocks[lane];
    if (q->pipe_live) live = std::max(live, q->live[lane].load(std::memory_order_relaxed));
    return zs3q::seal_blocks(live, q->pipe_pct, q->cap);
}

bool ready_to_close(DevQ* q, Slot* s, int lane, Clock::time_point now) {
    if (s->reqs.empty()) return false;
    if (s->front + s->back == q->cap || q->flush || q->stop) return true;
    // Pipelining cap (round 4): T synchronous submitters keep about T blocks live (open
    // slot + in flight); closing the slot at half of them keeps two batches alternating,
    // one's H2D under the other's kernel and D2H, instead of one batch of all of them
    // (1 MiB RS(8+4), 64 submitters: 29.9-30.5 GiB/s at batches of 32 vs 21-24 at 64-128;
    // 256 submitters: 33-35 at 64; profiles/r04/queue_ab3.jsonl), at most the slot's
    // size (zs3q::slot_blocks: 64 MiB of input); since round 6 at a third of them
    // (DevQ::pipe_pct), three batches in flight on the split copy streams
    if (s->front + s->back >= pipe_size(q, s, lane)) return true;
    // batch while busy: launch at once while fewer than slots-1 batches are in flight
    // (a small batch is bound by one hash chain's latency, ~0.5 ms for 128 KiB shards,
    // not by its bytes, so concurrent batches on their own streams overlap almost
    // fully); otherwise let the open slot grow until one completes
    if (q->inflight[lane] < q->nslots - 1) return true;
    return now - s->opened >= std::chrono::microseconds(q->max_wait_us);
}

void dispatcher(DevQ* q) {
    (void)hipSetDevice(q->device);
    std::unique_lock<std::mutex> lk(q->mu);
    for (;;) {
        bool launched_any = false;
        auto now = Clock::now();
        Clock::time_point wake = now + std::chrono::milliseconds(50);
        auto launch = [&](Slot* s, int lane) {
            s->state = Slot::LAUNCHED;
            q->inflight[lane]++;
            s->nblocks = (int)s->reqs.size();
            q->inflight_blocks[lane] += s->nblocks;
            q->cv_space.notify_all();  // submitters may open the next slot
            lk.unlock();
#if ZS3_DIAG
            const int64_t t0 = qt_now();
            launch_slot(q, s);
            q->tm[QT_DISP_LAUNCH] += qt_now() - t0;
#else
            launch_slot(q, s);
#endif
            lk.lock();
            q->launched.push_back(s);
            q->cv_comp.notify_one();
            launched_any = true;
        };
        for (int lane = 0; lane < NLANE; ++lane) {
            // sealed slots whose copiers are done, oldest first
            for (size_t i = 0; i < q->sealed[lane].size();) {
                Slot* s = q->sealed[lane][i];
                if (s->copying > 0) {
                    ++i;
                    continue;
                }
                q->sealed[lane].erase(q->sealed[lane].begin() + (std::ptrdiff_t)i);
                launch(s, lane);
                i = 0;  // the list may have changed while unlocked
            }
            Slot* s = q->open[lane];
            if (!s) continue;
            if (!ready_to_close(q, s, lane, now)) {
                if (!s->reqs.empty()) {
                    auto t = s->opened + std::chrono::microseconds(q->max_wait_us);
                    if (t < wake) wake = t;
                }
                continue;
            }
            if (s->copying > 0) continue;  // the last copier notifies
            q->open[lane] = nullptr;
            launch(s, lane);
        }
        bool pending = false;
        for (int lane = 0; lane < NLANE; ++lane)
            pending |= (q->open[lane] && !q->open[lane]->reqs.empty()) || !q->sealed[lane].empty();
        if (!pending) q->flush = false;
        if (q->stop && !pending) break;
        if (!launched_any) q->cv_disp.wait_until(lk, wake);
    }
}

// Copy one finished block's results from the pinned slot into its caller's buffers.
void finish_req(DevQ* q, Slot* s, zs3_req* r) {
#if ZS3_DIAG
    const int64_t t0 = qt_now();
    struct Acc {
        DevQ* q;
        int64_t t0;
        ~Acc() { q->tm[QT_COPY_OUT] += qt_now() - t0; }
    } acc{q, t0};
#endif
    int64_t rc = s->launch_status != ZS3_OK ? s->launch_status : r->status;
    const size_t o = (size_t)r->pos * q->E;
    const int k = q->k, R = q->R;
    if (rc == ZS3_OK) {
        if (r->lane == ENC) {
            if (!r->zc)
                std::memcpy(r->h_buf + (size_t)k * r->S, s->h + q->off_par() + (size_t)r->pos * q->m * q->S,
                            (size_t)(q->m * r->S));
            if (k * r->S > r->len)
                std::memset(r->h_buf + r->len, 0, (size_t)(k * r->S - r->len));  // Split zero-fill in place
            if (r->h_sums) std::memcpy(r->h_sums, s->h + q->off_sums() + (size_t)r->pos * R * 32, (size_t)R * 32);
            rc = r->S;
        } else {
            const int data_only = r->lane == GET;
            for (int i = 0; i < R && !r->zc; ++i)
                if (!r->present[i] && (i < k || !data_only))
                    std::memcpy(r->h_shards + (size_t)i * r->S, s->h + o + (size_t)i * r->S, (size_t)r->S);
            const int32_t* bad = (const int32_t*)(s->h + q->off_bad()) + (size_t)r->pos * R;
            bool corrupt = false;
            for (int i = 0; i < R; ++i) corrupt |= r->h_expect && bad[i];
            if (r->h_bad)
                for (int i = 0; i < R; ++i) r->h_bad[i] = r->h_expect ? bad[i] : 0;
            if (r->h_sums_out && r->lane == HEAL)
                std::memcpy(r->h_sums_out, s->h + q->off_out() + (size_t)r->pos * R * 32, (size_t)R * 32);
            if (corrupt) rc = ZS3_ERR_FILE_CORRUPT;
        }
    }
    r->result = rc;
    q->live[r->lane].fetch_sub(1, std::memory_order_relaxed);
}

// Drop one pending block of the slot; the last one frees the slot (caller holds no lock).
void finish_one(DevQ* q, Slot* s) {
    if (s->pending.fetch_sub(1) != 1) return;
    std::lock_guard<std::mutex> g(q->mu);
    s->reqs.clear();
    s->state = Slot::FREE;
    q->inflight[s->lane]--;
    q->inflight_blocks[s->lane] -= s->nblocks;
    q->cv_space.notify_all();
    q->cv_disp.notify_one();  // batch-while-busy: the next open slot may go now
}

void completer(DevQ* q) {
    std::unique_lock<std::mutex> lk(q->mu);
    for (;;) {
        q->cv_comp.wait(lk, [&] { return !q->launched.empty() || q->comp_stop; });
        if (q->launched.empty()) break;
        Slot* s = q->launched.front();
        q->launched.pop_front();
        lk.unlock();
#if ZS3_DIAG
        const int64_t tc0 = qt_now();
#endif
        if (hipEventSynchronize(s->done_ev) != hipSuccess && s->launch_status == ZS3_OK)
            s->launch_status = ZS3_ERR_DEVICE;
#if ZS3_DIAG
        q->tm[QT_COMP_SYNC] += qt_now() - tc0;
        float a_ms = 0.f, b_ms = 0.f;
        if (q->ref_ev && hipEventElapsedTime(&a_ms, q->ref_ev, s->start_ev) == hipSuccess &&
            hipEventElapsedTime(&b_ms, q->ref_ev, s->done_ev) == hipSuccess && b_ms >= a_ms) {
            q->tm[QT_GPU_SUM] += (int64_t)((b_ms - a_ms) * 1e6);
            const double from = std::max<double>(a_ms, q->last_end_ms);
            if (b_ms > from) q->tm[QT_GPU_UNION] += (int64_t)((b_ms - from) * 1e6);
            q->last_end_ms = std::max<double>(q->last_end_ms, b_ms);
        } else {
            (void)hipGetLastError();
        }
#endif
        const size_t n = s->reqs.size();
        std::vector<int> pos(n);  // read before any waiter can finish (and delete) its request
        for (size_t i = 0; i < n; ++i) pos[i] = s->reqs[i]->pos;
        for (size_t i = 0; i < (size_t)q->cap; ++i) s->claimed[i].store(0, std::memory_order_relaxed);
        s->pending.store((int)n + 1);  // + 1: this thread's scan below
        lk.lock();
        s->ready = true;
        q->cv_done.notify_all();  // waiters claim and copy out their own blocks
        lk.unlock();
        // copy out the blocks nobody claimed (un-waited async requests); a claimed
        // request is never touched again here (its waiter may delete it)
        std::vector<zs3_req*> mine;
        for (size_t i = 0; i < n; ++i) {
            if (s->claimed[pos[i]].exchange(1)) continue;
            zs3_req* r = s->reqs[i];
            finish_req(q, s, r);
            mine.push_back(r);
        }
        lk.lock();
        for (zs3_req* r : mine) r->done = true;
        if (!mine.empty()) q->cv_done.notify_all();
        lk.unlock();
        for (size_t i = 0; i < mine.size(); ++i) finish_one(q, s);
        finish_one(q, s);  // the scan itself
        lk.lock();
    }
}

// One device's queue part: validated codec parameters, its own threads; the slots of a
// lane are allocated on the lane's first submit (ensure_lane).
int devq_new(const zs3_codec* c, int device, const zs3_queue_opts* opts, DevQ** out) {
    *out = nullptr;
    auto* q = new DevQ();
    q->c = c;
    if (zs3_codec_params(c, &q->k, &q->m, &q->B) != ZS3_OK) {
        delete q;
        return ZS3_ERR_INVALID_ARG;
    }
    q->R = q->k + q->m;
    q->S = zs3_shard_size(c);
    q->E = (int64_t)q->R * q->S;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    q->device = device;
    if (opts) {
        if (opts->max_wait_us > 0) q->max_wait_us = opts->max_wait_us;
        if (opts->slots > 0) q->nslots = opts->slots;
    }
    if (q->nslots < 2) q->nslots = 2;
    q->cap = zs3q::slot_blocks(opts ? opts->max_batch : 0, q->B);
#if ZS3_DIAG
    // A/B switches of the diagnostics build only (a stray variable never changes a
    // production server's transport: ADVICE r04)
    if (const char* e = std::getenv("ZS3_QUEUE_ZC")) q->zc_mode = std::max(0, std::min(3, std::atoi(e)));
    if (const char* e = std::getenv("ZS3_QUEUE_PIPE_PCT")) q->pipe_pct = std::max(10, std::min(100, std::atoi(e)));
    if (const char* e = std::getenv("ZS3_QUEUE_PIPE_LIVE")) q->pipe_live = std::atoi(e) ? 1 : 0;
    if (const char* e = std::getenv("ZS3_QUEUE_SPLIT")) q->split = std::atoi(e) ? 1 : 0;
#endif
    int prev = dev;
    if (hipSetDevice(q->device) != hipSuccess) {
        delete q;
        return ZS3_ERR_DEVICE;
    }
#if ZS3_DIAG
    if (hipEventCreate(&q->ref_ev) != hipSuccess || hipEventRecord(q->ref_ev, nullptr) != hipSuccess) {
        (void)hipGetLastError();
        q->ref_ev = nullptr;
    }
#endif
    (void)hipSetDevice(prev);
    q->disp = std::thread(dispatcher, q);
    q->comp = std::thread(completer, q);
    *out = q;
    return ZS3_OK;
}

void devq_free(DevQ* q) {
    if (!q) return;
    {
        std::lock_guard<std::mutex> g(q->mu);
        q->stop = true;
        q->cv_disp.notify_all();
        q->cv_space.notify_all();
    }
    q->disp.join();
    {
        std::lock_guard<std::mutex> g(q->mu);
        q->comp_stop = true;
        q->cv_comp.notify_all();
    }
    q->comp.join();
    for (auto& v : q->slots)
        for (auto& s : v) {
            if (s.h) (void)hipHostFree(s.h);
            if (s.d) (void)hipFree(s.d);
            if (s.done_ev) (void)hipEventDestroy(s.done_ev);
            if (s.start_ev) (void)hipEventDestroy(s.start_ev);
            if (s.stream) (void)hipStreamDestroy(s.stream);
            if (s.ev_in) (void)hipEventDestroy(s.ev_in);
            if (s.ev_comp) (void)hipEventDestroy(s.ev_comp);
        }
    for (int lane = 0; lane < NLANE; ++lane) {
        if (q->s_in[lane]) (void)hipStreamDestroy(q->s_in[lane]);
        if (q->s_out[lane]) (void)hipStreamDestroy(q->s_out[lane]);
    }
#if ZS3_DIAG
    if (q->ref_ev) (void)hipEventDestroy(q->ref_ev);
#endif
    delete q;
}

// Submits on one device (the caller validated the arguments and counted the block in
// q->live[lane]; a failed reserve uncounts it).
int devq_submit_encode(DevQ* q, uint8_t* h_buf, int64_t len, uint8_t* h_sums, zs3_req** req) {
    const int64_t Sb = (len + q->k - 1) / q->k;
    auto* r = new zs3_req();
    r->q = q;
    r->lane = ENC;
    r->S = Sb;
    r->h_buf = h_buf;
    r->len = len;
    r->h_sums = h_sums;
    Slot* s;
    bool lone = false;  // no other batch of the lane in flight (zc_mode 1)
#if ZS3_DIAG
    const int64_t t0 = qt_now();
#endif
    {
        std::unique_lock<std::mutex> lk(q->mu);
        const int rc = reserve(q, lk, r, len == q->B);
        if (rc) {
            q->live[ENC].fetch_sub(1, std::memory_order_relaxed);
            delete r;
            return rc;
        }
        s = r->slot;
        lone = q->inflight_blocks[ENC] == 0;
    }
#if ZS3_DIAG
    const int64_t t1 = qt_now();
    q->tm[QT_SUB_LOCK] += t1 - t0;
#endif
    // Split (reedsolomon): data rows are the input bytes, zero-padded to k*S (the
    // kernel reads the pad of a full block as zero).  A full block in pinned memory is
    // DMA'd from the caller's buffer on the slot's stream, ahead of the batch's launch.
    // Copy-list mode: the batch's launch moves it (run_copy_list).
    const size_t KS = (size_t)q->k * q->S;
    void* dmap = nullptr;
    const bool zc_try = q->zc_mode == 2 || q->zc_mode == 3 || (q->zc_mode == 1 && r->pos == 0 && lone);
    if (len == q->B && zc_try && zs3i_pinned_map(h_buf, (size_t)q->R * q->S, &dmap)) {
        if (q->zc_mode == 3) {
            r->zc = true;
            r->d_map = (uint8_t*)dmap;
        } else {
            r->zc = hipMemcpyAsync(s->d + (size_t)r->pos * KS, h_buf, (size_t)len, hipMemcpyHostToDevice,
                                   s->stream) == hipSuccess;
        }
    }
    if (r->zc) q->n_zc.fetch_add(1);
    if (!r->zc) {
        uint8_t* dst = s->h + (size_t)r->pos * KS;
        std::memcpy(dst, h_buf, (size_t)len);
        if (q->k * Sb > len) std::memset(dst + len, 0, (size_t)(q->k * Sb - len));
    }
#if ZS3_DIAG
    q->tm[QT_SUB_COPY] += qt_now() - t1;
#endif
    copy_in_done(q, s);
    *req = r;
    return ZS3_OK;
}

int devq_submit_decode(DevQ* q, uint8_t* h_shards, int64_t shard_len, const uint8_t* h_present, int data_only,
                       const uint8_t* h_expect, int32_t* h_bad, uint8_t* h_sums_out, zs3_req** req) {
    auto* r = new zs3_req();
    r->q = q;
    r->lane = data_only ? GET : HEAL;
    r->S = shard_len;
    r->h_shards = h_shards;
    r->h_expect = h_expect;
    r->h_bad = h_bad;
    r->h_sums_out = h_sums_out;
    for (int i = 0; i < q->R; ++i) r->present[i] = h_present[i] ? 1 : 0;
    Slot* s;
    bool lone = false;  // no other batch of the lane in flight (zc_mode 1)
    {
        std::unique_lock<std::mutex> lk(q->mu);
        const int rc = reserve(q, lk, r, shard_len == q->S);
        if (rc) {
            q->live[r->lane].fetch_sub(1, std::memory_order_relaxed);
            delete r;
            return rc;
        }
        s = r->slot;
        lone = q->inflight_blocks[r->lane] == 0;
    }
    // survivors: DMA'd straight from a pinned caller buffer (runs of present rows, same
    // row layout as the slot), else copied into the pinned slot
    void* dmap = nullptr;
    const bool zc_try = q->zc_mode == 2 || (q->zc_mode == 1 && r->pos == 0 && lone);
    if (shard_len == q->S && q->zc_mode == 3 && zs3i_pinned_map(h_shards, (size_t)q->E, &dmap)) {
        r->zc = true;  // gathered by the batch's copy-list launch
        r->d_map = (uint8_t*)dmap;
        q->n_zc.fetch_add(1);
    } else if (shard_len == q->S && zc_try && zs3i_pinned(h_shards, (size_t)q->E)) {
        std::vector<uint8_t> absent((size_t)q->R);
        for (int i = 0; i < q->R; ++i) absent[(size_t)i] = !r->present[i];
        bool ok = true;
        for_runs(absent, q->R, [&](int a, int b) {
            ok &= hipMemcpyAsync(s->d + (size_t)r->pos * q->E + (size_t)a * q->S, h_shards + (size_t)a * q->S,
                                 (size_t)(b - a) * q->S, hipMemcpyHostToDevice, s->stream) == hipSuccess;
        });
        r->zc = ok;
        if (ok) q->n_zc.fetch_add(1);
    }
    uint8_t* dst = s->h + (size_t)r->pos * q->E;
    for (int i = 0; i < q->R && !r->zc; ++i)
        if (r->present[i]) std::memcpy(dst + (size_t)i * shard_len, h_shards + (size_t)i * shard_len, (size_t)shard_len);
    uint8_t* exp = s->h + q->off_sums() + (size_t)r->pos * q->R * 32;
    if (h_expect)
        std::memcpy(exp, h_expect, (size_t)q->R * 32);
    else
        std::memset(exp, 0, (size_t)q->R * 32);  // no stored sums: flags are ignored
    copy_in_done(q, s);
    *req = r;
    return ZS3_OK;
}

}  // namespace

// A queue: one DevQ per listed device (opts->devices, or the one opts->device), each with
// its own slots, streams and threads; a submitted block goes to the device with the
// fewest live blocks of its lane (zs3q::pick_device), so T concurrent callers spread
// over the devices' PCIe links and HBM, and each device batches its own blocks.
struct zs3_queue {
    std::vector<DevQ*> devs;
    std::atomic<unsigned> rr{0};  // rotating tie-break start

    DevQ* pick(int lane) {
        const int n = (int)devs.size();
        if (n == 1) {
            devs[0]->live[lane].fetch_add(1, std::memory_order_relaxed);
            return devs[0];
        }
        int live[64];
        for (int i = 0; i < n; ++i) live[i] = devs[(size_t)i]->live[lane].load(std::memory_order_relaxed);
        DevQ* d = devs[(size_t)zs3q::pick_device(live, n, rr.fetch_add(1, std::memory_order_relaxed))];
        d->live[lane].fetch_add(1, std::memory_order_relaxed);
        return d;
    }
};

extern "C" {

int zs3_queue_new(const zs3_codec* c, const zs3_queue_opts* opts, zs3_queue** out) {
    if (!c || !out) return ZS3_ERR_INVALID_ARG;
    *out = nullptr;
    int k = 0, m = 0;
    int64_t B = 0;
    if (zs3_codec_params(c, &k, &m, &B) != ZS3_OK) return ZS3_ERR_INVALID_ARG;
    std::vector<int> devices;
    if (opts && opts->n_devices > 0) {
        if (!opts->devices || opts->n_devices > 64) return ZS3_ERR_INVALID_ARG;
        for (int i = 0; i < opts->n_devices; ++i) {
            if (opts->devices[i] < 0) return ZS3_ERR_INVALID_ARG;
            devices.push_back(opts->devices[i]);
        }
    } else {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
        devices.push_back(opts && opts->device >= 0 ? opts->device : dev);
    }
    auto* q = new zs3_queue();
    for (int d : devices) {
        DevQ* dq = nullptr;
        const int rc = devq_new(c, d, opts, &dq);
        if (rc != ZS3_OK) {
            for (DevQ* x : q->devs) devq_free(x);
            delete q;
            return rc;
        }
        q->devs.push_back(dq);
    }
    *out = q;
    return ZS3_OK;
}

void zs3_queue_free(zs3_queue* q) {
    if (!q) return;
    for (DevQ* d : q->devs) devq_free(d);
    delete q;
}

int zs3_queue_submit_encode(zs3_queue* q, uint8_t* h_buf, int64_t len, int64_t cap, uint8_t* h_sums,
                            zs3_req** req) {
    if (!q || !req || q->devs.empty()) return ZS3_ERR_INVALID_ARG;
    const DevQ* d0 = q->devs[0];
    if (len < 0 || len > d0->B || (len > 0 && !h_buf)) return ZS3_ERR_INVALID_ARG;
    *req = nullptr;
    if (len == 0) return ZS3_OK;  // EncodeData len 0: k+m empty shards, nothing to do
    const int64_t Sb = (len + d0->k - 1) / d0->k;
    if (cap < (int64_t)d0->R * Sb) return ZS3_ERR_INVALID_ARG;
    return devq_submit_encode(q->pick(ENC), h_buf, len, h_sums, req);
}

int zs3_queue_submit_decode(zs3_queue* q, uint8_t* h_shards, int64_t shard_len, const uint8_t* h_present,
                            int data_only, const uint8_t* h_expect, int32_t* h_bad, uint8_t* h_sums_out,
                            zs3_req** req) {
    if (!q || !req || q->devs.empty()) return ZS3_ERR_INVALID_ARG;
    const DevQ* d0 = q->devs[0];
    if (!h_present || shard_len < 0 || shard_len > d0->S || (shard_len > 0 && !h_shards)) return ZS3_ERR_INVALID_ARG;
    *req = nullptr;
    if (shard_len == 0) return ZS3_ERR_SHARD_NO_DATA;
    return devq_submit_decode(q->pick(data_only ? GET : HEAL), h_shards, shard_len, h_present, data_only, h_expect,
                              h_bad, h_sums_out, req);
}

int64_t zs3_req_wait(zs3_req* r) {
    if (!r) return ZS3_OK;  // the empty-block case returned no handle
    DevQ* q = r->q;
    Slot* s = r->slot;  // not freed before r is finished
    bool own = false;
    {
#if ZS3_DIAG
        const int64_t t0 = qt_now();
#endif
        std::unique_lock<std::mutex> lk(q->mu);
        if (!r->done) q->cv_disp.notify_one();  // a lone waiter: the device may be idle
        q->cv_done.wait(lk, [&] { return r->done || s->ready; });
        if (!r->done) own = s->claimed[r->pos].exchange(1) == 0;
        if (!own) q->cv_done.wait(lk, [&] { return r->done; });
#if ZS3_DIAG
        q->tm[QT_WAIT_READY] += qt_now() - t0;
#endif
    }
    if (own) {  // copy this block's results out on the calling thread
        finish_req(q, s, r);
        finish_one(q, s);
    }
    const int64_t rc = r->result;
    delete r;
    return rc;
}

int zs3_queue_flush(zs3_queue* q) {
    if (!q) return ZS3_ERR_INVALID_ARG;
    for (DevQ* d : q->devs) {
        std::lock_guard<std::mutex> g(d->mu);
        d->flush = true;
        d->cv_disp.notify_one();
    }
    return ZS3_OK;
}

int zs3_queue_stats(const zs3_queue* q, int64_t* batches, int64_t* blocks) {
    if (!q) return ZS3_ERR_INVALID_ARG;
    int64_t b = 0, n = 0;
    for (const DevQ* d : q->devs) {
        b += d->n_batches.load();
        n += d->n_blocks.load();
    }
    if (batches) *batches = b;
    if (blocks) *blocks = n;
    return ZS3_OK;
}

int zs3_queue_device_stats(const zs3_queue* q, int index, int* device, int64_t* batches, int64_t* blocks) {
    if (!q || index < 0 || index >= (int)q->devs.size()) return ZS3_ERR_INVALID_ARG;
    const DevQ* d = q->devs[(size_t)index];
    if (device) *device = d->device;
    if (batches) *batches = d->n_batches.load();
    if (blocks) *blocks = d->n_blocks.load();
    return ZS3_OK;
}

#if ZS3_DIAG
int zs3_debug_queue_timers(const zs3_queue* q, double* us, int n) {
    if (!q || !us || n < 0) return ZS3_ERR_INVALID_ARG;
    for (int i = 0; i < n; ++i) us[i] = 0.0;
    for (const DevQ* d : q->devs)
        for (int i = 0; i < n && i < QT_N; ++i) us[i] += (double)d->tm[i].load() / 1e3;
    return QT_N;
}
#endif

int64_t zs3_queue_zero_copy_blocks(const zs3_queue* q) {
    if (!q) return ZS3_ERR_INVALID_ARG;
    int64_t n = 0;
    for (const DevQ* d : q->devs) n += d->n_zc.load();
    return n;
}

int64_t zs3_queue_encode_data(zs3_queue* q, uint8_t* h_buf, int64_t len, int64_t cap, uint8_t* h_sums) {
    zs3_req* r = nullptr;
    const int rc = zs3_queue_submit_encode(q, h_buf, len, cap, h_sums, &r);
    if (rc) return rc;
    return r ? zs3_req_wait(r) : 0;
}

int zs3_queue_decode_data_blocks(zs3_queue* q, uint8_t* h_shards, int64_t shard_len, const uint8_t* h_present,
                                 int data_only, const uint8_t* h_expect, int32_t* h_bad) {
    zs3_req* r = nullptr;
    const int rc = zs3_queue_submit_decode(q, h_shards, shard_len, h_present, data_only, h_expect, h_bad, nullptr, &r);
    if (rc) return rc;
    return (int)zs3_req_wait(r);
}

}  // extern "C"
