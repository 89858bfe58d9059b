// queue_policy.hpp — the batching queue's sizing and device-assignment rules (queue.hip),
// host-only and free of HIP so the CPU tests compile and check them directly
// (tests/sanitize/queue_policy_check.cpp).
#pragma once
#include <algorithm>
#include <cstdint>

namespace zs3q {

// Input bytes per device batch: big enough that a batch leaves the chain-latency regime
// of the fused kernels, small enough that two batches of the lane alternate (one's H2D
// under the other's kernel and D2H: 1 MiB RS(8+4), 64 submitters 29.9-30.5 GiB/s at
// batches of 32 vs 21-24 at 64-128, profiles/r04/queue_ab3.jsonl).
constexpr int64_t kBatchInputBytes = (int64_t)64 << 20;
constexpr int kMinBatch = 8;
constexpr int kMaxBatch = 512;

// Positions (blocks) per staging slot = the largest batch the queue launches:
// kBatchInputBytes of input, at least kMinBatch and at most kMaxBatch blocks, and at most
// max_batch when the caller sets one (> 0).  The slots are sized by this, so no slot
// memory sits beyond what a batch can use.
inline int slot_blocks(int max_batch, int64_t block_bytes) {
    const int64_t by_bytes = kBatchInputBytes / std::max<int64_t>(1, block_bytes);
    int cap = (int)std::min<int64_t>(kMaxBatch, std::max<int64_t>(kMinBatch, by_bytes));
    if (max_batch > 0) cap = std::min(cap, max_batch);
    return std::max(1, cap);
}

// Blocks at which the open slot is sealed: pct % of the lane's live blocks (open slot +
// in flight), so T synchronous submitters keep two batches of ~T/2 alternating; at least
// kMinBatch (or the slot's size, when smaller), at most the slot's size.
inline int seal_blocks(int live, int pct, int cap) {
    const int want = (live * pct + 99) / 100;
    return std::max(std::min(kMinBatch, cap), std::min(want, cap));
}

// Device for the next block of a lane: the fewest live blocks of that lane (submitted,
// not yet finished), ties broken from `start` onwards (a rotating start spreads a lone
// caller's blocks over the devices).  live[0..n) are the devices' counts.
inline int pick_device(const int* live, int n, unsigned start) {
    int best = 0;
    for (int i = 0; i < n; ++i) {
        const int d = (int)((start + (unsigned)i) % (unsigned)n);
        if (i == 0 || live[d] < live[best]) best = d;
    }
    return best;
}

}  // namespace zs3q
