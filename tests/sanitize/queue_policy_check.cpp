// CPU check of the batching queue's policy (zs3server_amd/csrc/queue_policy.hpp): slot
// sizing, sealing, and the assignment of blocks to the devices of a multi-device queue
// (VERDICT r04 item 4).  Built with -fsanitize=address,undefined by tests/test_queue_policy.py.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../zs3server_amd/csrc/queue_policy.hpp"

#define CHECK(c)                                                             \
    do {                                                                     \
        if (!(c)) {                                                          \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);         \
            std::exit(1);                                                    \
        }                                                                    \
    } while (0)

int main() {
    using namespace zs3q;
    const int64_t MiB = 1 << 20;
    // slots hold exactly the largest batch: 64 MiB of input, 8..512 blocks, <= max_batch
    CHECK(slot_blocks(0, MiB) == 64);
    CHECK(slot_blocks(256, MiB) == 64);       // the shim's old 256 no longer over-sizes the slot
    CHECK(slot_blocks(16, MiB) == 16);
    CHECK(slot_blocks(0, 10 * MiB) == 8);     // legacy 10 MiB blocks: 8 (80 MiB), not 6
    CHECK(slot_blocks(4, 10 * MiB) == 4);
    CHECK(slot_blocks(0, 64 << 10) == 512);
    CHECK(slot_blocks(0, 64 * MiB) == 8);
    // sealing: half the live blocks, at least 8 (or the slot), at most the slot
    CHECK(seal_blocks(64, 50, 64) == 32);
    CHECK(seal_blocks(256, 50, 64) == 64);
    CHECK(seal_blocks(4, 50, 64) == 8);
    CHECK(seal_blocks(4, 50, 4) == 4);
    CHECK(seal_blocks(10, 50, 8) == 8);       // 10 MiB: floor clamped to the slot
    for (int cap : {1, 4, 8, 64, 512})
        for (int live = 0; live < 1100; live += 7) {
            const int s = seal_blocks(live, 50, cap);
            CHECK(s >= 1 && s <= cap);
        }
    // device assignment: fewest live blocks, ties from the rotating start
    {
        int live[4] = {3, 1, 1, 2};
        CHECK(pick_device(live, 4, 0) == 1);
        CHECK(pick_device(live, 4, 2) == 2);
        CHECK(pick_device(live, 4, 3) == 1);
        int one[1] = {9};
        CHECK(pick_device(one, 1, 5) == 0);
    }
    // T synchronous submitters over n devices (each block assigned, then finished in
    // submission order once T are live): every device ends within one block of the others
    for (int n : {1, 2, 3, 4, 8})
        for (int T : {1, 2, 5, 16, 64, 256}) {
            std::vector<int> live(n, 0), total(n, 0), fifo;
            unsigned rr = 0;
            for (int b = 0; b < 4000; ++b) {
                if ((int)fifo.size() == T) {
                    live[fifo.front()]--;
                    fifo.erase(fifo.begin());
                }
                const int d = pick_device(live.data(), n, rr++);
                live[d]++;
                total[d]++;
                fifo.push_back(d);
                int mx = 0, mn = 1 << 30;
                for (int x : live) mx = x > mx ? x : mx, mn = x < mn ? x : mn;
                CHECK(mx - mn <= 1);
            }
            int mx = 0, mn = 1 << 30;
            for (int x : total) mx = x > mx ? x : mx, mn = x < mn ? x : mn;
            CHECK(mx - mn <= 1);
        }
    // a lone caller (T = 1) alternates over the devices instead of sticking to one
    {
        std::vector<int> live(2, 0), seq;
        unsigned rr = 0;
        for (int b = 0; b < 6; ++b) {
            const int d = pick_device(live.data(), 2, rr++);
            seq.push_back(d);
        }
        CHECK(seq[0] != seq[1] && seq[1] != seq[2]);
    }
    std::printf("queue_policy_check: ok\n");
    return 0;
}
