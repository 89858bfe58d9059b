// Native driver for the batching queue (zs3_queue_*): T OS threads — the stand-in for T
// goroutines inside cgo calling Erasure.EncodeData per 1 MiB block
// (cmd/erasure-encode.go:83-111) — each encode `per` blocks through one queue,
// synchronously (submit + wait per block, as EncodeData returns before the next block
// is read).  Prints one JSON line per T: aggregate GiB/s of object bytes, per-block
// latency p50 / p99, blocks per device batch.
//   tools/queue_bench [T,T,...] [per] [k] [m] [max_batch] [slots] [pinned] [devices]
// devices: a comma list of HIP ordinals for a multi-device queue (e.g. 0,0 on one GPU).
// pinned = 1: every caller's block buffer comes from zs3_host_alloc (the pinned bpool),
// so the queue DMAs it zero-copy; 0 (default): pageable buffers, staged by memcpy.
// Built a second time against the diagnostics library (tools/queue_bench_diag, -DQB_DIAG):
// each line then also carries the queue's host-side phase timers (zs3_debug_queue_timers)
// over the run, as thread-seconds per second of wall time, and the device's busy fraction.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../include/zs3gpu.h"
#ifdef QB_DIAG
#include "../include/zs3gpu_diag.h"
#endif

using Clock = std::chrono::steady_clock;

int main(int argc, char** argv) {
    std::vector<int> Ts = {1, 4, 16, 64};
    if (argc > 1) {
        Ts.clear();
        std::string s = argv[1];
        size_t p = 0;
        while (p < s.size()) {
            size_t q = s.find(',', p);
            Ts.push_back(std::atoi(s.substr(p, q - p).c_str()));
            p = q == std::string::npos ? s.size() : q + 1;
        }
    }
    const int per = argc > 2 ? std::atoi(argv[2]) : 32;
    const int k = argc > 3 ? std::atoi(argv[3]) : 8, m = argc > 4 ? std::atoi(argv[4]) : 4;
    zs3_queue_opts o = {-1, argc > 5 ? std::atoi(argv[5]) : 0, 0, argc > 6 ? std::atoi(argv[6]) : 0, nullptr, 0};
    std::vector<int> devs;
    if (argc > 8) {
        std::string d = argv[8];
        size_t p = 0;
        while (p < d.size()) {
            size_t q2 = d.find(',', p);
            devs.push_back(std::atoi(d.substr(p, q2 - p).c_str()));
            p = q2 == std::string::npos ? d.size() : q2 + 1;
        }
        o.devices = devs.data();
        o.n_devices = (int)devs.size();
    }
    const int64_t B = 1 << 20, S = (B + k - 1) / k, R = k + m;
    zs3_codec* c = nullptr;
    if (zs3_codec_new(k, m, B, &c) != ZS3_OK) return 2;
    zs3_queue* q = nullptr;
    if (zs3_queue_new(c, &o, &q) != ZS3_OK) return 3;
    const int tmax = *std::max_element(Ts.begin(), Ts.end());
    const bool pinned = argc > 7 && std::atoi(argv[7]) != 0;
    std::vector<std::vector<uint8_t>> pageable(pinned ? 0 : tmax, std::vector<uint8_t>((size_t)(R * S)));
    std::vector<uint8_t*> bufs(tmax);
    for (int t = 0; t < tmax; ++t) {
        if (pinned) {
            void* p = nullptr;
            if (zs3_host_alloc(&p, (size_t)(R * S)) != ZS3_OK) return 4;
            bufs[t] = (uint8_t*)p;
        } else {
            bufs[t] = pageable[t].data();
        }
    }
    std::vector<std::vector<uint8_t>> sums(tmax, std::vector<uint8_t>((size_t)(R * 32)));
    for (int t = 0; t < tmax; ++t)
        for (int64_t i = 0; i < B; ++i) bufs[t][(size_t)i] = (uint8_t)(i * 131 + t * 7 + (i >> 9));
    for (int rep = 0; rep < 2; ++rep)
        for (int T : Ts) {
            std::vector<std::vector<double>> lat(T);
            std::atomic<int> errs{0};
            int64_t b0 = 0, n0 = 0, b1 = 0, n1 = 0;
            zs3_queue_stats(q, &b0, &n0);
#ifdef QB_DIAG
            double tm0[8] = {}, tm1[8] = {};
            zs3_debug_queue_timers(q, tm0, 8);
#endif
            const auto t0 = Clock::now();
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t)
                th.emplace_back([&, t] {
                    for (int i = 0; i < per; ++i) {
                        const auto a = Clock::now();
                        if (zs3_queue_encode_data(q, bufs[t], B, R * S, sums[t].data()) != S) errs++;
                        lat[t].push_back(std::chrono::duration<double, std::micro>(Clock::now() - a).count());
                    }
                });
            for (auto& x : th) x.join();
            const double dt = std::chrono::duration<double>(Clock::now() - t0).count();
            zs3_queue_stats(q, &b1, &n1);
            std::vector<double> all;
            for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
            std::sort(all.begin(), all.end());
#ifdef QB_DIAG
            zs3_debug_queue_timers(q, tm1, 8);
            if (rep == 1) {
                const char* names[8] = {"sub_lock", "sub_copy", "disp_launch", "comp_sync", "wait_ready", "copy_out",
                                        "gpu_sum", "gpu_busy"};
                std::printf("{\"path\": \"queue_timers\", \"threads\": %d, \"pinned\": %s, \"wall_s\": %.4f", T,
                            pinned ? "true" : "false", dt);
                for (int i = 0; i < 8; ++i) std::printf(", \"%s\": %.3f", names[i], (tm1[i] - tm0[i]) / 1e6 / dt);
                std::printf("}\n");
            }
#endif
            if (rep == 1)
                std::printf("{\"path\": \"queue_encode_native\", \"devices\": %d, \"pinned\": %s, \"k\": %d, \"m\": %d, \"threads\": %d, \"blocks\": %d, "
                            "\"GiBps\": %.2f, \"block_latency_us_p50\": %.1f, \"block_latency_us_p99\": %.1f, "
                            "\"blocks_per_batch\": %.1f, \"errors\": %d}\n",
                            std::max(1, o.n_devices), pinned ? "true" : "false", k, m, T, T * per, (double)T * per * B / dt / (1 << 30), all[all.size() / 2],
                            all[(size_t)(all.size() * 0.99)], (double)(n1 - n0) / std::max<int64_t>(1, b1 - b0),
                            errs.load());
            std::fflush(stdout);
        }
    zs3_queue_free(q);
    if (pinned)
        for (auto* p : bufs) zs3_host_free(p);
    zs3_codec_free(c);
    return 0;
}
