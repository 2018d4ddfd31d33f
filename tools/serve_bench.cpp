// Serving-mode driver for the micro-batcher, in C++ threads (no Python GIL):
// T threads each call wv_index_search_by_vector (one query per call, host
// buffers -- how the cgo shim's goroutines would call it) on the C3 corpus for
// S seconds; prints one JSON line with QPS, launches, mean batch and latency.
// Build: hipcc -O2 -std=c++17 tools/serve_bench.cpp -Iinclude -Lweaviate_amd -lwvknn -Wl,-rpath,'$ORIGIN/../weaviate_amd' -o tools/serve_bench
// Run:   tools/serve_bench [n=10000000] [threads=256] [seconds=10] [window_us=1000, the library default] [allow_pct=0] [filtered_pct=100]
// allow_pct > 0: filtered_pct % of the threads search under their own allow
// list (a random allow_pct % of the ids, different per thread) -- filtered
// callers, batched through wv_index_search_by_vector_batch_multi_allow; the
// other threads search unfiltered (their own launch of the same batch).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "wv_knn.h"

#define CK(x)                                                                 \
    do {                                                                      \
        int rc_ = (x);                                                        \
        if (rc_) {                                                            \
            fprintf(stderr, "%s failed: %d %s\n", #x, rc_, wv_last_error()); \
            return 1;                                                         \
        }                                                                     \
    } while (0)

using clk = std::chrono::steady_clock;

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 10000000;
    const int T = argc > 2 ? atoi(argv[2]) : 256;
    const double secs = argc > 3 ? atof(argv[3]) : 10.0;
    const int64_t window = argc > 4 ? atoll(argv[4]) : 1000;
    const double allow_pct = argc > 5 ? atof(argv[5]) : 0.0;
    const double filtered_pct = argc > 6 ? atof(argv[6]) : 100.0;
    const int d = 768, k = 10, nq = 4096;
    wv_config cfg{};
    cfg.metric = WV_METRIC_COSINE_DOT;
    cfg.dims = d;
    cfg.rescore_limit = -1;
    cfg.variant = WV_VARIANT_AVX256;
    cfg.root_path = "serve_bench";
    wv_index* idx = nullptr;
    CK(wv_index_create(&cfg, &idx));
    CK(wv_index_reserve(idx, (uint64_t)n));
    const int64_t chunk = 1000000;
    float* stage = nullptr;
    if (hipMalloc(&stage, (size_t)std::min(chunk, n) * d * 4) != hipSuccess) return 1;
    for (int64_t r0 = 0; r0 < n; r0 += chunk) {
        int64_t m = std::min(chunk, n - r0);
        CK(wv_gen_device(0, 0, 1, (uint64_t)r0, m, d, stage, nullptr));
        CK(wv_index_add_range_device(idx, (uint64_t)r0, stage, m, d));
    }
    CK(wv_gen_device(0, 0, 2, 0, nq, d, stage, nullptr));
    std::vector<float> q((size_t)nq * d);
    if (hipMemcpy(q.data(), stage, q.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    hipFree(stage);
    CK(wv_index_set_option(idx, "batch_window_us", window));

    // serial: one caller
    uint64_t ids[16];
    float dists[16];
    int32_t cnt = 0;
    CK(wv_index_search_by_vector(idx, q.data(), d, k, nullptr, 0, 0, ids, dists, &cnt));
    auto s0 = clk::now();
    const int ser = 16;
    for (int i = 0; i < ser; i++) CK(wv_index_search_by_vector(idx, &q[(size_t)i * d], d, k, nullptr, 0, 0, ids, dists, &cnt));
    double serial_qps = ser / std::chrono::duration<double>(clk::now() - s0).count();

    int64_t st0[3], st1[3];
    CK(wv_index_batcher_stats(idx, st0));
    std::atomic<int> fails{0};
    std::vector<std::vector<double>> lat(T);
    std::vector<std::vector<uint64_t>> allow(T);
    int nfilt = 0;
    if (allow_pct > 0)
        for (int t = 0; t < T; t++) {  // thread t's list: ids whose hash falls below allow_pct %
            if (t >= (int)(T * filtered_pct / 100.0 + 0.5)) continue;  // an unfiltered caller
            nfilt++;
            const uint64_t thr = (uint64_t)(allow_pct / 100.0 * 4294967296.0);
            for (int64_t i = 0; i < n; i++) {
                uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull + (uint64_t)(t + 1) * 0xBF58476D1CE4E5B9ull;
                h ^= h >> 31;
                h *= 0x94D049BB133111EBull;
                if ((h >> 32) < thr) allow[t].push_back((uint64_t)i);
            }
        }
    auto stop = clk::now() + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(secs));
    auto t0 = clk::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            uint64_t li[16];
            float ld[16];
            int32_t lc = 0;
            for (int i = t; clk::now() < stop; i += T) {
                auto a = clk::now();
                const std::vector<uint64_t>& al = allow[t];
                const bool filtered = allow_pct > 0 && t < nfilt;
                if (wv_index_search_by_vector(idx, &q[(size_t)(i % nq) * d], d, k, filtered ? al.data() : nullptr,
                                              (int64_t)al.size(), filtered ? 1 : 0, li, ld, &lc))
                    fails++;
                lat[t].push_back(std::chrono::duration<double, std::milli>(clk::now() - a).count());
            }
        });
    for (auto& x : th) x.join();
    double el = std::chrono::duration<double>(clk::now() - t0).count();
    CK(wv_index_batcher_stats(idx, st1));
    std::vector<double> all;
    for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    auto pct = [&](double p) { return all.empty() ? 0.0 : all[std::min(all.size() - 1, (size_t)(p * all.size()))]; };
    int64_t calls = st1[0] - st0[0], launches = st1[1] - st0[1];
    printf("{\"workload\": \"%lld x %d cosine k=%d, single-query calls from %d C++ threads, %d of them with allow lists of %.2f %%\", \"qps\": %.1f, "
           "\"serial_qps\": %.1f, \"calls\": %lld, \"launches\": %lld, \"mean_batch\": %.1f, \"max_batch\": %lld, "
           "\"latency_ms\": {\"p50\": %.2f, \"p99\": %.2f}, \"window_us\": %lld, \"failures\": %d}\n",
           (long long)n, d, k, T, nfilt, allow_pct, calls / el, serial_qps, (long long)calls, (long long)launches,
           launches ? (double)calls / launches : 0.0, (long long)st1[2], pct(0.5), pct(0.99), (long long)window,
           fails.load());
    wv_index_destroy(idx);
    return fails.load() ? 1 : 0;
}
