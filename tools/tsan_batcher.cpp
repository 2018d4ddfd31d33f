// ThreadSanitizer harness for the host-side micro-batcher (weaviate_amd/csrc/
// batcher.hip): many threads call wv_index_search_by_vector at once -- the
// reference's concurrent SearchByVector callers (adapters/repos/db/
// shard_read.go:415-424) -- while another thread retunes batch_window_us /
// batch_max (wv_index_set_option's atomics).  The GPU batch entry point is
// replaced by a CPU mock with the same contract (per-index mutex, error text
// through the thread-local last error), so the leader/follower hand-off, the
// condition variables and the result copies run exactly as in the library.
// Every result is checked against a direct serial search; any data race
// aborts the run (TSAN_OPTIONS=halt_on_error=1).
//
// build + run: tools/tsan_batcher.sh
#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../include/wv_knn.h"

static thread_local std::string g_err;
static int set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
extern "C" const char* wv_last_error(void) { return g_err.c_str(); }

struct wv_batcher;
static void batcher_free(wv_index* idx, wv_batcher* b);

// the fields batcher.hip reads, as runtime.hip declares them
struct wv_index {
    std::mutex mu;
    wv_batcher* batcher = nullptr;
    std::atomic<int64_t> batch_window_us{0}, batch_max{4096};
    // mock corpus
    int dims = 0;
    std::vector<float> X;
    int64_t n = 0;
    std::atomic<int64_t> batch_calls{0};
};

// CPU stand-in for the HIP batch search: l2-squared over the corpus, top-k by
// (distance, id), the reference's error for a length mismatch; allow lists
// (mode 1 = allow) filter the rows
extern "C" int wv_index_search_by_vector_batch(wv_index* idx, const float* queries, int64_t nq, int64_t d, int32_t k,
                                               const uint64_t* allow_ids, int64_t n_allow, int32_t allow_mode,
                                               uint64_t* out_ids, float* out_dists, int32_t* out_counts) {
    std::lock_guard<std::mutex> g(idx->mu);
    idx->batch_calls++;
    if (d != idx->dims)
        return set_err(WV_ERR_VECTOR_LENGTH, "%lld vs %d: vector lengths don't match", (long long)d, idx->dims);
    if (k <= 0) return set_err(WV_ERR_INVALID, "k must be positive (reference heap Top() on empty queue)");
    std::vector<char> ok((size_t)idx->n, allow_mode == 0 ? 1 : 0);
    if (allow_mode)
        for (int64_t i = 0; i < n_allow; i++)
            if (allow_ids[i] < (uint64_t)idx->n) ok[allow_ids[i]] = 1;
    std::vector<std::pair<float, uint64_t>> v;
    for (int64_t q = 0; q < nq; q++) {
        v.clear();
        for (int64_t r = 0; r < idx->n; r++) {
            if (!ok[r]) continue;
            float s = 0.f;
            for (int c = 0; c < idx->dims; c++) {
                const float t = queries[q * d + c] - idx->X[r * idx->dims + c];
                s += t * t;
            }
            v.push_back({s, (uint64_t)r});
        }
        const int64_t m = std::min<int64_t>(k, (int64_t)v.size());
        std::partial_sort(v.begin(), v.begin() + m, v.end());
        for (int64_t i = 0; i < m; i++) { out_ids[q * k + i] = v[i].second; out_dists[q * k + i] = v[i].first; }
        out_counts[q] = (int32_t)m;
    }
    return WV_OK;
}

// per-query allow lists: the mock searches query by query (same contract)
extern "C" int wv_index_search_by_vector_batch_multi_allow(wv_index* idx, const float* queries, int64_t nq, int64_t d,
                                                           int32_t k, const uint64_t* allow_ids,
                                                           const int64_t* allow_offsets, const int32_t* allow_modes,
                                                           uint64_t* out_ids, float* out_dists, int32_t* out_counts) {
    for (int64_t q = 0; q < nq; q++) {
        const int rc = wv_index_search_by_vector_batch(idx, queries + q * d, 1, d, k, allow_ids + allow_offsets[q],
                                                       allow_offsets[q + 1] - allow_offsets[q], allow_modes[q],
                                                       out_ids + q * k, out_dists + q * k, out_counts + q);
        if (rc) return rc;
    }
    return WV_OK;
}

static void* batch_pinned_alloc(size_t bytes) { return malloc(bytes); }
static void batch_pinned_free(void* p) { free(p); }
static uint32_t* batch_row_alloc(int64_t words, const uint32_t** dev) {
    uint32_t* p = static_cast<uint32_t*>(malloc((size_t)std::max<int64_t>(words, 1) * sizeof(uint32_t)));
    *dev = p;
    return p;
}
static void batch_row_free(uint32_t* p) { free(p); }
static uint64_t batch_id_base(const wv_index*) { return 0; }
static bool batch_rows_on(const wv_index*) { return true; }

#include "../weaviate_amd/csrc/batch_row.h"
// the slot-bitmap batch: rows back to id lists, then query by query
static int batch_search_slot_bitmaps(wv_index* idx, const float* queries, int64_t nq, int64_t d, int32_t k,
                                     const wv_batch_row* rows, uint64_t* out_ids, float* out_dists,
                                     int32_t* out_counts) {
    for (int64_t q = 0; q < nq; q++) {
        std::vector<uint64_t> ids;
        for (int64_t w = 0; w < rows[q].words; w++)
            for (uint32_t v = rows[q].host[w]; v; v &= v - 1) ids.push_back((uint64_t)(w * 32 + __builtin_ctz(v)));
        ids.push_back(0);
        const int rc = wv_index_search_by_vector_batch(idx, queries + q * d, 1, d, k, ids.data(),
                                                       (int64_t)ids.size() - 1, 1, out_ids + q * k, out_dists + q * k,
                                                       out_counts + q);
        if (rc) return rc;
    }
    return WV_OK;
}

#include "../weaviate_amd/csrc/batcher.hip"

int main(int argc, char** argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 48;
    const int calls = argc > 2 ? atoi(argv[2]) : 60;
    wv_index idx;
    idx.dims = 16;
    idx.n = 600;
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    idx.X.resize((size_t)idx.n * idx.dims);
    for (float& x : idx.X) x = U(rng);
    std::atomic<bool> stop{false};
    std::atomic<int64_t> bad{0}, errs{0};
    // a tuner changes the batch window and size while searches run
    std::thread tuner([&] {
        std::mt19937 r2(3);
        while (!stop.load()) {
            idx.batch_window_us = (int64_t)(r2() % 3) * 50;
            idx.batch_max = 1 + (int64_t)(r2() % 64);
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    });
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        th.emplace_back([&, t] {
            std::mt19937 r(100 + t);
            std::uniform_real_distribution<float> V(-1.f, 1.f);
            for (int c = 0; c < calls; c++) {
                const int kind = (int)(r() % 8);
                const int64_t d = kind == 7 ? 15 : 16;   // a dimension error now and then
                const int32_t k = 1 + (int32_t)(r() % 12);
                std::vector<float> q((size_t)d);
                for (float& x : q) x = V(r);
                std::vector<uint64_t> allow;
                int32_t mode = 0;
                if (kind == 6) {  // a dense allow list: its slot bitmap built by this caller
                    mode = 1;
                    for (int i = 0; i < 40; i++) allow.push_back(r() % (uint64_t)idx.n);
                } else if (kind == 4) {  // dense lists shared by many callers (every other block) or a span
                    mode = 1;
                    if (c % 2) {
                        for (int64_t j = 0; j < idx.n; j++)
                            if ((j >> 5) % 2 == t % 2) allow.push_back((uint64_t)j);
                    } else {
                        const uint64_t a0 = r() % (uint64_t)(idx.n - 100);
                        for (uint64_t j = a0; j < a0 + 100; j++) allow.push_back(j);
                    }
                } else if (kind == 5) {  // a sparse one (ids kept; a bitmap batch gets the leader's row)
                    mode = 1;
                    for (int i = 0; i < 3; i++) allow.push_back(r() % (uint64_t)idx.n);
                    if (c % 5 == 0) allow.push_back(1ull << 40);  // an id past any slot
                }
                std::vector<uint64_t> ids((size_t)k);
                std::vector<float> dd((size_t)k);
                int32_t cnt = -1;
                const int rc = wv_index_search_by_vector(&idx, q.data(), d, k, allow.data(), (int64_t)allow.size(),
                                                         mode, ids.data(), dd.data(), &cnt);
                // the same search, serially, under the index mutex
                std::vector<uint64_t> ei((size_t)k);
                std::vector<float> ed((size_t)k);
                int32_t ecnt = -1;
                const int erc = wv_index_search_by_vector_batch(&idx, q.data(), 1, d, k, allow.data(),
                                                                (int64_t)allow.size(), mode, ei.data(), ed.data(),
                                                                &ecnt);
                if (rc != erc) { bad++; continue; }
                if (rc) {
                    errs++;
                    if (std::string(wv_last_error()).find("vector lengths don't match") == std::string::npos) bad++;
                    continue;
                }
                if (cnt != ecnt || memcmp(ids.data(), ei.data(), (size_t)cnt * 8) ||
                    memcmp(dd.data(), ed.data(), (size_t)cnt * 4))
                    bad++;
            }
        });
    }
    for (auto& x : th) x.join();
    stop = true;
    tuner.join();
    int64_t st[3];
    wv_index_batcher_stats(&idx, st);
    printf("tsan_batcher: %d threads x %d calls, %lld batches (max %lld), %lld dimension errors, %lld mismatches\n",
           threads, calls, (long long)st[1], (long long)st[2], (long long)errs.load(), (long long)bad.load());
    batcher_free(&idx, idx.batcher);
    return bad.load() == 0 && st[0] == (int64_t)threads * calls ? 0 : 1;
}
