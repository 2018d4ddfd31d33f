// Micro-batcher for concurrent single-query searches (host only, included by
// runtime.hip).
//
// Weaviate calls SearchByVector once per query from many goroutines at once
// (shard_read.go:415-424, flat/index.go:423-448).  One fp32 query alone
// streams the whole corpus (HBM-bound, SURVEY §8d C3: 3.84 ms at 10M x 768),
// while a batch of B queries costs the same HBM pass plus MFMA work.  So
// concurrent callers are coalesced: leader/follower, no background thread.
// A caller enqueues its request; if no batch is running it becomes the
// leader, optionally waits batch_window_us for company (at most until as many
// callers are pending as were in the system during the last batch), takes every pending
// request, groups them by (d, k), runs each group's unfiltered requests
// through wv_index_search_by_vector_batch and its filtered ones through
// wv_index_search_by_vector_batch_multi_allow (each query its own list, one
// block-key launch) and hands every follower its rows.  Requests
// that arrive while a batch runs form the next batch.  Results are identical
// to individual calls: each query of a batch is searched independently.
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>

#include "batch_row.h"

struct wv_batch_req {
    const float* q;
    int64_t d;
    int32_t k;
    const uint64_t* allow_ids;
    int64_t n_allow;
    int32_t allow_mode;
    uint64_t* out_ids;
    float* out_dists;
    int32_t* out_count;
    int rc = WV_OK;
    std::string err;
    // 0 = waiting, 1 = done (results written), 2 = lead the next batch; the
    // caller sleeps on this word alone (futex), so a finished batch wakes its
    // callers without a herd on the batcher's mutex
    std::atomic<int> sig{0};
    wv_batch_row row{};   // the list as a slot bitmap in a page-locked row (row.host), built by the caller
    int64_t row_cap = 0;
};

// page-locked host memory for the leader's concatenated allow lists (defined
// by the including unit: hipHostMalloc in the library, malloc in the TSan mock)
static void* batch_pinned_alloc(size_t bytes);
static void batch_pinned_free(void* p);
// page-locked, device-mapped host rows for the allow bitmaps (allocated once,
// pooled), filled by the caller's thread and read in place by the leader's
// search (batch_search_slot_bitmaps, defined by the includer)
static uint32_t* batch_row_alloc(int64_t words, const uint32_t** dev);
static void batch_row_free(uint32_t* p);
static uint64_t batch_id_base(const wv_index* idx);
static bool batch_rows_on(const wv_index* idx);  // option batch_rows

struct wv_batcher {
    std::mutex m;
    // the concatenated allow lists of a filtered group, reused across launches:
    // page-locked (the copy to the device is one DMA) and warm (no page faults
    // per launch); only the leader touches it
    uint64_t* pin = nullptr;
    size_t pin_cap = 0;
    std::condition_variable cv_window;  // the leader waiting out batch_window_us
    int64_t want = 0;                   // ... until this many requests are pending
    std::vector<wv_batch_req*> pending;
    bool busy = false, in_window = false;
    int64_t calls = 0, launches = 0, max_batch_seen = 0;
    // callers in the system (pending + in the running batch): the most seen
    // since the last launch, and the running batch's size.  A leader inside its
    // window stops waiting once that many are pending (the callers it just
    // served are coming back), so the pipeline settles on one full batch per
    // cycle instead of two half batches alternating
    int64_t in_system = 0, running = 0;
    // free page-locked bitmap rows for the leader's sparse lists (reused: an
    // allocation per call would cost more than the list); own mutex
    struct Row { uint32_t* h; const uint32_t* d; int64_t cap; };
    std::mutex pool_m;
    std::vector<Row> rows_free;
};

static void batch_futex_wait(std::atomic<int>* w, int v) {
    syscall(SYS_futex, reinterpret_cast<int*>(w), FUTEX_WAIT_PRIVATE, v, nullptr, nullptr, 0);
}
// the word may belong to a request whose caller has already returned (it saw
// the store first): waking a stale address is harmless, nothing is dereferenced
static void batch_futex_wake(std::atomic<int>* w) {
    syscall(SYS_futex, reinterpret_cast<int*>(w), FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
}

static void batcher_free(wv_index* idx, wv_batcher* b) {
    (void)idx;
    if (b && b->pin) batch_pinned_free(b->pin);
    if (b)
        for (auto& r : b->rows_free) batch_row_free(r.h);
    delete b;
}

// each calling thread's own row, kept across its calls (a thread has one call
// in flight, so no lock and no pool traffic per call).  At thread exit the row
// goes to a process-wide list the next new thread takes from -- never freed
// there: a thread-exit destructor may run after the HIP runtime is gone
struct wv_thread_row {
    uint32_t* h = nullptr;
    const uint32_t* d = nullptr;
    int64_t cap = 0;
    static std::mutex& spare_m() { static std::mutex* m = new std::mutex; return *m; }
    static std::vector<wv_batcher::Row>& spare() {
        static std::vector<wv_batcher::Row>* v = new std::vector<wv_batcher::Row>;
        return *v;
    }
    ~wv_thread_row() {
        if (!h) return;
        std::lock_guard<std::mutex> g(spare_m());
        spare().push_back({h, d, cap});
    }
};

// A list as a slot bitmap when that is the smaller form (8-byte ids against
// one bit per slot up to the largest listed slot: lists above ~1/64 of the
// span): built in cacheable memory, then one sequential copy into a pooled
// page-locked row (no HIP call here: a caller only spends the list's CPU
// time).  False: keep the id list (or, forced, out of memory).
static bool build_row(wv_index* idx, wv_batcher* b, const uint64_t* ids, int64_t n, wv_batch_row* row, int64_t* cap,
                      bool force = false) {
    // force (the leader's sparse lists): a pooled row, *cap its capacity;
    // otherwise the calling thread's own row, *cap = -1 (nothing to release)
    if (n <= 0) return false;
    const uint64_t id_base = batch_id_base(idx);
    constexpr uint64_t kSlots = 1ull << 36;  // beyond any index's capacity: such ids are never present
    uint64_t top = 0;
    bool any = false;
    for (int64_t i = 0; i < n; i++)
        if (ids[i] >= id_base && ids[i] - id_base < kSlots) { top = std::max<uint64_t>(top, ids[i] - id_base); any = true; }
    const int64_t words = (int64_t)(top >> 5) + 1;
    if (!force && (!any || 2 * n <= words)) return false;
    thread_local std::vector<uint32_t> bits;
    bits.assign((size_t)words, 0u);
    for (int64_t i = 0; i < n; i++)
        if (ids[i] >= id_base && ids[i] - id_base < kSlots) {
            const uint64_t sl = ids[i] - id_base;
            bits[sl >> 5] |= 1u << (sl & 31);
        }
    (void)idx;
    wv_batcher::Row r{nullptr, nullptr, 0};
    if (!force) {
        thread_local wv_thread_row mine;
        if (mine.cap < words) {
            if (mine.h) batch_row_free(mine.h);
            mine.h = nullptr;
            {
                std::lock_guard<std::mutex> g(wv_thread_row::spare_m());
                auto& sp = wv_thread_row::spare();
                for (size_t i = 0; i < sp.size(); i++)
                    if (sp[i].cap >= words) {
                        mine.h = sp[i].h; mine.d = sp[i].d; mine.cap = sp[i].cap;
                        sp.erase(sp.begin() + (std::ptrdiff_t)i);
                        break;
                    }
            }
            if (!mine.h) {
                mine.cap = (words + 1023) / 1024 * 1024;
                mine.h = batch_row_alloc(mine.cap, &mine.d);
                if (!mine.h) { mine.cap = 0; return false; }
            }
        }
        r = wv_batcher::Row{mine.h, mine.d, -1};
    } else {
        {
            std::lock_guard<std::mutex> g(b->pool_m);
            for (size_t i = 0; i < b->rows_free.size(); i++)
                if (b->rows_free[i].cap >= words) {
                    r = b->rows_free[i];
                    b->rows_free.erase(b->rows_free.begin() + (std::ptrdiff_t)i);
                    break;
                }
        }
        if (!r.h) {
            r.cap = (words + 1023) / 1024 * 1024;
            r.h = batch_row_alloc(r.cap, &r.d);
            if (!r.h) return false;
        }
    }
    memcpy(r.h, bits.data(), (size_t)words * sizeof(uint32_t));
    *row = wv_batch_row{r.d, r.h, words, n};
    *cap = r.cap;
    return true;
}

static void release_row(wv_batcher* b, wv_batch_row* row, int64_t cap) {
    if (!row->host || cap < 0) return;  // (a thread's own row stays with the thread)
    std::lock_guard<std::mutex> g(b->pool_m);
    b->rows_free.push_back({const_cast<uint32_t*>(row->host), row->dev, cap});
    row->host = nullptr;
    row->dev = nullptr;
}

static wv_batcher* get_batcher(wv_index* idx) {
    static std::mutex create_mu;
    std::lock_guard<std::mutex> g(create_mu);
    if (!idx->batcher) idx->batcher = new wv_batcher();
    return idx->batcher;
}

// One launch for requests sharing (d, k): no list among them ->
// wv_index_search_by_vector_batch; lists -> wv_index_search_by_vector_batch_multi_allow
// (each query its own list).  On success every request gets its rows; on
// failure nothing is written and the error is returned.
static int launch_requests(wv_index* idx, wv_batcher* b, const std::vector<wv_batch_req*>& grp) {
    const int64_t n = (int64_t)grp.size();
    const int64_t d = grp[0]->d;
    const int32_t k = grp[0]->k;
    std::vector<float> q((size_t)(n * std::max<int64_t>(d, 0)));
    for (int64_t i = 0; i < n; i++) memcpy(&q[(size_t)(i * d)], grp[i]->q, (size_t)d * sizeof(float));
    const int32_t kk = std::max(k, 0);
    std::vector<uint64_t> ids((size_t)(n * kk) + 1);
    std::vector<float> dists((size_t)(n * kk) + 1);
    std::vector<int32_t> cnt((size_t)n);
    bool lists = false;
    for (wv_batch_req* r : grp) lists |= r->allow_mode != 0;
    int rc;
    if (!lists || n == 1) {
        rc = wv_index_search_by_vector_batch(idx, q.data(), n, d, k, grp[0]->allow_ids, grp[0]->n_allow,
                                             grp[0]->allow_mode, ids.data(), dists.data(), cnt.data());
    } else if (std::any_of(grp.begin(), grp.end(), [](wv_batch_req* r) { return r->row.host != nullptr; })) {
        // the lists as slot bitmaps read in place by the device: the callers
        // built theirs; the leader builds the (sparse) rest
        std::vector<wv_batch_row> rows((size_t)n);
        std::vector<std::pair<wv_batch_row, int64_t>> mine;
        rc = WV_OK;
        for (int64_t i = 0; i < n && !rc; i++) {
            wv_batch_req* r = grp[i];
            if (r->row.host) {
                rows[(size_t)i] = r->row;
                continue;
            }
            wv_batch_row row{nullptr, nullptr, 0, r->n_allow};
            int64_t cap = 0;
            if (r->n_allow > 0) {  // a sparse list: a row of its own all the same
                if (!build_row(idx, b, r->allow_ids, r->n_allow, &row, &cap, true)) {
                    rc = set_err(WV_ERR_HIP, "could not stage the batch's allow bitmaps");
                    break;
                }
                mine.push_back({row, cap});
            }
            rows[(size_t)i] = row;
        }
        if (!rc)
            rc = batch_search_slot_bitmaps(idx, q.data(), n, d, k, rows.data(), ids.data(), dists.data(), cnt.data());
        for (auto& m : mine) release_row(b, &m.first, m.second);
    } else {
        std::vector<int64_t> off((size_t)n + 1, 0);
        std::vector<int32_t> modes((size_t)n);
        for (int64_t i = 0; i < n; i++) {
            modes[(size_t)i] = grp[i]->allow_mode;
            off[(size_t)i + 1] = off[(size_t)i] + (grp[i]->allow_mode != 0 ? grp[i]->n_allow : 0);
        }
        const size_t need = (size_t)off[(size_t)n] + 1;
        if (need > b->pin_cap) {
            if (b->pin) batch_pinned_free(b->pin);
            b->pin_cap = std::max(need, b->pin_cap * 2);
            b->pin = static_cast<uint64_t*>(batch_pinned_alloc(b->pin_cap * sizeof(uint64_t)));
            if (!b->pin) b->pin_cap = 0;
        }
        if (!b->pin) {
            rc = set_err(WV_ERR_INVALID, "out of host memory for the batch's allow lists");
        } else {
            for (int64_t i = 0; i < n; i++)
                if (off[(size_t)i + 1] > off[(size_t)i])
                    memcpy(b->pin + off[(size_t)i], grp[i]->allow_ids, (size_t)grp[i]->n_allow * sizeof(uint64_t));
            rc = wv_index_search_by_vector_batch_multi_allow(idx, q.data(), n, d, k, b->pin, off.data(), modes.data(),
                                                             ids.data(), dists.data(), cnt.data());
        }
    }
    if (rc) return rc;
    for (int64_t i = 0; i < n; i++) {
        wv_batch_req* r = grp[i];
        r->rc = WV_OK;
        *r->out_count = cnt[i];
        memcpy(r->out_ids, &ids[(size_t)(i * kk)], (size_t)cnt[i] * sizeof(uint64_t));
        memcpy(r->out_dists, &dists[(size_t)(i * kk)], (size_t)cnt[i] * sizeof(float));
    }
    return WV_OK;
}

// Runs one group of requests sharing (d, k): the requests without an allow
// list in one plain launch (they never pay for the per-query bitmaps of the
// filtered form), the filtered ones in one multi-allow launch.  A launch that
// fails is retried request by request, so every caller gets exactly the
// result or error of its own one-query call.
static void run_group(wv_index* idx, wv_batcher* b, std::vector<wv_batch_req*>& grp) {
    std::vector<wv_batch_req*> part[2];
    for (wv_batch_req* r : grp) part[r->allow_mode != 0 ? 1 : 0].push_back(r);
    for (auto& sub : part) {
        if (sub.empty()) continue;
        int rc = launch_requests(idx, b, sub);
        if (rc == WV_OK) continue;
        if (sub.size() == 1) {
            sub[0]->rc = rc;
            sub[0]->err = wv_last_error();
            continue;
        }
        for (wv_batch_req* r : sub) {
            const int rc1 = launch_requests(idx, b, {r});
            if (rc1) {
                r->rc = rc1;
                r->err = wv_last_error();
            }
        }
    }
}

static void run_batch(wv_index* idx, wv_batcher* b, std::vector<wv_batch_req*>& batch) {
    // group by (d, k); each request keeps its own allow list
    std::vector<std::vector<wv_batch_req*>> groups;
    for (wv_batch_req* r : batch) {
        bool placed = false;
        for (auto& g : groups)
            if (g[0]->d == r->d && g[0]->k == r->k) { g.push_back(r); placed = true; break; }
        if (!placed) groups.push_back({r});
    }
    for (auto& g : groups) run_group(idx, b, g);
}

// a caller's request is done: its row back, its own error text
static int finish_req(wv_batcher* b, wv_batch_req* req) {
    release_row(b, &req->row, req->row_cap);
    if (req->rc) return set_err(req->rc, "%s", req->err.c_str());
    return WV_OK;
}

extern "C" int wv_index_search_by_vector(wv_index* idx, const float* query, int64_t d, int32_t k,
                                         const uint64_t* allow_ids, int64_t n_allow, int32_t allow_mode,
                                         uint64_t* out_ids, float* out_dists, int32_t* out_count) {
    if (!idx || !out_count) return set_err(WV_ERR_INVALID, "nil argument");
    if (d > 0 && !query) return set_err(WV_ERR_INVALID, "nil query");
    // a malformed list fails this caller alone, before it can share a launch;
    // any non-zero mode is a list, as in a one-query batch call
    allow_mode = allow_mode != 0 ? 1 : 0;
    if (allow_mode == 1 && (n_allow < 0 || (n_allow > 0 && !allow_ids))) return set_err(WV_ERR_INVALID, "nil allow ids");
    wv_batcher* b = get_batcher(idx);
    wv_batch_req req{query, d, k, allow_ids, n_allow, allow_mode, out_ids, out_dists, out_count};
    // a dense list: its slot bitmap, built here (in parallel with the other
    // callers) instead of by the leader
    if (allow_mode == 1 && n_allow > 0 && batch_rows_on(idx))
        build_row(idx, b, allow_ids, n_allow, &req.row, &req.row_cap);
    std::unique_lock<std::mutex> lk(b->m);
    b->calls++;
    b->pending.push_back(&req);
    b->in_system = std::max<int64_t>(b->in_system, (int64_t)b->pending.size() + b->running);
    // only a leader inside its batch window wants to hear about arrivals, and
    // only about the one that completes its batch
    if (b->in_window && (int64_t)b->pending.size() >= b->want) b->cv_window.notify_one();
    bool lead = !b->busy;
    if (lead) b->busy = true;
    for (;;) {
        if (!lead) {
            // a follower: sleeps on its own word until its batch is done (1) or
            // the leader's slot is handed to it (2, busy stays reserved for it)
            lk.unlock();
            int st;
            while ((st = req.sig.load(std::memory_order_acquire)) == 0) batch_futex_wait(&req.sig, 0);
            if (st == 1) return finish_req(b, &req);
            req.sig.store(0, std::memory_order_relaxed);
            lk.lock();
        }
        const int64_t window = idx->batch_window_us;
        const int64_t want = std::min<int64_t>(idx->batch_max, std::max<int64_t>(b->in_system, 1));
        if (window > 0 && (int64_t)b->pending.size() < want) {
            b->in_window = true;
            b->want = want;
            b->cv_window.wait_for(lk, std::chrono::microseconds(window),
                                  [&] { return (int64_t)b->pending.size() >= want; });
            b->in_window = false;
        }
        std::vector<wv_batch_req*> batch;
        const size_t take = std::min(b->pending.size(), (size_t)std::max<int64_t>(idx->batch_max, 1));
        batch.assign(b->pending.begin(), b->pending.begin() + take);
        b->pending.erase(b->pending.begin(), b->pending.begin() + take);
        b->running = (int64_t)take;
        b->in_system = (int64_t)(take + b->pending.size());
        b->launches++;
        b->max_batch_seen = std::max<int64_t>(b->max_batch_seen, (int64_t)batch.size());
        lk.unlock();
        run_batch(idx, b, batch);
        lk.lock();
        b->running = 0;
        // the leader's slot goes to the oldest pending request (possibly our own,
        // when the batch was capped at batch_max before it)
        wv_batch_req* next = b->pending.empty() ? nullptr : b->pending.front();
        if (!next) b->busy = false;
        lk.unlock();
        if (next && next != &req) {
            next->sig.store(2, std::memory_order_release);
            batch_futex_wake(&next->sig);
        }
        bool mine = false;
        for (wv_batch_req* r : batch) {
            if (r == &req) { mine = true; continue; }
            std::atomic<int>* w = &r->sig;
            w->store(1, std::memory_order_release);
            batch_futex_wake(w);
        }
        if (mine) return finish_req(b, &req);
        lk.lock();
        lead = next == &req;
    }
}

extern "C" int wv_index_batcher_stats(wv_index* idx, int64_t* out) {
    if (!idx || !out) return set_err(WV_ERR_INVALID, "nil argument");
    wv_batcher* b = get_batcher(idx);
    std::lock_guard<std::mutex> g(b->m);
    out[0] = b->calls;
    out[1] = b->launches;
    out[2] = b->max_batch_seen;
    return WV_OK;
}
