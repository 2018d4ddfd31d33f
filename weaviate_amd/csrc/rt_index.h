// rt_index.h -- index state and helpers shared by the runtime's translation
// units, split so their device code compiles in parallel:
//   runtime.hip        lifecycle, Add / Delete, options, stats, the exact
//                      search dispatch (search_core, the f32 / GEMV select
//                      fallback, run_replay), entry points, LSM restore,
//                      VectorIndex extras, micro-batcher
//   qs_runtime.hip     the block-key search (search_qs), the sharded phases
//                      and the cross-shard replay / merge entries
//   qs_exact.hip       its exact pass (k_blk_exact, k_exact_bm)
//   qs_replay.hip      its bounded heap replays (k_rp_*, k_blk_replay*)
//   quant_runtime.hip  BQ, PQ (fit + search), SQ, RQ and hnsw's flat search
// The kernel headers live in an anonymous namespace inside wv: every unit
// compiles (and registers) the kernels it launches.
#pragma once
#include <cerrno>
#include <cpuid.h>
#include <stdarg.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <atomic>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/wv_knn.h"
#include "kernels.hip"
#include "bq_kernels.hip"
#include "pq_kernels.hip"
#include "kernels_bf3.hip"
#include "rq_kernels.hip"
#include "gemv_kernels.hip"
#include "qs_kernels.hip"
#include "q8_kernels.hip"
#include "rq8_mfma.hip"
#include "sq_kernels.hip"

using namespace wv;


// ---------------------------------------------------------------------------
// errors (runtime.hip)
// ---------------------------------------------------------------------------
int set_err(int code, const char* fmt, ...);

#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) return set_err(WV_ERR_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

struct DBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() { release(); }  // every device buffer of an index is freed with it
    hipError_t ensure(size_t b) {
        if (b <= bytes) return hipSuccess;
        if (p) { hipFree(p); p = nullptr; bytes = 0; }
        size_t nb = std::max(b, (size_t)256);
        hipError_t e = hipMalloc(&p, nb);
        if (e == hipSuccess) bytes = nb;
        return e;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

static inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
// u32 words per row of the PQ code store (256-row tiles of 16-segment groups,
// pq_kernels.hip); cap is a multiple of 256
static inline int64_t pq_mwp(int m) { return (int64_t)((m + 15) / 16) * 4; }
static inline int pq_g16(int m) { return (m + 15) / 16; }

struct wv_batcher;
static void batcher_free(wv_index* idx, wv_batcher* b);

struct wv_index {
    std::mutex mu;
    int metric = WV_METRIC_COSINE_DOT;
    int variant = WV_VARIANT_AVX256;
    int compression = WV_COMPRESSION_NONE;
    int rescore_limit = -1;
    int cache_opt = 0;   // BQ.Cache / RQ.Cache (flatent UserConfig): QueryVectorDistancer reads codes
    int replay_par = 2;  // block-key replay: 2 = pooled three-kernel form (k < 64), 3 = pooled for any k,
                         // 1 = 8-wave form, 0 = one wave
    int64_t rp_pool = 1 << 20;  // pooled replay: candidate blocks per batch (144 B each)
    int pq_adc = 2;             // PQ ADC queries per workgroup: 2 = k_pq_adc2 (b64 LUT pairs), 1 = k_pq_adc
    int qs_force_flag = 0;      // tests: flag every query of the block-key path (exercise the replay)
    int exact_bm = 1;           // block-major exact distances (rows <= 508 floats): 1 on, 0 off
    int device = 0;
    uint64_t id_base = 0;
    uint64_t id_base0 = 0;  // id_base as created (a ScanWindow shifts id_base under mu; the batcher's callers read this)
    std::string root_path;

    int dims = 0, dpad = 0;
    hipStream_t stream = nullptr;

    int64_t cap = 0;       // slots allocated (multiple of BN)
    int64_t hiwater = 0;   // 1 + highest slot ever written
    float* X = nullptr;
    float* xnorm2 = nullptr;
    uint32_t* present = nullptr;
    uint32_t* d_maxn2 = nullptr;
    uint64_t* codes = nullptr;   // BQ: [words][cap] word-major codes of the stored rows
    int words = 0;
    // BQ codes unpacked to +-1 int8 ([cap][dpb8b], the int8 plane tiling) for the
    // block minima on the integer matrix cores (k_q8_blockkey<..., BQ>), 7..24 words
    unsigned char* bq8 = nullptr;
    int dpb8b = 0;
    int bq8_opt = 1;             // option bq8: block minima from the +-1 plane (1) or the VALU kernels (0)
    int64_t bq_last_nq = 0, bq_last_nblk = 0, bq_last_blk = 256;  // debug hook (wv_index_debug_bqmin): the last BQ batch's first group
    int scan_window = 1;         // option scan_window: an allow list scans only [allow.Min, allow.Max]
    // gathered allow-list search: a sparse allow list's rows (ascending id) as
    // a temporary sub-index searched by the same pipeline (option gather_max:
    // the largest such list, 0 = off)
    int64_t gather_max = 1 << 20;
    wv_index* sub = nullptr;
    DBuf subSlots;
    DBuf allowIds, allowCnt;     // the allow list on the device, its candidate count
    int64_t bq_nq = 0;           // BQ batch in flight (bq_begin): queries and R
    int bq_R = 0;
    int64_t qt_nq = 0, qt_ld = 0;  // sharded hnsw flat batch in flight (wv_index_quant_begin)
    int qt_k = 0, qt_R = 0, qt_trim = 0, qt_rescore = 0, qt_comp = 0, qt_form = 0;
    // PQ (compressionhelpers.ProductQuantizer): codebook [m][ks][ds], codes
    // [ceil(m/4)][cap] u32 (4 segment bytes per word, see pq_kernels.hip)
    int pq_m = 0, pq_ks = 0, pq_ds = 0, pq_training_limit = 0, pq_rescore = 1, pq_trained = 0;
    float* pq_centers = nullptr;
    uint32_t* pq_codes = nullptr;
    // bf16 hi plane of X for the block-key path (qs_kernels.hip): [cap][dpb],
    // dpb = dims rounded up to 128, built when dpb <= QS_MAX_DPB
    int use_qs = 0, qs_planes = 0, dpb = 0;
    int exact_filter = 1;           // k_blk_exact's bf16-plane row filter (option exact_filter)
    uint16_t* Xb = nullptr;
    // int8 block-key plane (q8_kernels.hip): [cap][dpb8] codes, one scale per
    // 32-row block, built beside the bf16 plane when 384 < dims <= 1536
    int q8_planes = 0, dpb8 = 0;
    int q8_only = 0;                // 1536 < dims <= 3072: int8 planes without the bf16 plane
    int64_t sel_split_max = 512;    // option sel_split_max: batches up to this many queries use the split selection
    int sel_filter = 1;             // option sel_filter: k_blk_select_f (1) or the sorted-list k_blk_select (0)
    int q8_opt = 1;                 // option q8: block keys from the int8 plane (1) or the bf16 plane (0)
    int q8_R = 0;                   // option q8_R: candidate lists for int8 keys (0: R = 8, 448 blocks)
    int q8_shape = 16;              // option q8_shape: 16 = v_mfma_i32_16x16x64_i8 kernel, 32 = 32x32x32
    int q8_stag = 0;
    int q8_pf = 1;                  // option q8_pf: A-fragment reads 1 or 2 chunks ahead                // option q8_stag: waves 4-7 reduce each block P0 chunks late (RB = 2)
    int q8_gemv = 1;                // option q8_gemv: batches of <= 32 queries stream the int8 plane through registers (k_q8_gemv)
    int q8_live = 1;                // option q8_live: waves of a partial query group's padding skip their MFMAs (k_q8_blockkey LIVE)
    int q8_prio = 0;                // option q8_prio: s_setprio 1 for waves 4-7 of k_q8_blockkey (experiment)
    int rp_few = 16;                // option rp_few: a device-counted replay list of at most this many queries takes k_blk_replay_par
    int bq_fast = 0;                // option bq_fast: BQ queries whose result no hamming tie can change skip the replay (k_bq_fast)
    int q8_filter = 1;              // option q8_filter: the exact pass bounds rows from the int8 plane (1) or bf16 (0)
    unsigned char* X8 = nullptr;
    float* sb8 = nullptr;
    uint32_t* qmax8 = nullptr;      // device [4]: max |x - x^|^2, max |x^|^2 (float bits)
    DBuf q8Qb, q8Scale, q8Info, q8Blk;
    uint32_t* qsmax = nullptr;      // device [4]: max |x - x_h|^2, max |x_h|^2 (float bits), non-finite flag
    uint32_t* qscount = nullptr;    // device [4]: [0] replayed queries (cumulative), [1] this batch's flagged,
                                    // [2] overflow second passes (cumulative), [3] this batch's
    int has_nonfinite = 0;          // host mirror of qsmax[2]
    uint64_t replayed_host = 0;     // replays counted on the host (legacy paths)
    int timed = 0;                  // ev0/ev1 bracket the last batch's dominant kernel
    int timed_total = 0;            // evt0/evt1 bracket the last batch's whole block-key pipeline
    int64_t rq_dbg_nq = 0, rq_dbg_nb = 0;  // first chunk of the last rq MFMA batch (debug hook)
    int64_t qs_last_nq = 0, qs_last_nb = 0, qs_last_ldk = 0;  // first chunk of the last block-key batch (debug hook)
    // > 0: the block keys / eps / query planes of the last search (nq queries,
    // one chunk, no allow list) still describe the stored rows -- the
    // cross-shard replay may bound its scan with them.  Reset by any write or search.
    int64_t qs_keys_nq = 0;
    hipEvent_t evt0 = nullptr, evt1 = nullptr;
    float last_eps_scale = 0.f, last_eps_base = 0.f;  // exactness-proof eps of the last MFMA batch (debug hook)
    int64_t last_nq = 0;
    int last_KP = 0;
    // rq-8 / rq-1 (rq_kernels.hip): rotation tables built at the first Add
    // (initializeDimensionsAndRQ, flat/index.go:338-360), codes + meta per slot
    int rq_bits = 0, rq_D = 0, rq_ready = 0;
    uint16_t* rq_src = nullptr;   // [3][D]
    float* rq_sign = nullptr;     // [3][D]
    float* rq_round = nullptr;    // [D] (rq-1)
    void* rq_codes = nullptr;     // rq-8: tiled [cap][D] bytes; rq-1: [D/64][cap] u64
    unsigned char* rq1_pm = nullptr;  // rq-1: the +-1 plane of the codes, tiled [cap][D] bytes (k_rq8_keys<.., 1>)
    float4* rq_meta = nullptr;    // [cap] meta, then (rq-8) [cap] uint32 code sums: rq_csum()
    // scalar quantizer (sq_kernels.hip): range a, b and the Go float32 constants
    int sq_ready = 0, sq_Dq = 0;
    float sq_a = 0.f, sq_b = 0.f, sq_a2 = 0.f, sq_ab = 0.f, sq_ib2 = 0.f;
    uint4* sq_codes = nullptr;    // rq-8 layout, Dq = round_up(d, 16) bytes per row
    uint2* sq_meta = nullptr;     // [cap] {sum, sum2} of the codes
    DBuf sqq, sqm;                // query codes / meta
    // hnsw.flatSearch parameters (wv_index_hnsw_flat_search)
    int hnsw_ef = -1, ef_min = 100, ef_max = 500, ef_factor = 8, hnsw_rescore = 1;
    std::vector<uint8_t> h_present;
    uint64_t count = 0;    // flat.count: incremented per Add (flat/index.go:380-385)
    int64_t npresent = 0;

    DBuf stage, slots, qraw, qn, qn2, spanA, spanI, candA, candI, candE, oIds, oD, oN, oF, valid, qlist, hI, hD, hN, rE, rB, qcodes, bqmin, bqSkip, cslot, cn, ident, lut, ascI, ascD, ascN, rqq, rqm;

    int margin = 8, force_replay = 0, spans_opt = 0, timing = 0, cbuf_opt = 0, kernel_opt = 3, bq_kernel = 0, sel_dbg = 0, qgroup_opt = 0, sel_opt = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // replay stream: the quantized searches' one-wave-per-query heap replays
    // run there, beside the next query group's full-GPU distance kernel
    hipStream_t aux = nullptr;
    hipEvent_t evd[2] = {nullptr, nullptr}, evr[2] = {nullptr, nullptr};
    DBuf rE2, rB2;
    DBuf qsQb, qsInfo, qsKey, qsCand, qsNc, qsEps, qsFlags, qsList, qsScratch;
    DBuf rpBlk, rpLb, rpQ, rpE, rpVm, rpOff, rpTot, rpCtr;  // pooled replay (k_rp_*)
    DBuf bmCnt, bmOff, bmPairs, bmE;                          // block-major exact (k_inv_*, k_exact_bm)
    DBuf fMask;                                               // block-major int8 row filter: survivor masks [cn][L]
    DBuf bmPart;                                              // chunk sums of the inversion's prefix scan
    int q8_bm = 1;                                            // option q8_bm: the int8 row filter block-major (1) or per query (0)
    void* bmCnt_zp = nullptr;                                 // bmCnt.p / .bytes when it is known all-zero
    size_t bmCnt_zb = 0;                                      // (a grown buffer may come back at the same address)
    // hipGraph replay of a repeated identical wv_index_search_device call
    // (option graph): the captured launch sequence is valid while the corpus,
    // its buffers and the options are unchanged (mut_gen) and the call's
    // pointers and sizes are the same (GraphKey)
    struct GraphKey {
        const void* q = nullptr;
        int64_t nq = 0, d = 0;
        int32_t k = 0, mode = 0;
        const void *ids = nullptr, *dd = nullptr, *cnt = nullptr, *flags = nullptr, *stream = nullptr;
        uint64_t gen = 0;
        bool operator==(const GraphKey& o) const {
            return q == o.q && nq == o.nq && d == o.d && k == o.k && mode == o.mode && ids == o.ids && dd == o.dd &&
                   cnt == o.cnt && flags == o.flags && stream == o.stream && gen == o.gen;
        }
    };
    int graph_opt = 1;
    uint64_t mut_gen = 1;
    GraphKey g_key, g_seen;
    bool g_failed = false;  // capture failed for g_seen: run it uncaptured
    hipGraph_t g_graph = nullptr;
    hipGraphExec_t g_exec = nullptr;
    uint64_t g_dq = 0, g_db = 0, g_dm = 0;  // stats deltas of the captured call
    int g_timed = 0, g_timed_total = 0;     // its timing-event state
    DBuf qsCap;                                               // per query: upper bound of the (k+1)-th exact distance
    int exact_cap = 1;                                        // k_blk_exact drops values above qsCap (phase 0)
    int replay_dbg = 0;                                       // k_blk_replay clock diagnostics (printf)
    int pq_cand = 1;                                          // PQ search: block minima + candidate blocks (k_pq_cand)
    int pq_adc3 = 2;                                          // minima: 2 k_pq_adc4 (16-byte LUT reads), 1 k_pq_adc3, 0 k_pq_adc2
    DBuf lutg;                                                // the LUT regrouped for k_pq_adc3 [64-query group][s][c][64]
    // PQ block keys on the integer matrix cores (l2-squared, 384 < d <= 1536):
    // the centred reconstruction x_c = x~ - mu as an int8 plane (k_block_q8
    // layout and scales), its fp32 |x_c|^2 and maxima ([0] R^2, [1] H^2, [2]
    // non-finite, [4] max |x_c|^2, float bits); rebuilt lazily over the dirty
    // slot range [pq8_lo, pq8_hi) written since the last search
    int pq8_opt = 1;                                          // option pq8
    int64_t pq8_cap = 0, pq8_lo = 0, pq8_hi = 0;
    int pq8_dpb8 = 0, pq8_mu_dirty = 1, pq8_bad = 0;
    unsigned char* pq8_X8 = nullptr;
    float* pq8_sb = nullptr;
    float* pq8_n2 = nullptr;
    DBuf pq8Max, pq8Mu, pq8Tmp, pq8Qc, qsCand2;
    DBuf rq8Qp, rq8Qcs, rq8Qm, rq8Fq, rq8Fm;                  // rq-8 MFMA route: query planes, flagged queries
    int rq_mfma = 1;
    // per-query allow lists (wv_index_search_by_vector_batch_allow): the exact
    // pass and the replays of search_qs read query q's bitmap at
    // pqa_valid + q * pqa_vq; cur_vq / cur_tq are set only while search_qs runs
    // in that mode (the launchers pass them to the kernels)
    const uint32_t* pqa_valid = nullptr;
    const int32_t* pqa_m = nullptr;  // per query: the select's threshold depth (k_blk_select mq)
    int pqa_R = 8;
    int sel_lower = 0;  // k_blk_select lowers an overflowing threshold instead of flagging                   // the select / exact list size 64 (R - 1) for them
    int pqa = 1;
    int64_t pqa_budget_mb = 4096;
    int64_t pqa_split_max = 64;
    int pqa_alone = 1;
    int pqa_keys = 1;       // option pqa_keys: per-query masked int8 keys (k_q8_blockkey<.., MASK>)
    std::atomic<int> batch_rows{1};  // option batch_rows: the batcher's dense lists as slot bitmaps (read by callers)
    int64_t pqa_vq = 0;
    int64_t cur_vq = 0;
    const float* cur_tq = nullptr;
    bool cur_pqk = false;   // search_qs: this batch's keys are per-query (the replays' upper bounds hold)
    DBuf pqaBits, pqaUnion, pqaIds, pqaQ, pqaM, pqaM2, qsT;
    int64_t q8_bm_min = 64;                                   // option q8_bm_min: smallest batch for the block-major int8 filter
    int rq_serial = 0;                                        // option rq_serial (debug): k_rq8_keys without the DMA lookahead                                          // option rq_mfma: rq-8 on the integer matrix cores
    DBuf pqZero;                                              // zero norms / qinfo for k_blk_select over ADC minima
    DBuf flCtr;                      // device flag-list counters (replay_flags)
    int64_t qs_phase_nq = 0;         // sharded phase 1 done for this batch size
    int qs_phase_k = 0;
    DBuf gmA, gmI;  // GEMV path: first level of the two-level span merge
    wv_stats stats{};
    // micro-batcher of concurrent single-query searches (batcher.hip)
    wv_batcher* batcher = nullptr;
    // written by set_option under mu, read by the batcher leader without it
    std::atomic<int64_t> batch_window_us{1000}, batch_max{4096};
    int gemv_max = 8, gemv_wg = 1024, exact_multi = 1;  // batches up to this many queries take the GEMV select kernel (kver 6)
};

// The block keys, eps and prepared query rows of the last batch (qs_keys_nq),
// a pending sharded phase 1 (qs_phase_nq), a sharded hnsw flat batch (qt_nq)
// and a sharded BQ batch (bq_nq) describe one batch on one corpus state: an
// Add, a Delete or another batch's query preparation ends them.
// the corpus, its buffers or the options changed: captured search graphs are stale
static inline void note_mutation(wv_index* idx) { idx->mut_gen++; }
// rq-8: the per-slot code sums stored behind the meta (rq_meta + cap)
static inline uint32_t* rq_csum(wv_index* idx) { return reinterpret_cast<uint32_t*>(idx->rq_meta + idx->cap); }
// PQ codes of slots [lo, hi) were (re)written: the int8 reconstruction plane
// of their blocks is stale
static inline void pq8_mark(wv_index* idx, int64_t lo, int64_t hi) {
    if (hi <= lo) return;
    if (idx->pq8_hi <= idx->pq8_lo) { idx->pq8_lo = lo; idx->pq8_hi = hi; return; }
    idx->pq8_lo = std::min(idx->pq8_lo, lo);
    idx->pq8_hi = std::max(idx->pq8_hi, hi);
}
static void invalidate_batch(wv_index* idx) {
    idx->qs_keys_nq = 0;
    idx->qs_phase_nq = 0;
    idx->qt_nq = 0;
    idx->bq_nq = 0;  // a sharded BQ batch's minima and query rows (wv_index_bq_begin)
}

// ---------------------------------------------------------------------------
// create / destroy / capacity
// ---------------------------------------------------------------------------
// k_qs_blockkey keeps 32 queries x dpb bf16 in VGPRs (two waves per SIMD) up
// to 768 dims; k_qs_blockkey_w4 (one wave per SIMD, query fragments in the
// 512-entry register file, dpb 1024 or 1536) up to 1536
constexpr int QS_MAX_DPB = 1536;
constexpr int Q8_MAX_DPB = 3072;  // int8-only block-key planes (k_q8_blockkey_cp), two column parts
constexpr int Q8_WIDE_DPB = 6144;  // ... NP = dpb8 / 1024 parts of 16 chunks above 3072
constexpr int QS_W4_DPB = 768;  // dpb above this: k_qs_blockkey_w4

// ---------------------------------------------------------------------------
// functions shared across the units (defined where noted)
// ---------------------------------------------------------------------------
// runtime.hip
double gamma_n(int n);
int prepare_queries(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t nq_pad);
int run_replay(wv_index* idx, hipStream_t s, const uint32_t* valid, const float* Qn, const int32_t* d_qlist,
               int nlist, int k, const uint64_t* in_i, const float* in_d, const int32_t* in_n, int extract,
               int out_by_query, int kout, uint64_t* oi, float* od, int32_t* on, int by_query = 0,
               uint64_t* rec_i = nullptr, float* rec_d = nullptr, int32_t* rec_n = nullptr, int rec_cap = 0);
void launch_pq_encode(wv_index* idx, int64_t n, const uint32_t* d_slots);
bool pqa_keys_route(const wv_index* idx);  // qs_runtime.hip: per-query masked keys for multi-allow batches
int shard_filter_bitmap(wv_index* idx, hipStream_t s, const uint64_t* allow, int64_t n_allow, const uint32_t** valid,
                        int64_t* n_valid);
void launch_rq_encode(wv_index* idx, hipStream_t s, const float* rows, int64_t ld, int64_t n, const uint32_t* d_slots,
                      int query, void* codes, int64_t cap, float4* meta, uint32_t* csum = nullptr,
                      unsigned char* pm = nullptr);
// qs_runtime.hip
int qs_R(int k);
int qs_R_flat(int k);
int search_qs(wv_index* idx, hipStream_t s, int64_t nq, int k, int mode, const uint32_t* valid, uint64_t* o_ids,
              float* o_d, int32_t* o_n, int32_t* o_flags, int phase = 0, float* topA = nullptr,
              const float* gA = nullptr, const float* gE = nullptr, int W = 0);
int launch_q8_keys(wv_index* idx, hipStream_t s, Q8Args a, int dpb8, bool l2);
int invert_lists(wv_index* idx, hipStream_t s, const uint32_t* cand, const int32_t* ncand, const int32_t* flags,
                 int64_t cn, int L, int64_t nb);
// qs_exact.hip
void launch_blk_exact(wv_index* idx, hipStream_t s, int RV, int metric, bool v5, const float* Qn,
                      const uint32_t* valid, int cn, int k, int kout, uint64_t* o_ids, float* o_d, int32_t* o_n,
                      int32_t* flags, const int32_t* list, const uint32_t* cnt, const float* eb, int64_t ldE,
                      const float* capv, const float4* qinfo, const Q8Filter* q8f, const uint32_t* fmask = nullptr);
void launch_q8_filt_bm(wv_index* idx, hipStream_t s, int metric, const Q8Filter& f, const float* xn2,
                       const uint32_t* valid, int64_t nb, int L, const float* capv, const float4* qinfo, float gd,
                       uint32_t* fmask);
void launch_exact_bm(wv_index* idx, hipStream_t s, int metric, bool v5, const float* Qn, int64_t nb, size_t bm_lds,
                     int64_t ldE);
// qs_replay.hip
bool blk_pooled(const wv_index* idx, int k, int64_t nb);
int launch_blk_replay(wv_index* idx, hipStream_t s, const float* key, int64_t ldk, int64_t nb, const float* eps,
                      const float4* qinfo, const uint32_t* valid, const float* Qn, const int32_t* list,
                      const uint32_t* counters, int nlist, int64_t max_list, int k, int kout, uint64_t* oi,
                      float* od, int32_t* on, const uint64_t* in_i, const float* in_d, const int32_t* in_n,
                      int extract, int by_list, uint64_t* rec_i = nullptr, float* rec_d = nullptr,
                      int32_t* rec_n = nullptr, int rec_cap = 0);
// quant_runtime.hip
int search_bq(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k, const uint32_t* valid,
              uint64_t* o_ids, float* o_d, int32_t* o_n);
int search_rq(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k, const uint32_t* valid,
              uint64_t* o_ids, float* o_d, int32_t* o_n);
int search_pq(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k, const uint32_t* valid,
              uint64_t* o_ids, float* o_d, int32_t* o_n);
int search_hnsw_flat(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k,
                     const uint32_t* valid, uint64_t* o_ids, float* o_d, int32_t* o_n);
int pq_fit_rows(wv_index* idx, const float* dT, int64_t n, uint64_t seed);
int64_t bq_max_batch(const wv_index* idx);
int rq_init(wv_index* idx);
int rq_encode_queries(wv_index* idx, hipStream_t s, int64_t nq);
int rq_dist(wv_index* idx, hipStream_t s, const uint32_t* valid, int64_t q0, int F, int64_t ld, float* E, float* bmin,
            const void* qcodes = nullptr, const float4* qmeta = nullptr);
