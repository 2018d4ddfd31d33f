// runtime.hip -- host runtime and C ABI (include/wv_knn.h) of the gfx950
// flat-index engine.  One translation unit: the kernels are included so the
// template instantiations live next to their launches.
//
// Memory layout in HBM (DESIGN.md "data layout"):
//   X       [cap][dpad] fp32   slot-major store, slot = doc id - id_base, rows
//                               normalised for cosine (flat/index.go:371),
//                               dpad = dims rounded up to 32 (zero padded)
//   xnorm2  [cap]              sum of squares per stored row (approx. L2 path)
//   present [cap/32] u32       bitmap of slots holding a vector (LSM key exists)
// cap is a multiple of 128 (the MFMA tile) so tiles never read out of bounds.
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
#include "sq_kernels.hip"

using namespace wv;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string g_err;

static int set_err(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) return set_err(WV_ERR_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

extern "C" const char* wv_last_error(void) { return g_err.c_str(); }

// ---------------------------------------------------------------------------
// reference kernel-variant dispatch rule: distancer/l2_amd64.go:19-26
// (AVX-512 kernels only if cpu.X86.HasAMXBF16 && cpu.X86.HasAVX512)
// ---------------------------------------------------------------------------
static bool host_has_amxbf16_avx512() {
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
    bool avx512f = (b >> 16) & 1u;
    bool amxbf16 = (d >> 22) & 1u;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
    bool osxsave = (c >> 27) & 1u;
    if (!osxsave) return false;
    unsigned lo, hi;
    __asm__ volatile("xgetbv" : "=a"(lo), "=d"(hi) : "c"(0));
    bool os_avx512 = (lo & 0xE6) == 0xE6;
    return avx512f && os_avx512 && amxbf16;
}

extern "C" int wv_resolve_variant(int32_t requested) {
    if (requested == WV_VARIANT_AVX256 || requested == WV_VARIANT_AVX512) return requested;
    return host_has_amxbf16_avx512() ? WV_VARIANT_AVX512 : WV_VARIANT_AVX256;
}

// ---------------------------------------------------------------------------
// device buffers
// ---------------------------------------------------------------------------
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
static void batcher_free(wv_batcher* b);

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
    int64_t bq_nq = 0;           // BQ batch in flight (bq_begin): queries and R
    int bq_R = 0;
    // PQ (compressionhelpers.ProductQuantizer): codebook [m][ks][ds], codes
    // [ceil(m/4)][cap] u32 (4 segment bytes per word, see pq_kernels.hip)
    int pq_m = 0, pq_ks = 0, pq_ds = 0, pq_training_limit = 0, pq_rescore = 1, pq_trained = 0;
    float* pq_centers = nullptr;
    uint32_t* pq_codes = nullptr;
    // bf16 hi plane of X for the block-key path (qs_kernels.hip): [cap][dpb],
    // dpb = dims rounded up to 128, built when dpb <= QS_MAX_DPB
    int use_qs = 0, qs_planes = 0, dpb = 0;
    uint16_t* Xb = nullptr;
    uint32_t* qsmax = nullptr;      // device [4]: max |x - x_h|^2, max |x_h|^2 (float bits), non-finite flag
    uint32_t* qscount = nullptr;    // device [4]: [0] replayed queries (cumulative), [1] this batch's flagged,
                                    // [2] overflow second passes (cumulative), [3] this batch's
    int has_nonfinite = 0;          // host mirror of qsmax[2]
    uint64_t replayed_host = 0;     // replays counted on the host (legacy paths)
    int timed = 0;                  // ev0/ev1 bracket the last batch's dominant kernel
    int timed_total = 0;            // evt0/evt1 bracket the last batch's whole block-key pipeline
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
    float4* rq_meta = nullptr;    // [cap]
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

    DBuf stage, slots, qraw, qn, qn2, spanA, spanI, candA, candI, candE, oIds, oD, oN, oF, valid, qlist, hI, hD, hN, rE, rB, qcodes, bqmin, cslot, cn, ident, lut, ascI, ascD, ascN, rqq, rqm;

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
    DBuf qsCap;                                               // per query: upper bound of the (k+1)-th exact distance
    int exact_cap = 1;                                        // k_blk_exact drops values above qsCap (phase 0)
    int pq_cand = 1;                                          // PQ search: block minima + candidate blocks (k_pq_cand)
    DBuf pqZero;                                              // zero norms / qinfo for k_blk_select over ADC minima
    DBuf flCtr;                      // device flag-list counters (replay_flags)
    int64_t qs_phase_nq = 0;         // sharded phase 1 done for this batch size
    int qs_phase_k = 0;
    DBuf gmA, gmI;  // GEMV path: first level of the two-level span merge
    wv_stats stats{};
    // micro-batcher of concurrent single-query searches (batcher.hip)
    wv_batcher* batcher = nullptr;
    // written by set_option under mu, read by the batcher leader without it
    std::atomic<int64_t> batch_window_us{0}, batch_max{4096};
    int gemv_max = 8, gemv_wg = 1024, exact_multi = 1;  // batches up to this many queries take the GEMV select kernel (kver 6)
};

// The block keys, eps and prepared query rows of the last batch (qs_keys_nq)
// and a pending sharded phase 1 (qs_phase_nq) describe one batch on one corpus
// state: an Add, a Delete or another batch's query preparation ends them.
static void invalidate_batch(wv_index* idx) {
    idx->qs_keys_nq = 0;
    idx->qs_phase_nq = 0;
}

// ---------------------------------------------------------------------------
// create / destroy / capacity
// ---------------------------------------------------------------------------
// k_qs_blockkey keeps 32 queries x dpb bf16 in VGPRs (two waves per SIMD) up
// to 768 dims; k_qs_blockkey_w4 (one wave per SIMD, query fragments in the
// 512-entry register file, dpb 1024 or 1536) up to 1536
constexpr int QS_MAX_DPB = 1536;
constexpr int QS_W4_DPB = 768;  // dpb above this: k_qs_blockkey_w4

// dims fixed (config or first Add, initializeDimensionsAndRQ flat/index.go:338-360)
static void set_dims(wv_index* idx, int64_t d) {
    idx->dims = (int)d;
    idx->dpad = (int)round_up(d, BK);
    idx->dpb = (int)round_up(d, 128);
    if (idx->dpb > QS_W4_DPB) idx->dpb = (int)round_up(d, 512);  // 512-column ring parts
    idx->qs_planes = (idx->use_qs && idx->dpb <= QS_MAX_DPB) ? 1 : 0;
}

extern "C" int wv_index_create(const wv_config* cfg, wv_index** out) {
    if (!cfg || !out) return set_err(WV_ERR_INVALID, "invalid config: nil");
    if (cfg->metric < 0 || cfg->metric > WV_METRIC_HAMMING)
        return set_err(WV_ERR_INVALID, "invalid config: unknown distance metric %d", cfg->metric);
    if (cfg->compression != WV_COMPRESSION_NONE && cfg->compression != WV_COMPRESSION_BQ &&
        cfg->compression != WV_COMPRESSION_PQ && cfg->compression != WV_COMPRESSION_RQ8 &&
        cfg->compression != WV_COMPRESSION_RQ1 && cfg->compression != WV_COMPRESSION_SQ)
        return set_err(WV_ERR_UNSUPPORTED, "invalid config: unsupported compression %d", cfg->compression);
    // distancerIndicatorsAndError (rotational_quantization.go:41-55)
    if ((cfg->compression == WV_COMPRESSION_RQ8 || cfg->compression == WV_COMPRESSION_RQ1) &&
        cfg->metric == WV_METRIC_HAMMING)
        return set_err(WV_ERR_UNSUPPORTED, "Distance not supported yet hamming");
    if (cfg->dims > RQ_MAXD - 64 && (cfg->compression == WV_COMPRESSION_RQ8 || cfg->compression == WV_COMPRESSION_RQ1))
        return set_err(WV_ERR_UNSUPPORTED, "rq: dimensions > %d not supported", RQ_MAXD - 64);
    HIPCHK(hipSetDevice(cfg->device));
    wv_index* idx = new wv_index();
    idx->metric = cfg->metric;
    idx->variant = wv_resolve_variant(cfg->variant);
    idx->compression = cfg->compression;
    idx->rescore_limit = cfg->rescore_limit;
    idx->device = cfg->device;
    idx->id_base = cfg->id_base;
    idx->root_path = cfg->root_path ? cfg->root_path : "";
    // block-key path for the exact fp32 search (qs_kernels.hip); the bf16x3
    // select kernels (kernels_bf3.hip) need option bf3_planes before the first Add
    idx->use_qs = (cfg->compression == WV_COMPRESSION_NONE && cfg->metric != WV_METRIC_HAMMING) ? 1 : 0;
    idx->kernel_opt = 0;  // auto: the block-key path (7) when the planes exist, else the legacy select kernels
    if (cfg->compression == WV_COMPRESSION_RQ8) idx->rq_bits = 8;
    if (cfg->compression == WV_COMPRESSION_RQ1) idx->rq_bits = 1;
    if (cfg->compression == WV_COMPRESSION_PQ) {
        idx->pq_m = cfg->pq_segments;
        idx->pq_ks = cfg->pq_centroids;
        idx->pq_training_limit = cfg->pq_training_limit;
        idx->pq_rescore = cfg->pq_rescore;
    }
    if (cfg->dims > 0) set_dims(idx, cfg->dims);
    hipError_t e = hipStreamCreateWithFlags(&idx->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&idx->d_maxn2, sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(idx->d_maxn2, 0, sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&idx->qsmax, 4 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(idx->qsmax, 0, 4 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&idx->qscount, 4 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(idx->qscount, 0, 4 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipEventCreate(&idx->ev0);
    if (e == hipSuccess) e = hipEventCreate(&idx->ev1);
    if (e == hipSuccess) e = hipEventCreate(&idx->evt0);
    if (e == hipSuccess) e = hipEventCreate(&idx->evt1);
    if (e != hipSuccess) {
        delete idx;
        return set_err(WV_ERR_HIP, "create: %s", hipGetErrorString(e));
    }
    *out = idx;
    return WV_OK;
}

extern "C" void wv_index_destroy(wv_index* idx) {
    if (!idx) return;
    batcher_free(idx->batcher);
    hipSetDevice(idx->device);
    if (idx->stream) hipStreamSynchronize(idx->stream);
    for (DBuf* b : {&idx->stage, &idx->slots, &idx->qraw, &idx->qn, &idx->qn2, &idx->spanA, &idx->spanI, &idx->candA,
                    &idx->candI, &idx->candE, &idx->oIds, &idx->oD, &idx->oN, &idx->oF, &idx->valid, &idx->qlist,
                    &idx->hI, &idx->hD, &idx->hN, &idx->rE, &idx->rB, &idx->qcodes, &idx->bqmin, &idx->cslot,
                    &idx->cn, &idx->ident, &idx->lut, &idx->ascI, &idx->ascD, &idx->ascN, &idx->rqq, &idx->rqm,
                    &idx->rE2, &idx->rB2, &idx->gmA, &idx->gmI, &idx->qsQb, &idx->qsInfo, &idx->qsKey, &idx->qsCand,
                    &idx->qsNc, &idx->qsEps, &idx->qsFlags, &idx->qsList, &idx->qsScratch, &idx->rpBlk, &idx->rpLb,
                    &idx->rpQ, &idx->rpE, &idx->rpVm, &idx->rpOff, &idx->rpTot, &idx->rpCtr, &idx->flCtr})
        b->release();
    if (idx->aux) hipStreamSynchronize(idx->aux);
    for (hipEvent_t e : {idx->evd[0], idx->evd[1], idx->evr[0], idx->evr[1]})
        if (e) hipEventDestroy(e);
    if (idx->aux) hipStreamDestroy(idx->aux);
    if (idx->sq_codes) hipFree(idx->sq_codes);
    if (idx->sq_meta) hipFree(idx->sq_meta);
    idx->sqq.release();
    idx->sqm.release();
    if (idx->X) hipFree(idx->X);
    if (idx->xnorm2) hipFree(idx->xnorm2);
    if (idx->present) hipFree(idx->present);
    if (idx->d_maxn2) hipFree(idx->d_maxn2);
    if (idx->codes) hipFree(idx->codes);
    if (idx->pq_centers) hipFree(idx->pq_centers);
    if (idx->pq_codes) hipFree(idx->pq_codes);
    if (idx->Xb) hipFree(idx->Xb);
    if (idx->qsmax) hipFree(idx->qsmax);
    if (idx->qscount) hipFree(idx->qscount);
    for (void* p : {(void*)idx->rq_src, (void*)idx->rq_sign, (void*)idx->rq_round, idx->rq_codes, (void*)idx->rq_meta})
        if (p) hipFree(p);
    if (idx->ev0) hipEventDestroy(idx->ev0);
    if (idx->ev1) hipEventDestroy(idx->ev1);
    if (idx->evt0) hipEventDestroy(idx->evt0);
    if (idx->evt1) hipEventDestroy(idx->evt1);
    if (idx->stream) hipStreamDestroy(idx->stream);
    delete idx;
}

// grow the id-indexed store to hold `need` slots (requires dims set).
// Transactional: every new buffer is allocated and filled first; only then are
// the old ones freed and the new ones committed.  On any failure the partial
// new buffers are freed and the index is left exactly as it was.
static int ensure_capacity(wv_index* idx, int64_t need) {
    if (need <= idx->cap) return WV_OK;
    int64_t nc = std::max<int64_t>(need, idx->cap * 2);
    nc = round_up(std::max<int64_t>(nc, 1024), BN3);
    const int64_t oc = idx->cap;
    hipStream_t s = idx->stream;
    std::vector<void*> fresh;
    auto alloc = [&](void** p, size_t bytes) -> hipError_t {
        hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 256));
        if (e == hipSuccess) fresh.push_back(*p);
        else *p = nullptr;
        return e;
    };
    float* X = nullptr;
    float* xn = nullptr;
    uint32_t* pr = nullptr;
    uint64_t* cd = nullptr;
    uint16_t* xb = nullptr;
    void* rqc = nullptr;
    float4* rqm = nullptr;
    uint32_t* pc = nullptr;
    uint4* sqc = nullptr;
    uint2* sqmt = nullptr;
    const int words = (idx->dims + 63) / 64;
    const size_t rq_cb = idx->rq_bits == 8 ? (size_t)nc * idx->rq_D : (size_t)(idx->rq_D / 64) * nc * sizeof(uint64_t);
    const int64_t pq_w = idx->compression == WV_COMPRESSION_PQ && idx->pq_m > 0 ? pq_mwp(idx->pq_m) : 0;
    const size_t qs_b = (size_t)nc * idx->dpb * sizeof(uint16_t);
    hipError_t e = hipSuccess;
    const char* what = "";
#define WV_STEP(W, X_)                        \
    do {                                      \
        if (e == hipSuccess) { what = W; e = (X_); } \
    } while (0)
    WV_STEP("X", alloc((void**)&X, (size_t)nc * idx->dpad * sizeof(float)));
    WV_STEP("xnorm2", alloc((void**)&xn, (size_t)nc * sizeof(float)));
    WV_STEP("present", alloc((void**)&pr, (size_t)(nc / 32) * sizeof(uint32_t)));
    if (idx->compression == WV_COMPRESSION_BQ) WV_STEP("bq codes", alloc((void**)&cd, (size_t)words * nc * sizeof(uint64_t)));
    if (idx->qs_planes) WV_STEP("bf16 block-key plane", alloc((void**)&xb, qs_b));
    if (idx->rq_ready) {
        WV_STEP("rq codes", alloc(&rqc, rq_cb));
        WV_STEP("rq meta", alloc((void**)&rqm, (size_t)nc * sizeof(float4)));
    }
    if (pq_w) WV_STEP("pq codes", alloc((void**)&pc, (size_t)pq_w * nc * sizeof(uint32_t)));
    if (idx->sq_ready) {
        WV_STEP("sq codes", alloc((void**)&sqc, (size_t)nc * idx->sq_Dq));
        WV_STEP("sq meta", alloc((void**)&sqmt, (size_t)nc * sizeof(uint2)));
    }
    // zero the new tails, copy the old contents
    WV_STEP("memset", hipMemsetAsync(pr, 0, (size_t)(nc / 32) * sizeof(uint32_t), s));
    WV_STEP("memset", hipMemsetAsync(xn, 0, (size_t)nc * sizeof(float), s));
    WV_STEP("memset", hipMemsetAsync(X + (size_t)oc * idx->dpad, 0, (size_t)(nc - oc) * idx->dpad * sizeof(float), s));
    if (oc > 0) {
        WV_STEP("copy", hipMemcpyAsync(X, idx->X, (size_t)oc * idx->dpad * sizeof(float), hipMemcpyDeviceToDevice, s));
        WV_STEP("copy", hipMemcpyAsync(xn, idx->xnorm2, (size_t)oc * sizeof(float), hipMemcpyDeviceToDevice, s));
        WV_STEP("copy", hipMemcpyAsync(pr, idx->present, (size_t)(oc / 32) * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    }
    if (cd) {
        WV_STEP("memset", hipMemsetAsync(cd, 0, (size_t)words * nc * sizeof(uint64_t), s));
        if (oc > 0 && idx->codes)  // word-major: copy each word plane
            WV_STEP("copy", hipMemcpy2DAsync(cd, (size_t)nc * sizeof(uint64_t), idx->codes, (size_t)oc * sizeof(uint64_t),
                                             (size_t)oc * sizeof(uint64_t), words, hipMemcpyDeviceToDevice, s));
    }
    if (xb) {
        WV_STEP("memset", hipMemsetAsync(xb, 0, qs_b, s));
        if (oc > 0 && idx->Xb)
            WV_STEP("copy", hipMemcpyAsync(xb, idx->Xb, (size_t)oc * idx->dpb * sizeof(uint16_t), hipMemcpyDeviceToDevice, s));
    }
    if (rqc) {
        WV_STEP("memset", hipMemsetAsync(rqc, 0, rq_cb, s));
        WV_STEP("memset", hipMemsetAsync(rqm, 0, (size_t)nc * sizeof(float4), s));
        if (oc > 0 && idx->rq_codes) {
            if (idx->rq_bits == 8)  // tiles of 256 rows are contiguous: the old tiles are a prefix
                WV_STEP("copy", hipMemcpyAsync(rqc, idx->rq_codes, (size_t)oc * idx->rq_D, hipMemcpyDeviceToDevice, s));
            else
                WV_STEP("copy", hipMemcpy2DAsync(rqc, (size_t)nc * sizeof(uint64_t), idx->rq_codes,
                                                 (size_t)oc * sizeof(uint64_t), (size_t)oc * sizeof(uint64_t),
                                                 idx->rq_D / 64, hipMemcpyDeviceToDevice, s));
            WV_STEP("copy", hipMemcpyAsync(rqm, idx->rq_meta, (size_t)oc * sizeof(float4), hipMemcpyDeviceToDevice, s));
        }
    }
    if (pc) {
        WV_STEP("memset", hipMemsetAsync(pc, 0, (size_t)pq_w * nc * sizeof(uint32_t), s));
        if (oc > 0 && idx->pq_codes)
            WV_STEP("copy", hipMemcpyAsync(pc, idx->pq_codes, (size_t)pq_w * oc * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    }
    if (sqc) {  // 256-row tiles: the old tiles are a prefix
        WV_STEP("memset", hipMemsetAsync(sqc, 0, (size_t)nc * idx->sq_Dq, s));
        WV_STEP("memset", hipMemsetAsync(sqmt, 0, (size_t)nc * sizeof(uint2), s));
        if (oc > 0 && idx->sq_codes) {
            WV_STEP("copy", hipMemcpyAsync(sqc, idx->sq_codes, (size_t)oc * idx->sq_Dq, hipMemcpyDeviceToDevice, s));
            WV_STEP("copy", hipMemcpyAsync(sqmt, idx->sq_meta, (size_t)oc * sizeof(uint2), hipMemcpyDeviceToDevice, s));
        }
    }
    const hipError_t es = hipStreamSynchronize(s);
    if (e == hipSuccess && es != hipSuccess) { e = es; what = "sync"; }
#undef WV_STEP
    if (e != hipSuccess) {
        for (void* p : fresh) hipFree(p);
        (void)hipGetLastError();
        return set_err(WV_ERR_HIP, "ensure_capacity(%lld slots): %s: %s", (long long)nc, what, hipGetErrorString(e));
    }
    // commit
    auto swap_in = [](auto*& cur, auto* nw) {
        if (!nw) return;
        if (cur) hipFree(cur);
        cur = nw;
    };
    swap_in(idx->X, X);
    swap_in(idx->xnorm2, xn);
    swap_in(idx->present, pr);
    if (cd) { swap_in(idx->codes, cd); idx->words = words; }
    swap_in(idx->Xb, xb);
    if (rqc) {
        if (idx->rq_codes) hipFree(idx->rq_codes);
        idx->rq_codes = rqc;
        swap_in(idx->rq_meta, rqm);
    }
    swap_in(idx->pq_codes, pc);
    swap_in(idx->sq_codes, sqc);
    swap_in(idx->sq_meta, sqmt);
    idx->cap = nc;
    idx->h_present.resize((size_t)nc, 0);
    return WV_OK;
}

extern "C" int wv_index_reserve(wv_index* idx, uint64_t nslots) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->dims == 0) return set_err(WV_ERR_INVALID, "reserve: dimensions not set yet");
    return ensure_capacity(idx, (int64_t)nslots);
}

// ---------------------------------------------------------------------------
// insert path
// ---------------------------------------------------------------------------

// flat.ValidateBeforeInsert (flat/index.go:823-842)
static int validate_insert(wv_index* idx, int64_t d) {
    if (d == 0) return set_err(WV_ERR_INSERT, "cannot insert vector of dimension 0");
    if (idx->dims == 0) return WV_OK;
    if (idx->dims != d)
        return set_err(WV_ERR_INSERT, "insert called with a vector of the wrong size: %lld. Saved length: %d, path: %s",
                       (long long)d, idx->dims, idx->root_path.c_str());
    return WV_OK;
}

extern "C" int wv_index_validate_before_insert(wv_index* idx, int64_t d) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    return validate_insert(idx, d);
}

// ProductQuantizer.Encode of stored rows (slots list, or slots [0, n))
static void launch_pq_encode(wv_index* idx, int64_t n, const uint32_t* d_slots) {
    if (n <= 0) return;
    const size_t lds = (size_t)idx->pq_ks * idx->pq_ds * sizeof(float);
    dim3 grid((unsigned)((n + 255) / 256), (unsigned)idx->pq_m);
#define WV_PE(DSV) k_pq_encode<DSV><<<grid, 256, lds, idx->stream>>>(idx->X, idx->dpad, n, d_slots, idx->pq_ks, idx->pq_ds, idx->pq_centers, idx->variant, idx->pq_codes, pq_g16(idx->pq_m))
    switch (idx->pq_ds) {
    case 1: WV_PE(1); break;
    case 2: WV_PE(2); break;
    case 4: WV_PE(4); break;
    case 8: WV_PE(8); break;
    case 16: WV_PE(16); break;
    default: WV_PE(0); break;
    }
#undef WV_PE
}

// rq-8 / rq-1 encode of n rows (rows[slot * ld], slot = slots[r] or r) into the
// data layout (query = 0) or the group-tiled query layout (query = 1)
static void launch_rq_encode(wv_index* idx, hipStream_t s, const float* rows, int64_t ld, int64_t n,
                             const uint32_t* d_slots, int query, void* codes, int64_t cap, float4* meta) {
    if (n <= 0) return;
    const size_t lds = 2 * (size_t)idx->rq_D * sizeof(float);
    const bool v5 = idx->variant == WV_VARIANT_AVX512;
#define WV_RQE(B, V, Q) k_rq_encode<B, V, Q><<<(unsigned)n, 256, lds, s>>>(rows, ld, n, idx->dims, d_slots, idx->rq_D, idx->rq_src, idx->rq_sign, idx->rq_round, codes, cap, meta)
    if (idx->rq_bits == 8) {
        if (query) { if (v5) WV_RQE(8, AVX512, 1); else WV_RQE(8, AVX256, 1); }
        else { if (v5) WV_RQE(8, AVX512, 0); else WV_RQE(8, AVX256, 0); }
    } else {
        if (query) WV_RQE(1, AVX256, 1);
        else WV_RQE(1, AVX256, 0);
    }
#undef WV_RQE
}

// as_stored: the rows are the stored bytes already (LSM segment restore: flat.Add
// normalised them before storeVector, flat/index.go:376-378), so cosine rows are
// copied as they are -- fp32 normalisation is not idempotent.
static void launch_prepare(wv_index* idx, const float* d_in, int64_t n, const uint32_t* d_slots, bool as_stored = false) {
    dim3 grid((unsigned)((n + 255) / 256));
    switch (as_stored ? WV_METRIC_L2_SQUARED : idx->metric) {
    case WV_METRIC_COSINE_DOT:
        k_prepare_rows<COSINE><<<grid, 256, 0, idx->stream>>>(d_in, n, idx->dims, d_slots, idx->X, idx->dpad,
                                                              idx->xnorm2, idx->present, idx->d_maxn2);
        break;
    default:
        k_prepare_rows<L2><<<grid, 256, 0, idx->stream>>>(d_in, n, idx->dims, d_slots, idx->X, idx->dpad, idx->xnorm2,
                                                          idx->present, idx->d_maxn2);
        break;
    }
    if (idx->qs_planes)  // bf16 hi plane + residual-norm maxima of the block-key path
        k_rows_split<<<(unsigned)((n + 3) / 4), 256, 0, idx->stream>>>(idx->X, idx->dpad, idx->dpb, n, d_slots, idx->Xb,
                                                                       idx->qsmax);
    if (idx->compression == WV_COMPRESSION_PQ && idx->pq_trained) launch_pq_encode(idx, n, d_slots);
    if (idx->sq_ready)  // the compressor encodes every inserted vector (hnsw insert -> compressor.Preload)
        k_sq_encode<0><<<(unsigned)((n + 3) / 4), 256, 0, idx->stream>>>(idx->X, idx->dpad, n, idx->dims, d_slots,
                                                                        idx->sq_Dq, idx->sq_a, idx->sq_b,
                                                                        idx->sq_codes, idx->sq_meta);
    if (idx->rq_ready)  // Preload: quantizer.EncodeBytes / EncodeUint64 of the stored row (flat/index.go:844-865)
        launch_rq_encode(idx, idx->stream, idx->X, idx->dpad, n, d_slots, 0, idx->rq_codes, idx->cap, idx->rq_meta);
    if (idx->compression == WV_COMPRESSION_BQ) {  // Preload: quantizer.Encode of the stored row (flat/index.go:376)
        const int64_t nt = n * idx->words;
        k_bq_encode_rows<<<(unsigned)((nt + 255) / 256), 256, 0, idx->stream>>>(idx->X, idx->dpad, n, idx->dims, d_slots,
                                                                                 idx->codes, idx->cap);
    }
}

static int rq_init(wv_index* idx);

// host mirror of the device non-finite flag (rows with NaN/Inf route the exact
// search to the all-rows path); called after a synchronised Add
static int refresh_nonfinite(wv_index* idx) {
    if (!idx->qs_planes || idx->has_nonfinite) return WV_OK;
    uint32_t f = 0;
    HIPCHK(hipMemcpy(&f, idx->qsmax + 2, sizeof(uint32_t), hipMemcpyDeviceToHost));
    idx->has_nonfinite = f ? 1 : 0;
    return WV_OK;
}

// shared by the host and device insert entry points: dims (lazily fixed by
// the first Add), id range of the slot store
static int validate_rows(wv_index* idx, int64_t d, uint64_t first_slot, uint64_t last_slot) {
    int rc = validate_insert(idx, d);
    if (rc) return rc;
    if (idx->dims == 0 && d > (1 << 20)) return set_err(WV_ERR_INVALID, "dimensions too large: %lld", (long long)d);
    if (first_slot > last_slot || last_slot >= (1ull << 32) - BN)
        return set_err(WV_ERR_INVALID, "id %llu out of range", (unsigned long long)last_slot);
    return WV_OK;
}

// rows: host pointer to n x d floats; ids: host doc ids
static int add_rows_locked(wv_index* idx, const uint64_t* ids, const float* vecs, int64_t n, int64_t d,
                           bool as_stored = false) {
    int rc = validate_insert(idx, d);
    if (rc) return rc;
    if (idx->dims == 0) {  // initOnce: initializeDimensionsAndRQ (flat/index.go:338-360)
        if (d > (1 << 20)) return set_err(WV_ERR_INVALID, "dimensions too large: %lld", (long long)d);
        set_dims(idx, d);
    }
    if (idx->rq_bits && !idx->rq_ready) {
        rc = rq_init(idx);
        if (rc) return rc;
    }
    // upsert semantics of the replace bucket: the last write of an id wins.
    std::unordered_map<uint64_t, int64_t> last;
    last.reserve((size_t)n * 2);
    int64_t maxslot = -1;
    for (int64_t i = 0; i < n; i++) {
        if (ids[i] < idx->id_base) return set_err(WV_ERR_INVALID, "id %llu below shard id_base %llu",
                                                  (unsigned long long)ids[i], (unsigned long long)idx->id_base);
        uint64_t s = ids[i] - idx->id_base;
        if (s >= (1ull << 32) - BN) return set_err(WV_ERR_INVALID, "id %llu out of range", (unsigned long long)ids[i]);
        last[ids[i]] = i;
        maxslot = std::max<int64_t>(maxslot, (int64_t)s);
    }
    invalidate_batch(idx);
    rc = ensure_capacity(idx, maxslot + 1);
    if (rc) return rc;
    std::vector<int64_t> rows;
    rows.reserve(last.size());
    for (int64_t i = 0; i < n; i++)
        if (last[ids[i]] == i) rows.push_back(i);
    const int64_t chunk = std::max<int64_t>(1, (256ll << 20) / (d * 4));
    std::vector<float> hbuf;
    std::vector<uint32_t> hslots;
    for (size_t c0 = 0; c0 < rows.size(); c0 += (size_t)chunk) {
        size_t c1 = std::min(rows.size(), c0 + (size_t)chunk);
        size_t m = c1 - c0;
        hbuf.resize(m * d);
        hslots.resize(m);
        for (size_t j = 0; j < m; j++) {
            int64_t r = rows[c0 + j];
            memcpy(&hbuf[j * d], vecs + r * d, d * sizeof(float));
            hslots[j] = (uint32_t)(ids[r] - idx->id_base);
        }
        HIPCHK(idx->stage.ensure(m * d * sizeof(float)));
        HIPCHK(idx->slots.ensure(m * sizeof(uint32_t)));
        HIPCHK(hipMemcpyAsync(idx->stage.p, hbuf.data(), m * d * sizeof(float), hipMemcpyHostToDevice, idx->stream));
        HIPCHK(hipMemcpyAsync(idx->slots.p, hslots.data(), m * sizeof(uint32_t), hipMemcpyHostToDevice, idx->stream));
        launch_prepare(idx, idx->stage.as<float>(), (int64_t)m, idx->slots.as<uint32_t>(), as_stored);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(idx->stream));
        for (size_t j = 0; j < m; j++) {
            uint32_t s = hslots[j];
            if (!idx->h_present[s]) { idx->h_present[s] = 1; idx->npresent++; }
            idx->hiwater = std::max<int64_t>(idx->hiwater, (int64_t)s + 1);
        }
    }
    idx->count += (uint64_t)n;
    return refresh_nonfinite(idx);
}

extern "C" int wv_index_add(wv_index* idx, uint64_t id, const float* vec, int64_t d) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    return add_rows_locked(idx, &id, vec, 1, d);
}

extern "C" int wv_index_add_batch(wv_index* idx, const uint64_t* ids, const float* vecs, int64_t n, int64_t d) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (n == 0) return set_err(WV_ERR_INSERT, "insertBatch called with empty lists");  // flat/index.go:297
    if (n < 0 || !ids || !vecs) return set_err(WV_ERR_INSERT, "ids and vectors sizes does not match");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    return add_rows_locked(idx, ids, vecs, n, d);
}

extern "C" int wv_index_add_range_device(wv_index* idx, uint64_t first_id, const float* d_vecs, int64_t n,
                                         int64_t d) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (n == 0) return set_err(WV_ERR_INSERT, "insertBatch called with empty lists");
    if (n < 0 || !d_vecs) return set_err(WV_ERR_INSERT, "ids and vectors sizes does not match");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (first_id < idx->id_base) return set_err(WV_ERR_INVALID, "id below shard id_base");
    const uint64_t s0u = first_id - idx->id_base;
    int rc = validate_rows(idx, d, s0u, s0u + (uint64_t)n - 1);
    if (rc) return rc;
    if (idx->dims == 0) set_dims(idx, d);
    if (idx->rq_bits && !idx->rq_ready) {
        rc = rq_init(idx);
        if (rc) return rc;
    }
    const int64_t s0 = (int64_t)s0u;
    invalidate_batch(idx);
    rc = ensure_capacity(idx, s0 + n);
    if (rc) return rc;
    std::vector<uint32_t> hs((size_t)n);
    for (int64_t i = 0; i < n; i++) hs[i] = (uint32_t)(s0 + i);
    HIPCHK(idx->slots.ensure((size_t)n * sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(idx->slots.p, hs.data(), (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice, idx->stream));
    launch_prepare(idx, d_vecs, n, idx->slots.as<uint32_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(idx->stream));
    for (int64_t i = 0; i < n; i++) {
        if (!idx->h_present[s0 + i]) { idx->h_present[s0 + i] = 1; idx->npresent++; }
    }
    idx->hiwater = std::max<int64_t>(idx->hiwater, s0 + n);
    idx->count += (uint64_t)n;
    return refresh_nonfinite(idx);
}

// flat.Delete (flat/index.go:392-411): drop the key; count is not decremented
extern "C" int wv_index_delete(wv_index* idx, const uint64_t* ids, int64_t n) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    invalidate_batch(idx);
    bool dirty = false;
    for (int64_t i = 0; i < n; i++) {
        if (ids[i] < idx->id_base) continue;
        uint64_t s = ids[i] - idx->id_base;
        if ((int64_t)s >= idx->cap || !idx->h_present[s]) continue;
        idx->h_present[s] = 0;
        idx->npresent--;
        dirty = true;
    }
    if (dirty) {
        // rebuild the device bitmap from the host mirror
        std::vector<uint32_t> bits((size_t)(idx->cap / 32), 0);
        for (int64_t s = 0; s < idx->hiwater; s++)
            if (idx->h_present[s]) bits[s >> 5] |= 1u << (s & 31);
        HIPCHK(hipMemcpyAsync(idx->present, bits.data(), bits.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                              idx->stream));
        HIPCHK(hipStreamSynchronize(idx->stream));
    }
    return WV_OK;
}

extern "C" int wv_index_contains_doc(wv_index* idx, uint64_t id) {
    if (!idx) return 0;
    std::lock_guard<std::mutex> g(idx->mu);
    if (id < idx->id_base) return 0;
    uint64_t s = id - idx->id_base;
    return (int64_t)s < idx->cap && idx->h_present[s] ? 1 : 0;
}

extern "C" uint64_t wv_index_already_indexed(wv_index* idx) {
    if (!idx) return 0;
    std::lock_guard<std::mutex> g(idx->mu);
    return idx->count;
}

extern "C" int32_t wv_index_dims(wv_index* idx) {
    if (!idx) return 0;
    std::lock_guard<std::mutex> g(idx->mu);
    return idx->dims;
}

extern "C" int wv_index_set_option(wv_index* idx, const char* key, int64_t value) {
    if (!idx || !key) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    std::string k(key);
    if (k == "batch_window_us") { if (value < 0 || value > 1000000) return set_err(WV_ERR_INVALID, "batch_window_us out of range"); idx->batch_window_us = value; return WV_OK; }
    if (k == "exact_multi") { idx->exact_multi = value ? 1 : 0; return WV_OK; }
    if (k == "gemv_wg") { if (value < 8 || value > 65536) return set_err(WV_ERR_INVALID, "gemv_wg out of range"); idx->gemv_wg = (int)value; return WV_OK; }
    if (k == "gemv_max") { if (value < 0 || value > 4096) return set_err(WV_ERR_INVALID, "gemv_max out of range"); idx->gemv_max = (int)value; return WV_OK; }
    if (k == "batch_max") { if (value < 1) return set_err(WV_ERR_INVALID, "batch_max out of range"); idx->batch_max = value; return WV_OK; }
    if (k == "margin") { if (value < 2 || value > 30) return set_err(WV_ERR_INVALID, "margin out of range"); idx->margin = (int)value; }
    else if (k == "force_replay") idx->force_replay = (int)value;
    else if (k == "spans") idx->spans_opt = (int)value;
    else if (k == "timing") idx->timing = (int)value;
    else if (k == "cbuf") idx->cbuf_opt = (int)value;
    else if (k == "kernel") {  // 0 auto, 3 f32 MFMA select, 6 GEMV select, 7 block keys
        if (value != 0 && value != 3 && value != 6 && value != 7)
            return set_err(WV_ERR_INVALID, "kernel must be 0 (auto), 3, 6 or 7");
        idx->kernel_opt = (int)value;
    } else if (k == "qs") {
        if (idx->cap > 0 && (value != 0) != (idx->use_qs != 0))
            return set_err(WV_ERR_INVALID, "qs must be set before the first Add");
        idx->use_qs = value ? 1 : 0;
        if (idx->dims) set_dims(idx, idx->dims);
    }
    else if (k == "bq_kernel") idx->bq_kernel = (int)value;
    else if (k == "pq_cand") {  // 1: minima-only PQ search with candidate blocks (default), 0: full ADC matrix
        if (value < 0 || value > 1) return set_err(WV_ERR_INVALID, "pq_cand must be 0 or 1");
        idx->pq_cand = (int)value;
    } else if (k == "replay_par") {  // 2: pooled k_rp_* for k < 64 (default), 3: pooled for every k,
                                   // 1: k_blk_replay_par for k < 64, 0: k_blk_replay only
        if (value < 0 || value > 3) return set_err(WV_ERR_INVALID, "replay_par must be 0..3");
        idx->replay_par = (int)value;
    }
    else if (k == "qs_force_flag") idx->qs_force_flag = value ? 1 : 0;
    else if (k == "exact_bm") idx->exact_bm = value ? 1 : 0;
    else if (k == "exact_cap") idx->exact_cap = value ? 1 : 0;
    else if (k == "ef") idx->hnsw_ef = (int)value;  // hnsw UserConfig.EF (-1: dynamic)
    else if (k == "ef_min") idx->ef_min = (int)value;
    else if (k == "ef_max") idx->ef_max = (int)value;
    else if (k == "ef_factor") idx->ef_factor = (int)value;
    else if (k == "hnsw_rescore") idx->hnsw_rescore = value ? 1 : 0;  // 0: doNotRescore
    else if (k == "rescore_limit") idx->rescore_limit = (int)value;
    else if (k == "pq_adc") {
        if (value != 1 && value != 2) return set_err(WV_ERR_INVALID, "pq_adc must be 1 or 2");
        idx->pq_adc = (int)value;
    }
    else if (k == "rp_pool") {  // pooled replay capacity in 32-row blocks (tests force the fallback with 1)
        if (value < 1 || value > (1ll << 26)) return set_err(WV_ERR_INVALID, "rp_pool out of range");
        idx->rp_pool = value;
        idx->rpBlk.release(); idx->rpLb.release(); idx->rpQ.release(); idx->rpE.release(); idx->rpVm.release();
    }
    else if (k == "cache") {  // BQ.Cache / RQ.Cache: QueryVectorDistancer uses the cached codes
        if (value != 0 && value != 1) return set_err(WV_ERR_INVALID, "cache must be 0 or 1");
        idx->cache_opt = (int)value;
    }
    else if (k == "sel_dbg") idx->sel_dbg = (int)value;
    else if (k == "qgroup") idx->qgroup_opt = (int)value;
    else if (k == "sel_opt") idx->sel_opt = (int)value;
    else return set_err(WV_ERR_INVALID, "unknown option %s", key);
    return WV_OK;
}

extern "C" int wv_index_debug_candidates(wv_index* idx, float* A, float* E, uint32_t* I, float* eps, int64_t nq,
                                         int32_t* KP) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (nq != idx->last_nq || idx->last_KP == 0) return set_err(WV_ERR_INVALID, "debug_candidates: no matching batch");
    *KP = idx->last_KP;
    const size_t m = (size_t)nq * idx->last_KP;
    if (A) {
        HIPCHK(hipMemcpyAsync(A, idx->candA.p, m * sizeof(float), hipMemcpyDeviceToHost, idx->stream));
        HIPCHK(hipMemcpyAsync(E, idx->candE.p, m * sizeof(float), hipMemcpyDeviceToHost, idx->stream));
        HIPCHK(hipMemcpyAsync(I, idx->candI.p, m * sizeof(uint32_t), hipMemcpyDeviceToHost, idx->stream));
        std::vector<float> qn2((size_t)nq);
        HIPCHK(hipMemcpyAsync(qn2.data(), idx->qn2.p, (size_t)nq * sizeof(float), hipMemcpyDeviceToHost, idx->stream));
        HIPCHK(hipStreamSynchronize(idx->stream));
        for (int64_t q = 0; q < nq; q++) {  // k_finalize's eps
            const float qn = std::sqrt(qn2[q]);
            if (idx->metric == WV_METRIC_L2_SQUARED) { float t = qn + idx->last_eps_base; eps[q] = idx->last_eps_scale * t * t; }
            else eps[q] = idx->last_eps_scale * (qn * idx->last_eps_base + 1.f);
        }
    }
    return WV_OK;
}

extern "C" int wv_index_debug_blockkeys(wv_index* idx, int64_t q, float* A, float* eps, int64_t* nb) {
    if (!idx || !nb) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->qs_last_nq <= 0 || q < 0 || q >= idx->qs_last_nq)
        return set_err(WV_ERR_INVALID, "debug_blockkeys: no such query in the last block-key batch");
    *nb = idx->qs_last_nb;
    if (!A) return WV_OK;
    HIPCHK(hipStreamSynchronize(idx->stream));
    std::vector<float> key((size_t)idx->qs_last_nb);
    float4 qi;
    HIPCHK(hipMemcpy(key.data(), idx->qsKey.as<float>() + q * idx->qs_last_ldk, key.size() * sizeof(float),
                     hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&qi, idx->qsInfo.as<float4>() + q, sizeof(float4), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(eps, idx->qsEps.as<float>() + q, sizeof(float), hipMemcpyDeviceToHost));
    for (size_t b = 0; b < key.size(); b++) {  // qs_key_to_a, host side (same fp32 ops)
        const float kv = key[b];
        float a;
        if (idx->metric == WV_METRIC_L2_SQUARED) a = kv + qi.x;
        else if (idx->metric == WV_METRIC_DOT) a = kv;
        else { const float p = 1.f + kv; a = p < 0.f ? 0.f : p; }
        A[b] = a;
    }
    return WV_OK;
}

extern "C" int wv_index_stats(wv_index* idx, wv_stats* out) {
    if (!idx || !out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    // device-side counters and timings of the block-key path are read here,
    // never inside the search pipeline
    uint32_t dev_replays = 0;
    if (idx->qscount) {
        HIPCHK(hipStreamSynchronize(idx->stream));
        HIPCHK(hipMemcpy(&dev_replays, idx->qscount, sizeof(uint32_t), hipMemcpyDeviceToHost));
    }
    if (idx->timed) {
        HIPCHK(hipEventSynchronize(idx->ev1));
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, idx->ev0, idx->ev1) == hipSuccess) idx->stats.last_select_ms = ms;
    }
    if (idx->timed_total) {
        HIPCHK(hipEventSynchronize(idx->evt1));
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, idx->evt0, idx->evt1) == hipSuccess) idx->stats.last_total_ms = ms;
    }
    *out = idx->stats;
    out->replayed_queries = idx->stats.replayed_queries + dev_replays;
    return WV_OK;
}

// ---------------------------------------------------------------------------
// search path
// ---------------------------------------------------------------------------

// gamma_n = n u / (1 - n u), u = 2^-24 (Higham): |fl(sum) - sum| <= gamma_n sum|terms|
static double gamma_n(int n) {
    const double u = 5.9604644775390625e-08;
    return n * u / (1.0 - n * u);
}

// Exact heap replay for the listed query rows (device qlist): exact-order
// distances of every row (k_exact_rows) then the id-ordered heap replay
// (k_replay_scan), in groups bounded by a 2 GiB distance buffer.
// in_* / raw outputs are [nlist][k] device arrays indexed by list position;
// extract + out_by_query writes results to row qlist[i] of [nq][kout] arrays.
// by_query = 1: in-states and raw (non-extracted) outputs are [nq][k] rows
// indexed by query (qlist[i]) as well; rec_*: record every insertion
// ([nlist][rec_cap] by list position, count rec_cap + 1 = overflow).
static int run_replay(wv_index* idx, hipStream_t s, const uint32_t* valid, const float* Qn, const int32_t* d_qlist,
                      int nlist, int k, const uint64_t* in_i, const float* in_d, const int32_t* in_n, int extract,
                      int out_by_query, int kout, uint64_t* oi, float* od, int32_t* on, int by_query = 0,
                      uint64_t* rec_i = nullptr, float* rec_d = nullptr, int32_t* rec_n = nullptr, int rec_cap = 0) {
    const int64_t nslots = idx->hiwater;
    const int64_t ld = std::max<int64_t>(round_up(nslots, EBLK), EBLK);
    int64_t G = std::max<int64_t>(1, std::min<int64_t>(nlist, (2ll << 30) / (ld * 4)));
    HIPCHK(idx->rE.ensure((size_t)G * ld * sizeof(float)));
    HIPCHK(idx->rB.ensure((size_t)G * (ld / EBLK) * sizeof(float)));
    const size_t lds = (size_t)k * sizeof(uint64_t) + 64 * sizeof(float) + (size_t)k * sizeof(float) + 16;
    if (lds > 160 * 1024)
        return set_err(WV_ERR_INVALID, "k=%d exceeds the exact replay heap limit of %d results", k,
                       (int)((160 * 1024 - 272) / 12));
    HIPCHK(hipFuncSetAttribute((const void*)k_replay_scan, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const bool v5 = idx->variant == WV_VARIANT_AVX512;
    for (int64_t g0 = 0; g0 < nlist; g0 += G) {
        const int F = (int)std::min<int64_t>(G, nlist - g0);
        if (nslots > 0 && Qn) {
            const unsigned grid = (unsigned)(F * (ld / EBLK));
#define WV_EX(M, V) k_exact_rows<M, V><<<grid, EBLK, 0, s>>>(idx->X, idx->dpad, valid, nslots, Qn, idx->dims, d_qlist + g0, F, ld, idx->rE.as<float>(), idx->rB.as<float>())
            // AVX2 order (or AVX-512 below 128 dims, the same order): 4 queries per thread
            const bool multi = idx->metric != WV_METRIC_HAMMING && (!v5 || idx->dims < 128) && idx->exact_multi &&
                               (int64_t)idx->dpad * 16 <= 65536;
            const size_t lds_q = (size_t)4 * idx->dpad * sizeof(float);
            const unsigned gridm = (unsigned)(((F + 3) / 4) * (ld / EBLK));
#define WV_EXM(M) k_exact_rows_multi<M, 4><<<gridm, EBLK, lds_q, s>>>(idx->X, idx->dpad, valid, nslots, Qn, idx->dims, d_qlist + g0, F, ld, idx->rE.as<float>(), idx->rB.as<float>())
            if (multi) {
                switch (idx->metric) {
                case WV_METRIC_L2_SQUARED: WV_EXM(L2); break;
                case WV_METRIC_DOT: WV_EXM(DOT); break;
                default: WV_EXM(COSINE); break;
                }
            } else
            switch (idx->metric) {
            case WV_METRIC_L2_SQUARED: if (v5) WV_EX(L2, AVX512); else WV_EX(L2, AVX256); break;
            case WV_METRIC_DOT: if (v5) WV_EX(DOT, AVX512); else WV_EX(DOT, AVX256); break;
            case WV_METRIC_COSINE_DOT: if (v5) WV_EX(COSINE, AVX512); else WV_EX(COSINE, AVX256); break;
            default: WV_EX(HAMMING, AVX256); break;
            }
#undef WV_EX
#undef WV_EXM
            HIPCHK(hipGetLastError());
        }
        const bool raw = !extract;
        const int64_t ooff = by_query ? 0 : (raw || !out_by_query) ? g0 : 0;
        const int64_t ioff = by_query ? 0 : g0;
        k_replay_scan<<<F, 64, lds, s>>>(idx->rE.as<float>(), idx->rB.as<float>(), valid, Qn ? nslots : 0, ld,
                                         d_qlist + g0, F, k, idx->id_base, in_n ? in_i + ioff * k : nullptr,
                                         in_n ? in_d + ioff * k : nullptr, in_n ? in_n + ioff : nullptr, extract,
                                         out_by_query || by_query, kout, oi + ooff * (raw ? k : kout),
                                         od + ooff * (raw ? k : kout), on + ooff, by_query, by_query,
                                         rec_n ? rec_i + g0 * rec_cap : nullptr, rec_n ? rec_d + g0 * rec_cap : nullptr,
                                         rec_n ? rec_n + g0 : nullptr, rec_cap);
        HIPCHK(hipGetLastError());
    }
    return WV_OK;
}

// prepare padded (and for cosine exactly normalised) query rows + norms
// (overwrites idx->qn: the block keys / shard phase of an earlier batch no longer apply)
static int prepare_queries(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t nq_pad) {
    invalidate_batch(idx);
    HIPCHK(idx->qn.ensure((size_t)nq_pad * idx->dpad * sizeof(float)));
    HIPCHK(idx->qn2.ensure((size_t)nq_pad * sizeof(float)));
    float* Qn = idx->qn.as<float>();
    if (nq_pad > nq)
        HIPCHK(hipMemsetAsync(Qn + nq * idx->dpad, 0, (size_t)(nq_pad - nq) * idx->dpad * sizeof(float), s));
    if (idx->metric == WV_METRIC_COSINE_DOT)
        k_normalize_rows<<<(unsigned)((nq + 3) / 4), 256, 0, s>>>(d_qraw, nq, idx->dims, Qn, idx->dpad);
    else
        k_copy_pad_rows<<<(unsigned)((nq * idx->dpad + 255) / 256), 256, 0, s>>>(d_qraw, nq, idx->dims, Qn, idx->dpad);
    k_row_norm2<<<(unsigned)((nq_pad + 3) / 4), 256, 0, s>>>(Qn, nq_pad, idx->dpad, idx->qn2.as<float>());
    HIPCHK(hipGetLastError());
    return WV_OK;
}

// searchByVectorQuantized (flat/index.go:460-532) for BQ indexes, every query
// through the exact R-heap replay (bq_kernels.hip).  Outputs [nq][k].
// Phase 1 of the BQ search: validation, query normalisation + codes, identity
// query list.  Returns R (searchTimeRescore) via *R_out and the query group
// size (block-minima buffer bounded to 1 GiB) via *G_out.
static int bq_begin(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k, int* R_out,
                    int64_t* G_out) {
    // query code length vs stored code length: HammingBitwise (distancer/hamming.go:63-66)
    if ((qd + 63) / 64 != idx->words) return set_err(WV_ERR_VECTOR_LENGTH, "both vectors should have the same len");
    // the rescoring SingleDist then checks the float lengths (distancer/errors.go:16)
    if (qd != idx->dims)
        return set_err(WV_ERR_VECTOR_LENGTH, "%lld vs %d: vector lengths don't match", (long long)qd, idx->dims);
    if (k <= 0) return set_err(WV_ERR_INVALID, "k must be positive (reference heap Top() on empty queue)");
    const int R = idx->rescore_limit > k ? idx->rescore_limit : k;  // searchTimeRescore (:413-421)
    if (R > 8192) return set_err(WV_ERR_UNSUPPORTED, "rescore limit %d > 8192", R);
    const int64_t nq_pad = round_up(nq, QB);
    int rc = prepare_queries(idx, s, d_qraw, nq, nq_pad);
    if (rc) return rc;
    const float* Qn = idx->qn.as<float>();
    const int words = idx->words;
    HIPCHK(idx->qcodes.ensure((size_t)nq * words * sizeof(uint64_t)));
    {
        const int64_t nt = nq * words;
        // word-major query codes: word w of query q at qcodes[w * nq + q]
        k_bq_encode_rows<<<(unsigned)((nt + 255) / 256), 256, 0, s>>>(Qn, idx->dpad, nq, idx->dims, nullptr,
                                                                       idx->qcodes.as<uint64_t>(), nq);
        HIPCHK(hipGetLastError());
    }
    idx->stats.queries += (uint64_t)nq;
    idx->stats.batches++;
    idx->stats.replayed_queries += (uint64_t)nq;
    const int64_t nslots = idx->hiwater;
    const int64_t nblk = std::max<int64_t>((nslots + BQBLK - 1) / BQBLK, 1);
    // identity query list
    HIPCHK(idx->ident.ensure((size_t)nq * sizeof(int32_t)));
    {
        std::vector<int32_t> id((size_t)nq);
        for (int64_t i = 0; i < nq; i++) id[i] = (int32_t)i;
        HIPCHK(hipMemcpyAsync(idx->ident.p, id.data(), (size_t)nq * sizeof(int32_t), hipMemcpyHostToDevice, s));
    }
    constexpr int QPB = 16;
    *G_out = std::max<int64_t>(QPB, std::min<int64_t>(round_up(nq, QPB), ((1ll << 30) / (nblk * 4)) / QPB * QPB));
    *R_out = R;
    HIPCHK(idx->bqmin.ensure((size_t)(*G_out) * nblk * sizeof(float)));
    idx->bq_nq = nq;
    idx->bq_R = R;
    return WV_OK;
}

// compile-time word count for the LDS-broadcast block-minima kernel and the
// replay's unrolled loads (words <= 32, i.e. d <= 2048); 0 = generic kernels
static int bq_nw(wv_index* idx) {
    const int words = idx->words;
    const int nw = words <= 2 ? 2 : words <= 4 ? 4 : words <= 8 ? 8 : words <= 12 ? 12 : words <= 16 ? 16
                 : words <= 24 ? 24 : words <= 32 ? 32 : 0;
    return idx->bq_kernel == 1 ? 0 : nw;
}

// Phase 1b: block minima of query group [g0, g0 + F) into idx->bqmin
static int bq_blockmin(wv_index* idx, hipStream_t s, const uint32_t* valid, int64_t g0, int F) {
    constexpr int QPB = 16;
    const int64_t nq = idx->bq_nq;
    const int64_t nslots = idx->hiwater;
    const int64_t nblk = std::max<int64_t>((nslots + BQBLK - 1) / BQBLK, 1);
    const int words = idx->words;
    const int nw = bq_nw(idx);
    const int32_t* qlist = idx->ident.as<int32_t>();
    // timing (bench roofline): the block-minima pass of the first group
    if (idx->timing && g0 == 0) HIPCHK(hipEventRecord(idx->ev0, s));
    const uint64_t* qc = idx->qcodes.as<uint64_t>();
    float* bm = idx->bqmin.as<float>();
    {
        if (nw == 0) {
            dim3 grid((unsigned)nblk, (unsigned)((F + QPB - 1) / QPB));
            k_bq_blockmin<QPB><<<grid, 256, 0, s>>>(idx->codes, idx->cap, words, valid, nslots, qc, nq, qlist + g0, F,
                                                    nblk, bm);
        } else {
            const int64_t qg = (F + 255) / 256;
            const int64_t spans = std::max<int64_t>(1, std::min<int64_t>(nblk, (2048 + qg - 1) / qg));
            const int64_t bps = (nblk + spans - 1) / spans;
            dim3 grid((unsigned)((nblk + bps - 1) / bps), (unsigned)qg);
#define WV_BM(NWV) k_bq_blockmin_lds<NWV><<<grid, 256, 0, s>>>(idx->codes, idx->cap, words, valid, nslots, qc, nq, qlist + g0, F, nblk, bps, bm)
            switch (nw) {
            case 2: WV_BM(2); break;
            case 4: WV_BM(4); break;
            case 8: WV_BM(8); break;
            case 12: WV_BM(12); break;
            case 16: WV_BM(16); break;
            case 24: WV_BM(24); break;
            default: WV_BM(32); break;
            }
#undef WV_BM
        }
        HIPCHK(hipGetLastError());
        if (idx->timing && g0 == 0) HIPCHK(hipEventRecord(idx->ev1, s));
    }
    return WV_OK;
}

// Phase 2: the R-heap replay of query group [g0, g0 + F) over this shard, from
// heap states in_* (NULL = empty) [F][R]; pop = 1 writes the popped
// candidates (pop order), 0 the heap states.  Ids are global (id_base + slot).
// rec_*: record every insertion ([F][cap], count cap + 1 = overflow); out_n
// may then be NULL (no state written).
static int bq_replay(wv_index* idx, hipStream_t s, const uint32_t* valid, int64_t g0, int F, const uint64_t* in_ids,
                     const float* in_d, const int32_t* in_len, int pop, uint64_t* out_ids, float* out_d,
                     int32_t* out_n, uint64_t* rec_ids = nullptr, float* rec_d = nullptr, int32_t* rec_n = nullptr,
                     int cap = 0) {
    const int64_t nq = idx->bq_nq;
    const int R = idx->bq_R;
    const int64_t nslots = idx->hiwater;
    const int64_t nblk = std::max<int64_t>((nslots + BQBLK - 1) / BQBLK, 1);
    const int words = idx->words;
    const int nw = bq_nw(idx);
    const int32_t* qlist = idx->ident.as<int32_t>();
    const uint64_t* qc = idx->qcodes.as<uint64_t>();
    const float* bm = idx->bqmin.as<float>();
    const size_t lds_r = (size_t)R * sizeof(uint64_t) + 64 * sizeof(float) + (size_t)R * sizeof(float) + 16;
#define WV_RP(NWV)                                                                                              \
    do {                                                                                                        \
        if (lds_r > 64 * 1024)                                                                                  \
            HIPCHK(hipFuncSetAttribute((const void*)k_bq_replay<NWV>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                       (int)lds_r));                                                            \
        k_bq_replay<NWV><<<(unsigned)F, 64, lds_r, s>>>(idx->codes, idx->cap, words, valid, nslots, qc, nq,      \
                                                        qlist + g0, F, bm, nblk, R, idx->id_base, in_ids, in_d, \
                                                        in_len, pop, out_ids, out_d, out_n, rec_ids, rec_d,     \
                                                        rec_n, cap);                                            \
    } while (0)
    switch (nw) {
    case 2: WV_RP(2); break;
    case 4: WV_RP(4); break;
    case 8: WV_RP(8); break;
    case 12: WV_RP(12); break;
    case 16: WV_RP(16); break;
    case 24: WV_RP(24); break;
    case 32: WV_RP(32); break;
    default: WV_RP(0); break;
    }
#undef WV_RP
    HIPCHK(hipGetLastError());
    return WV_OK;
}

// Phase 3: exact distances of the candidate ids this shard holds
static int bq_rescore(wv_index* idx, hipStream_t s, const uint64_t* ids, const int32_t* cnt, float* E) {
    const int64_t nq = idx->bq_nq;
    const int R = idx->bq_R;
    const int64_t npairs = nq * R;
    const float* Qn = idx->qn.as<float>();
    const int32_t* qlist = idx->ident.as<int32_t>();
    const bool v5 = idx->variant == WV_VARIANT_AVX512;
#define WV_RS(M, V) k_rescore_ids<M, V><<<(unsigned)((npairs + 63) / 64), 64, 0, s>>>(idx->X, idx->dpad, Qn, idx->dims, ids, cnt, qlist, (int)nq, R, idx->id_base, idx->hiwater, E)
    switch (idx->metric) {
    case WV_METRIC_L2_SQUARED: if (v5) WV_RS(L2, AVX512); else WV_RS(L2, AVX256); break;
    case WV_METRIC_DOT: if (v5) WV_RS(DOT, AVX512); else WV_RS(DOT, AVX256); break;
    case WV_METRIC_COSINE_DOT: if (v5) WV_RS(COSINE, AVX512); else WV_RS(COSINE, AVX256); break;
    default: WV_RS(HAMMING, AVX256); break;
    }
#undef WV_RS
    HIPCHK(hipGetLastError());
    return WV_OK;
}

// Phase 4: insertToHeap(heap, k, ...) in pop order + extractHeap
static int bq_final(hipStream_t s, int64_t nq, int R, int k, int world, uint64_t id_stride, const int32_t* qlist,
                    const uint64_t* ids, const int32_t* cnt, const float* E, uint64_t* o_ids, float* o_d,
                    int32_t* o_n) {
    const size_t lds_f = (size_t)k * (sizeof(uint64_t) + sizeof(float)) + 16;
    if (lds_f > 64 * 1024)
        HIPCHK(hipFuncSetAttribute((const void*)k_bq_final, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_f));
    k_bq_final<<<(unsigned)nq, 64, lds_f, s>>>(ids, E, cnt, qlist, (int)nq, R, k, world, id_stride, o_ids, o_d, o_n, 0);
    HIPCHK(hipGetLastError());
    return WV_OK;
}

static int search_bq(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k,
                     const uint32_t* valid, uint64_t* o_ids, float* o_d, int32_t* o_n) {
    int R = 0;
    int64_t G = 0;
    int rc = bq_begin(idx, s, d_qraw, nq, qd, k, &R, &G);
    if (rc) return rc;
    HIPCHK(idx->ascI.ensure((size_t)nq * R * sizeof(uint64_t)));
    HIPCHK(idx->ascD.ensure((size_t)nq * R * sizeof(float)));
    HIPCHK(idx->cn.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(idx->candE.ensure((size_t)nq * R * sizeof(float)));
    for (int64_t g0 = 0; g0 < nq; g0 += G) {
        const int F = (int)std::min<int64_t>(G, nq - g0);
        rc = bq_blockmin(idx, s, valid, g0, F);
        if (rc) return rc;
        rc = bq_replay(idx, s, valid, g0, F, nullptr, nullptr, nullptr, 1, idx->ascI.as<uint64_t>() + g0 * R,
                       idx->ascD.as<float>() + g0 * R, idx->cn.as<int32_t>() + g0);
        if (rc) return rc;
    }
    rc = bq_rescore(idx, s, idx->ascI.as<uint64_t>(), idx->cn.as<int32_t>(), idx->candE.as<float>());
    if (rc) return rc;
    rc = bq_final(s, nq, R, k, 1, 0, idx->ident.as<int32_t>(), idx->ascI.as<uint64_t>(), idx->cn.as<int32_t>(),
                  idx->candE.as<float>(), o_ids, o_d, o_n);
    if (rc) return rc;
    if (idx->timing) {
        HIPCHK(hipStreamSynchronize(s));
        float ms = 0.f;
        hipEventElapsedTime(&ms, idx->ev0, idx->ev1);
        idx->stats.last_select_ms = ms;
    }
    return WV_OK;
}

// ---- sharded BQ (weaviate_amd/sharded.py ShardedBQSearch) ----
extern "C" int wv_index_bq_begin(wv_index* idx, const float* d_queries, int64_t nq, int64_t d, int32_t k,
                                 void* stream) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->compression != WV_COMPRESSION_BQ) return set_err(WV_ERR_INVALID, "bq_begin: index is not BQ-compressed");
    hipStream_t s = (hipStream_t)stream;  // NULL: the null stream (ordered with the caller's default-stream work)
    int R = 0;
    int64_t G = 0;
    int rc = bq_begin(idx, s, d_queries, nq, d, k, &R, &G);
    if (rc) return rc;
    if (G < nq) return set_err(WV_ERR_UNSUPPORTED, "bq_begin: batch of %lld queries exceeds one block-minima group",
                               (long long)nq);
    rc = bq_blockmin(idx, s, idx->present, 0, (int)nq);
    if (rc) return rc;
    if (!stream || idx->timing) HIPCHK(hipStreamSynchronize(s));
    if (idx->timing) {
        float ms = 0.f;
        hipEventElapsedTime(&ms, idx->ev0, idx->ev1);
        idx->stats.last_select_ms = ms;
    }
    return WV_OK;
}

extern "C" int wv_index_bq_replay(wv_index* idx, const uint64_t* d_in_ids, const float* d_in_d,
                                  const int32_t* d_in_len, int32_t pop, uint64_t* d_out_ids, float* d_out_d,
                                  int32_t* d_out_len, void* stream) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->bq_nq <= 0) return set_err(WV_ERR_INVALID, "bq_replay: no batch begun");
    hipStream_t s = (hipStream_t)stream;  // NULL: the null stream (ordered with the caller's default-stream work)
    int rc = bq_replay(idx, s, idx->present, 0, (int)idx->bq_nq, d_in_ids, d_in_d, d_in_len, pop, d_out_ids, d_out_d,
                       d_out_len);
    if (rc) return rc;
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

// parallel cross-shard BQ replay: per query the R smallest block minima of this
// shard ([nq][R] ascending, +inf padded) -- upper bounds of distinct rows
extern "C" int wv_index_bq_bounds(wv_index* idx, float* d_out, void* stream) {
    if (!idx || !d_out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->bq_nq <= 0) return set_err(WV_ERR_INVALID, "bq_bounds: no batch begun");
    hipStream_t s = (hipStream_t)stream;
    const int64_t nblk = std::max<int64_t>((idx->hiwater + BQBLK - 1) / BQBLK, 1);
    const int nbins = idx->words * 64 + 1;
    const size_t lds = (size_t)nbins * sizeof(uint32_t);
    if (lds > 64 * 1024)
        HIPCHK(hipFuncSetAttribute((const void*)k_bq_bounds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    k_bq_bounds<<<(unsigned)idx->bq_nq, 256, lds, s>>>(idx->bqmin.as<float>(), nblk, nbins, idx->bq_R, d_out);
    HIPCHK(hipGetLastError());
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

// parallel cross-shard BQ replay: this shard's R-heap replay from heap states
// d_in_* (k copies of a bound, by query), recording every insertion in id order
// (ids, dists [nq][cap], counts [nq]; cap + 1 = the record overflowed)
extern "C" int wv_index_bq_replay_record(wv_index* idx, const uint64_t* d_in_ids, const float* d_in_d,
                                         const int32_t* d_in_len, int32_t cap, uint64_t* d_rec_ids, float* d_rec_d,
                                         int32_t* d_rec_n, void* stream) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (cap < 1 || !d_rec_ids || !d_rec_d || !d_rec_n) return set_err(WV_ERR_INVALID, "invalid record buffers");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->bq_nq <= 0) return set_err(WV_ERR_INVALID, "bq_replay_record: no batch begun");
    hipStream_t s = (hipStream_t)stream;
    int rc = bq_replay(idx, s, idx->present, 0, (int)idx->bq_nq, d_in_ids, d_in_d, d_in_len, 0, nullptr, nullptr,
                       nullptr, d_rec_ids, d_rec_d, d_rec_n, cap);
    if (rc) return rc;
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

extern "C" int wv_index_bq_rescore(wv_index* idx, const uint64_t* d_ids, const int32_t* d_len, float* d_E,
                                   void* stream) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->bq_nq <= 0) return set_err(WV_ERR_INVALID, "bq_rescore: no batch begun");
    hipStream_t s = (hipStream_t)stream;  // NULL: the null stream (ordered with the caller's default-stream work)
    int rc = bq_rescore(idx, s, d_ids, d_len, d_E);
    if (rc) return rc;
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

extern "C" int wv_bq_final(int32_t device, int64_t nq, int32_t R, int32_t k, int32_t world, uint64_t id_stride,
                           const uint64_t* d_ids, const int32_t* d_len, const float* d_E, uint64_t* d_out_ids,
                           float* d_out_d, int32_t* d_out_n, void* stream) {
    HIPCHK(hipSetDevice(device));
    if (nq <= 0) return WV_OK;
    if (k <= 0 || R < k || world < 1) return set_err(WV_ERR_INVALID, "bq_final: invalid k / R / world");
    hipStream_t s = (hipStream_t)stream;
    std::vector<int32_t> id((size_t)nq);
    for (int64_t i = 0; i < nq; i++) id[i] = (int32_t)i;
    DBuf ql;
    HIPCHK(ql.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(hipMemcpyAsync(ql.p, id.data(), (size_t)nq * sizeof(int32_t), hipMemcpyHostToDevice, s));
    int rc = bq_final(s, nq, R, k, world, id_stride, ql.as<int32_t>(), d_ids, d_len, d_E, d_out_ids, d_out_d, d_out_n);
    HIPCHK(hipStreamSynchronize(s));  // ql is freed on return
    ql.release();
    return rc;
}

// ---------------------------------------------------------------------------
// product quantizer
// ---------------------------------------------------------------------------

// Go math/rand/v2 PCG-DXSM + Rand.IntN / Float64 / Shuffle (the Go standard
// library's published algorithm), as kmeans.temporaryData.init seeds it:
// rand.New(rand.NewPCG(seed, 0x385ab5285169b1ac)) (kmeans/kmeans.go:50).
struct GoPCG {
    uint64_t hi, lo;
    uint64_t next_u64() {
        const uint64_t mulHi = 2549297995355413924ULL, mulLo = 4865540595714422341ULL;
        const uint64_t incHi = 6364136223846793005ULL, incLo = 1442695040888963407ULL;
        __uint128_t m = (__uint128_t)lo * mulLo;
        uint64_t h = (uint64_t)(m >> 64), l = (uint64_t)m;
        h += hi * mulLo + lo * mulHi;
        __uint128_t sum = (__uint128_t)l + incLo;
        l = (uint64_t)sum;
        h = h + incHi + (uint64_t)(sum >> 64);
        lo = l;
        hi = h;
        const uint64_t cheapMul = 0xda942042e4dd58b5ULL;  // DXSM output
        h ^= h >> 32;
        h *= cheapMul;
        h ^= h >> 48;
        h *= (l | 1);
        return h;
    }
    uint64_t u64n(uint64_t n) {
        if ((n & (n - 1)) == 0) return next_u64() & (n - 1);
        __uint128_t m = (__uint128_t)next_u64() * n;
        uint64_t h = (uint64_t)(m >> 64), l = (uint64_t)m;
        if (l < n) {
            const uint64_t thresh = (0 - n) % n;
            while (l < thresh) {
                m = (__uint128_t)next_u64() * n;
                h = (uint64_t)(m >> 64);
                l = (uint64_t)m;
            }
        }
        return h;
    }
    double f64() { return (double)((next_u64() << 11) >> 11) / 9007199254740992.0; }
};

// kmeans.randomSubset (kmeans/kmeans.go:238-274)
static std::vector<int64_t> random_subset(GoPCG& r, int64_t n, int k) {
    std::vector<int64_t> out((size_t)k);
    if (k > n / 2) {  // r.Perm(n)[:k]
        std::vector<int64_t> p((size_t)n);
        for (int64_t i = 0; i < n; i++) p[i] = i;
        for (int64_t i = n - 1; i > 0; i--) std::swap(p[i], p[(size_t)r.u64n((uint64_t)(i + 1))]);
        std::copy(p.begin(), p.begin() + k, out.begin());
        return out;
    }
    std::unordered_map<int64_t, double> rank;
    std::vector<int64_t> keys;
    while ((int)rank.size() < k) {  // m[r.IntN(n)] = r.Float64()
        const int64_t i = (int64_t)r.u64n((uint64_t)n);
        const double v = r.f64();
        if (!rank.count(i)) keys.push_back(i);
        rank[i] = v;
    }
    std::stable_sort(keys.begin(), keys.end(), [&](int64_t a, int64_t b) { return rank[a] < rank[b]; });
    std::copy(keys.begin(), keys.end(), out.begin());
    return out;
}

// NewProductQuantizer validation (product_quantization.go:206-239)
static int pq_validate(wv_index* idx) {
    if (idx->pq_m <= 0) return set_err(WV_ERR_INVALID, "segments cannot be 0 nor negative");
    if (idx->pq_ks > 256)
        return set_err(WV_ERR_INVALID, "centroids should not be higher than 256. Attempting to use %d", idx->pq_ks);
    if (idx->pq_ks <= 0) return set_err(WV_ERR_INVALID, "centroids must be positive");
    if (idx->dims == 0) return set_err(WV_ERR_INVALID, "pq: dimensions not set yet");
    if (idx->dims % idx->pq_m != 0) return set_err(WV_ERR_INVALID, "segments should be an integer divisor of dimensions");
    idx->pq_ds = idx->dims / idx->pq_m;
    if (idx->pq_ds > 32) return set_err(WV_ERR_UNSUPPORTED, "pq: segment length %d > 32", idx->pq_ds);
    return WV_OK;
}

static int pq_alloc(wv_index* idx) {
    if (!idx->pq_centers)
        HIPCHK(hipMalloc(&idx->pq_centers, (size_t)idx->pq_m * idx->pq_ks * idx->pq_ds * sizeof(float)));
    if (!idx->pq_codes && idx->cap > 0) {
        const int64_t mw = pq_mwp(idx->pq_m);
        HIPCHK(hipMalloc(&idx->pq_codes, (size_t)mw * idx->cap * sizeof(uint32_t)));
        HIPCHK(hipMemsetAsync(idx->pq_codes, 0, (size_t)mw * idx->cap * sizeof(uint32_t), idx->stream));
    }
    return WV_OK;
}

static int pq_encode_all(wv_index* idx) {
    launch_pq_encode(idx, idx->hiwater, nullptr);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(idx->stream));
    idx->pq_trained = 1;
    return WV_OK;
}

extern "C" int wv_index_pq_fit(wv_index* idx, uint64_t seed) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->compression != WV_COMPRESSION_PQ) return set_err(WV_ERR_INVALID, "pq_fit: index is not PQ-compressed");
    int rc = pq_validate(idx);
    if (rc) return rc;
    const int m = idx->pq_m, K = idx->pq_ks, ds = idx->pq_ds;
    hipStream_t s = idx->stream;
    // training data: ProductQuantizer.Fit truncates to trainingLimit (:379-381)
    std::vector<uint32_t> tslots;
    for (int64_t sl = 0; sl < idx->hiwater; sl++)
        if (idx->h_present[sl]) tslots.push_back((uint32_t)sl);
    int64_t n = (int64_t)tslots.size();
    if (idx->pq_training_limit > 0 && n > idx->pq_training_limit) n = idx->pq_training_limit;
    if (n < K) return set_err(WV_ERR_INVALID, "not enough data to fit k-means");  // kmeans.go:459-461
    rc = pq_alloc(idx);
    if (rc) return rc;
    // T = the n training rows (gathered, dpad stride)
    DBuf T, sub, asg, nbi, nbd, chg, act;
    const int64_t ldt = idx->dpad;
    HIPCHK(T.ensure((size_t)n * ldt * sizeof(float)));
    {
        // contiguous copy when the first n present slots are 0..n-1, else a gather
        bool contiguous = true;
        for (int64_t i = 0; i < n; i++)
            if (tslots[i] != (uint32_t)i) { contiguous = false; break; }
        if (contiguous) {
            HIPCHK(hipMemcpyAsync(T.p, idx->X, (size_t)n * ldt * sizeof(float), hipMemcpyDeviceToDevice, s));
        } else {
            for (int64_t i = 0; i < n; i++)
                HIPCHK(hipMemcpyAsync(T.as<float>() + i * ldt, idx->X + (int64_t)tslots[i] * ldt, ldt * sizeof(float),
                                      hipMemcpyDeviceToDevice, s));
        }
    }
    float* C = idx->pq_centers;
    const size_t lds_c = (size_t)K * ds * sizeof(float);
    if (K == 1) {  // computeCentroid (kmeans.go:447-452): every row in cluster 0
        HIPCHK(asg.ensure((size_t)m * n * sizeof(uint32_t)));
        HIPCHK(hipMemsetAsync(asg.p, 0, (size_t)m * n * sizeof(uint32_t), s));
        const size_t lds_u = (size_t)K * ds * sizeof(double) + KM_T * sizeof(uint32_t) + (size_t)KM_T * ds * sizeof(float);
        k_km_update_centers<<<m, KM_T, lds_u, s>>>(T.as<float>(), ldt, n, K, ds, asg.as<uint32_t>(), nullptr, C);
        HIPCHK(hipGetLastError());
        return pq_encode_all(idx);
    }
    // initializeRandom (:279-299): per segment its own PCG stream
    std::vector<int64_t> hsub((size_t)m * K);
    for (int sg = 0; sg < m; sg++) {
        GoPCG r{seed + (uint64_t)sg, 0x385ab5285169b1acULL};
        std::vector<int64_t> ss = random_subset(r, n, K);
        std::copy(ss.begin(), ss.end(), hsub.begin() + (size_t)sg * K);
    }
    HIPCHK(sub.ensure(hsub.size() * sizeof(int64_t)));
    HIPCHK(hipMemcpyAsync(sub.p, hsub.data(), hsub.size() * sizeof(int64_t), hipMemcpyHostToDevice, s));
    {
        const int64_t tot = (int64_t)m * K * ds;
        k_km_gather_centers<<<(unsigned)((tot + 255) / 256), 256, 0, s>>>(T.as<float>(), ldt, sub.as<int64_t>(), m, K, ds,
                                                                          C);
    }
    HIPCHK(asg.ensure((size_t)m * n * sizeof(uint32_t)));
    HIPCHK(nbi.ensure((size_t)m * K * (K - 1) * sizeof(uint32_t)));
    HIPCHK(nbd.ensure((size_t)m * K * (K - 1) * sizeof(float)));
    HIPCHK(chg.ensure((size_t)m * sizeof(unsigned long long)));
    HIPCHK(act.ensure((size_t)m * sizeof(int32_t)));
    const int iteration_threshold = 10;  // KMeansEncoder.Fit: km.IterationThreshold = 10
    const float delta_threshold = 0.01f; // km.DeltaThreshold = 0.01
    std::vector<int32_t> active((size_t)m, iteration_threshold > 1 ? 1 : 0);
    HIPCHK(hipMemcpyAsync(act.p, active.data(), (size_t)m * sizeof(int32_t), hipMemcpyHostToDevice, s));
    const dim3 rgrid((unsigned)((n + 255) / 256), (unsigned)m);
    if (lds_c > 64 * 1024) {
        HIPCHK(hipFuncSetAttribute((const void*)k_km_assign_brute, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_c));
        HIPCHK(hipFuncSetAttribute((const void*)k_km_assign_prune, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_c));
        for (const void* f : {(const void*)k_pq_encode<0>, (const void*)k_pq_encode<1>, (const void*)k_pq_encode<2>,
                              (const void*)k_pq_encode<4>, (const void*)k_pq_encode<8>, (const void*)k_pq_encode<16>})
            HIPCHK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_c));
    }
    const size_t lds_u = (size_t)K * ds * sizeof(double) + KM_T * sizeof(uint32_t) + (size_t)KM_T * ds * sizeof(float);
    if (lds_u > 64 * 1024)
        HIPCHK(hipFuncSetAttribute((const void*)k_km_update_centers, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_u));
    k_km_assign_brute<<<rgrid, 256, lds_c, s>>>(T.as<float>(), ldt, n, K, ds, C, idx->variant, nullptr, asg.as<uint32_t>());
    k_km_update_centers<<<m, KM_T, lds_u, s>>>(T.as<float>(), ldt, n, K, ds, asg.as<uint32_t>(), nullptr, C);
    HIPCHK(hipGetLastError());
    int iterations = 1;  // initializeRandom counts as the first iteration (Metrics.update)
    std::vector<unsigned long long> hchg((size_t)m);
    while (iterations < iteration_threshold) {
        bool any = false;
        for (int sg = 0; sg < m; sg++) any = any || active[sg];
        if (!any) break;
        k_km_neighbors<<<dim3((unsigned)K, (unsigned)m), KM_T, 0, s>>>(C, K, ds, idx->variant, act.as<int32_t>(),
                                                                       nbi.as<uint32_t>(), nbd.as<float>());
        HIPCHK(hipMemsetAsync(chg.p, 0, (size_t)m * sizeof(unsigned long long), s));
        k_km_assign_prune<<<rgrid, 256, lds_c, s>>>(T.as<float>(), ldt, n, K, ds, C, idx->variant, nbi.as<uint32_t>(),
                                                    nbd.as<float>(), act.as<int32_t>(), asg.as<uint32_t>(),
                                                    chg.as<unsigned long long>());
        k_km_update_centers<<<m, KM_T, lds_u, s>>>(T.as<float>(), ldt, n, K, ds, asg.as<uint32_t>(), act.as<int32_t>(),
                                                   C);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(hchg.data(), chg.p, (size_t)m * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        iterations++;
        for (int sg = 0; sg < m; sg++) {
            // kmeans.go:490: float32(changes) <= DeltaThreshold * float32(n)
            if (active[sg] && ((float)hchg[sg] <= delta_threshold * (float)n || iterations >= iteration_threshold))
                active[sg] = 0;
        }
        HIPCHK(hipMemcpyAsync(act.p, active.data(), (size_t)m * sizeof(int32_t), hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    T.release(); sub.release(); asg.release(); nbi.release(); nbd.release(); chg.release(); act.release();
    return pq_encode_all(idx);
}

extern "C" int wv_index_pq_set_centers(wv_index* idx, const float* centers, int64_t n_floats) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->compression != WV_COMPRESSION_PQ) return set_err(WV_ERR_INVALID, "pq: index is not PQ-compressed");
    int rc = pq_validate(idx);
    if (rc) return rc;
    if (n_floats != (int64_t)idx->pq_m * idx->pq_ks * idx->pq_ds) return set_err(WV_ERR_INVALID, "pq: codebook size mismatch");
    rc = pq_alloc(idx);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(idx->pq_centers, centers, (size_t)n_floats * sizeof(float), hipMemcpyHostToDevice, idx->stream));
    return pq_encode_all(idx);
}

extern "C" int wv_index_pq_centers(wv_index* idx, float* out, int64_t n_floats) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (!idx->pq_trained) return set_err(WV_ERR_QUANTIZER, "quantizer not initialized");
    if (n_floats != (int64_t)idx->pq_m * idx->pq_ks * idx->pq_ds) return set_err(WV_ERR_INVALID, "pq: codebook size mismatch");
    HIPCHK(hipMemcpyAsync(out, idx->pq_centers, (size_t)n_floats * sizeof(float), hipMemcpyDeviceToHost, idx->stream));
    HIPCHK(hipStreamSynchronize(idx->stream));
    return WV_OK;
}

extern "C" int wv_index_pq_codes(wv_index* idx, uint8_t* out, int64_t n) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (!idx->pq_trained) return set_err(WV_ERR_QUANTIZER, "quantizer not initialized");
    if (round_up(n, 256) > idx->cap) return set_err(WV_ERR_INVALID, "pq_codes: n beyond capacity");
    const int64_t mw = pq_mwp(idx->pq_m);
    const int64_t npad = round_up(n, 256);
    std::vector<uint32_t> h((size_t)mw * npad);
    HIPCHK(hipMemcpyAsync(h.data(), idx->pq_codes, (size_t)mw * npad * sizeof(uint32_t), hipMemcpyDeviceToHost, idx->stream));
    HIPCHK(hipStreamSynchronize(idx->stream));
    for (int64_t r = 0; r < n; r++)
        for (int sg = 0; sg < idx->pq_m; sg++)
            out[r * idx->pq_m + sg] = (uint8_t)(h[(size_t)pq_code_word(r, sg, pq_g16(idx->pq_m))] >> (8 * (sg & 3)));
    return WV_OK;
}

extern "C" int wv_index_pq_info(wv_index* idx, int32_t* out) {
    if (!idx || !out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    out[0] = idx->pq_m; out[1] = idx->pq_ks; out[2] = idx->pq_ds; out[3] = idx->pq_trained;
    return WV_OK;
}

extern "C" int wv_index_pq_distance(wv_index* idx, const float* query, int64_t d, const uint8_t* codes, int64_t n,
                                    float* out) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (!idx->pq_trained) return set_err(WV_ERR_QUANTIZER, "quantizer not initialized");
    if (d != idx->dims) return set_err(WV_ERR_VECTOR_LENGTH, "%lld vs %d: vector lengths don't match", (long long)d, idx->dims);
    if (n <= 0) return WV_OK;
    hipStream_t s = idx->stream;
    const int m = idx->pq_m, K = idx->pq_ks;
    const int64_t mw = pq_mwp(m);
    DBuf Q, L, Cd, E, B, ql;
    HIPCHK(Q.ensure((size_t)d * sizeof(float)));
    HIPCHK(hipMemcpyAsync(Q.p, query, (size_t)d * sizeof(float), hipMemcpyHostToDevice, s));
    HIPCHK(L.ensure((size_t)m * K * sizeof(float)));
    k_pq_lut<<<(unsigned)(((int64_t)m * K + 255) / 256), 256, 0, s>>>(Q.as<float>(), d, 1, m, K, idx->pq_ds,
                                                                      idx->metric == WV_METRIC_L2_SQUARED ? L2 : DOT,
                                                                      idx->pq_centers, L.as<float>());
    // pack the given codes [n][m] into the plane layout
    const int64_t ld = round_up(n, 256);
    std::vector<uint32_t> h((size_t)mw * ld, 0);
    for (int64_t r = 0; r < n; r++)
        for (int sg = 0; sg < m; sg++) h[(size_t)pq_code_word(r, sg, pq_g16(m))] |= (uint32_t)codes[r * m + sg] << (8 * (sg & 3));
    HIPCHK(Cd.ensure(h.size() * sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(Cd.p, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    std::vector<uint32_t> ones((size_t)(ld / 32), 0xFFFFFFFFu);
    DBuf V;
    HIPCHK(V.ensure(ones.size() * sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(V.p, ones.data(), ones.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    HIPCHK(E.ensure((size_t)ld * sizeof(float)));
    HIPCHK(B.ensure((size_t)(ld / 256) * sizeof(float)));
    int32_t zero = 0;
    HIPCHK(ql.ensure(sizeof(int32_t)));
    HIPCHK(hipMemcpyAsync(ql.p, &zero, sizeof(int32_t), hipMemcpyHostToDevice, s));
    const int wrapm = idx->metric == WV_METRIC_L2_SQUARED ? L2 : idx->metric == WV_METRIC_DOT ? DOT : COSINE;
    dim3 grid(1, (unsigned)((n + 256 * PQ_RPT - 1) / (256 * PQ_RPT)));
    if (K == 256)
        k_pq_adc<256><<<grid, 256, (size_t)PQ_CH * K * sizeof(float), s>>>(Cd.as<uint32_t>(), pq_g16(m), m, K, V.as<uint32_t>(), n,
                                                                       L.as<float>(), ql.as<int32_t>(), wrapm, ld,
                                                                       E.as<float>(), B.as<float>());
    else
        k_pq_adc<0><<<grid, 256, (size_t)PQ_CH * K * sizeof(float), s>>>(Cd.as<uint32_t>(), pq_g16(m), m, K, V.as<uint32_t>(), n,
                                                                     L.as<float>(), ql.as<int32_t>(), wrapm, ld,
                                                                     E.as<float>(), B.as<float>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, E.p, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

// hnsw.flatSearch over the PQ codes (flat_search.go:28-141, one worker) with
// optional h.rescore (search.go:1047-1110, one worker).  limit = rescore ?
// max(rescore_limit, k) : k.  Outputs [nq][k].
// bytes already held by the first distance buffer (counted as available
// when sizing the groups: ensure() reuses it)
static size_t Eb0_bytes(const wv_index* idx) { return idx->rE.bytes; }

// replay stream + events (created at the first quantized search that uses them)
static int ensure_aux(wv_index* idx) {
    if (idx->aux) return WV_OK;
    HIPCHK(hipStreamCreateWithFlags(&idx->aux, hipStreamNonBlocking));
    for (hipEvent_t* e : {&idx->evd[0], &idx->evd[1], &idx->evr[0], &idx->evr[1]})
        HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    return WV_OK;
}

static int rq_encode_queries(wv_index* idx, hipStream_t s, int64_t nq);
static int rq_dist(wv_index* idx, hipStream_t s, const uint32_t* valid, int64_t q0, int F, int64_t ld, float* E,
                   float* bmin);

// SQ query codes: idx->qn (prepared, normalised for cosine) -> group-tiled sqq / sqm
static int sq_encode_queries(wv_index* idx, hipStream_t s, int64_t nq) {
    const int64_t nq32 = round_up(nq, RQ_QPB);
    HIPCHK(idx->sqq.ensure((size_t)nq32 * idx->sq_Dq));
    HIPCHK(idx->sqm.ensure((size_t)nq32 * sizeof(uint2)));
    if (nq32 > nq) {
        HIPCHK(hipMemsetAsync(idx->sqq.p, 0, (size_t)nq32 * idx->sq_Dq, s));
        HIPCHK(hipMemsetAsync(idx->sqm.p, 0, (size_t)nq32 * sizeof(uint2), s));
    }
    k_sq_encode<1><<<(unsigned)((nq + 3) / 4), 256, 0, s>>>(idx->qn.as<float>(), idx->dpad, nq, idx->dims, nullptr,
                                                             idx->sq_Dq, idx->sq_a, idx->sq_b, idx->sqq.as<uint4>(),
                                                             idx->sqm.as<uint2>());
    HIPCHK(hipGetLastError());
    return WV_OK;
}

// hnsw.flatSearch over the compressed vectors (flat_search.go:28-141, one
// worker) + optional h.rescore (search.go:1047-1110, one worker).  The
// compressor distance of every (query, allowed row) is materialised per query
// group (k_pq_adc / k_sq_dist / k_rq*_dist / k_bq_dist, with 256-row block
// minima), the worker heap (addResult == insertToHeap with `limit`) is
// replayed in id order by k_replay_scan on the aux stream beside the next
// group's distance kernel, k_pq_finish merges it into the result heap in pop
// order (and trims SQ / RQ to `trim`), k_rescore + k_pq_rescore_final rescore.
// Outputs [nq][k].
static int search_hnsw(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k, int limit,
                       int trim, int rescore, const uint32_t* valid, uint64_t* o_ids, float* o_d, int32_t* o_n) {
    const int comp = idx->rq_bits ? WV_COMPRESSION_RQ8 : idx->compression;
    if (comp == WV_COMPRESSION_BQ && (qd + 63) / 64 != idx->words)  // HammingBitwise (distancer/hamming.go:63-66)
        return set_err(WV_ERR_VECTOR_LENGTH, "both vectors should have the same len");
    if (comp == WV_COMPRESSION_SQ && qd != idx->dims)  // DistanceBetweenCompressedVectors (scalar_quantization.go:46-49)
        return set_err(WV_ERR_INVALID, "vector lengths don't match: %lld vs %d", (long long)qd + 8, idx->dims + 8);
    if (qd != idx->dims)
        return set_err(WV_ERR_VECTOR_LENGTH, "%lld vs %d: vector lengths don't match", (long long)qd, idx->dims);
    if (k <= 0) return set_err(WV_ERR_INVALID, "k must be positive (reference heap Top() on empty queue)");
    if (comp == WV_COMPRESSION_SQ && idx->metric == WV_METRIC_HAMMING)  // scalar_quantization.go:56
        return set_err(WV_ERR_UNSUPPORTED, "Distance not supported yet hamming");
    if (comp == WV_COMPRESSION_SQ && !idx->sq_ready) return set_err(WV_ERR_QUANTIZER, "quantizer not initialized");
    if (comp == WV_COMPRESSION_PQ && !idx->pq_trained) return set_err(WV_ERR_QUANTIZER, "quantizer not initialized");
    if (idx->rq_bits && !idx->rq_ready) return set_err(WV_ERR_QUANTIZER, "quantizer not initialized");
    if (limit < k) limit = k;
    const int R = limit;
    if (R > 8192) return set_err(WV_ERR_UNSUPPORTED, "limit %d > 8192", R);
    const int64_t nq_pad = round_up(nq, QB);
    int rc = prepare_queries(idx, s, d_qraw, nq, nq_pad);
    if (rc) return rc;
    const float* Qn = idx->qn.as<float>();
    idx->stats.queries += (uint64_t)nq;
    idx->stats.batches++;
    // per-compressor query state
    if (comp == WV_COMPRESSION_PQ) {
        const int m = idx->pq_m, K = idx->pq_ks;
        HIPCHK(idx->lut.ensure((size_t)nq * m * K * sizeof(float)));
        k_pq_lut<<<(unsigned)((nq * m * K + 255) / 256), 256, 0, s>>>(Qn, idx->dpad, nq, m, K, idx->pq_ds,
                                                                       idx->metric == WV_METRIC_L2_SQUARED ? L2 : DOT,
                                                                       idx->pq_centers, idx->lut.as<float>());
        HIPCHK(hipGetLastError());
    } else if (comp == WV_COMPRESSION_RQ8) {
        rc = rq_encode_queries(idx, s, nq);
        if (rc) return rc;
    } else if (comp == WV_COMPRESSION_SQ) {
        rc = sq_encode_queries(idx, s, nq);
        if (rc) return rc;
    } else if (comp == WV_COMPRESSION_BQ) {
        HIPCHK(idx->qcodes.ensure((size_t)nq * idx->words * sizeof(uint64_t)));
        const int64_t nt = nq * idx->words;
        k_bq_encode_rows<<<(unsigned)((nt + 255) / 256), 256, 0, s>>>(Qn, idx->dpad, nq, idx->dims, nullptr,
                                                                       idx->qcodes.as<uint64_t>(), nq);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(idx->ident.ensure((size_t)nq * sizeof(int32_t)));
    {
        std::vector<int32_t> id((size_t)nq);
        for (int64_t i = 0; i < nq; i++) id[i] = (int32_t)i;
        HIPCHK(hipMemcpyAsync(idx->ident.p, id.data(), (size_t)nq * sizeof(int32_t), hipMemcpyHostToDevice, s));
    }
    const int32_t* qlist = idx->ident.as<int32_t>();
    const int64_t nslots = idx->hiwater;
    const int64_t ld = std::max<int64_t>(round_up(nslots, EBLK), EBLK);
    HIPCHK(idx->ascI.ensure((size_t)nq * R * sizeof(uint64_t)));
    HIPCHK(idx->ascD.ensure((size_t)nq * R * sizeof(float)));
    HIPCHK(idx->ascN.ensure((size_t)nq * sizeof(int32_t)));
    const int wrapm = idx->metric == WV_METRIC_L2_SQUARED ? L2 : idx->metric == WV_METRIC_DOT ? DOT : COSINE;
    // the queries the exact heap replay below takes (every query, or the ones
    // the PQ candidate path flags), and whether its outputs go by query
    int64_t nrep = nq;
    int rep_by_query = 0;
    if (comp == WV_COMPRESSION_PQ && idx->pq_cand && R + 1 <= 64) {
        // minima-only PQ search: block minima of every query (no B x N matrix),
        // candidate blocks, exact ADC of their rows, strict order -> asc
        const int m = idx->pq_m, K = idx->pq_ks;
        const int64_t nblk = ld / EBLK;
        HIPCHK(idx->rB.ensure((size_t)nq * nblk * sizeof(float)));
        HIPCHK(idx->pqZero.ensure((size_t)std::max<int64_t>(nq, 1) * sizeof(float4)));
        HIPCHK(idx->qsCand.ensure((size_t)nq * 64 * sizeof(uint32_t)));
        HIPCHK(idx->qsNc.ensure((size_t)nq * sizeof(int32_t)));
        HIPCHK(idx->qsEps.ensure((size_t)nq * sizeof(float)));
        HIPCHK(idx->qsFlags.ensure((size_t)nq * sizeof(int32_t)));
        HIPCHK(idx->oF.ensure((size_t)nq * sizeof(int32_t)));
        HIPCHK(idx->qsList.ensure((size_t)nq * sizeof(int32_t)));
        HIPCHK(idx->flCtr.ensure(2 * sizeof(uint32_t)));
        HIPCHK(hipMemsetAsync(idx->pqZero.p, 0, (size_t)std::max<int64_t>(nq, 1) * sizeof(float4), s));
        const size_t lds_adc = (size_t)PQ_CH * K * sizeof(float);
        dim3 grid2((unsigned)((nq + 1) / 2), (unsigned)((nslots + 256 * PQ_RPT - 1) / (256 * PQ_RPT)));
        if (idx->timing) HIPCHK(hipEventRecord(idx->ev0, s));
#define WV_ADC2M(KCV)                                                                                        \
    do {                                                                                                     \
        HIPCHK(hipFuncSetAttribute((const void*)k_pq_adc2<KCV, PQ_RPT>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                   (int)(2 * lds_adc)));                                                     \
        k_pq_adc2<KCV, PQ_RPT><<<grid2, 256, 2 * lds_adc, s>>>(idx->pq_codes, pq_g16(m), m, K, valid, nslots,  \
                                                               idx->lut.as<float>(), qlist, (int)nq, wrapm, ld, \
                                                               nullptr, idx->rB.as<float>());                \
    } while (0)
        if (K == 256) WV_ADC2M(256);
        else WV_ADC2M(0);
#undef WV_ADC2M
        HIPCHK(hipGetLastError());
        if (idx->timing) HIPCHK(hipEventRecord(idx->ev1, s));
        idx->stats.last_group_queries = (uint64_t)nq;
        // blocks whose minimum is within a rounding-size eps of the (R+1)-th
        // smallest (DOT: the key is the value; zero norms: eps = 4u)
        const uint32_t* z = idx->pqZero.as<uint32_t>();
        k_blk_select<2><<<(unsigned)((nq + 3) / 4), 256, 0, s>>>(
            idx->rB.as<float>(), nblk, nblk, (int)nq, R, DOT, idx->pqZero.as<float4>(), z, z + 3, 0.f, 0.f,
            idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(), idx->qsFlags.as<int32_t>(), idx->qsEps.as<float>(),
            nullptr, nullptr, nullptr, nullptr);
        HIPCHK(hipGetLastError());
        int32_t* pflag = idx->oF.as<int32_t>();
#define WV_PQC(KCV) k_pq_cand<KCV><<<(unsigned)nq, 256, 0, s>>>(idx->pq_codes, pq_g16(m), m, K, valid, nslots, idx->lut.as<float>(), idx->rB.as<float>(), nblk, idx->qsCand.as<uint32_t>(), 64, idx->qsNc.as<int32_t>(), idx->qsFlags.as<int32_t>(), R, wrapm, idx->id_base, idx->ascI.as<uint64_t>(), idx->ascD.as<float>(), idx->ascN.as<int32_t>(), pflag)
        if (K == 256) WV_PQC(256);
        else WV_PQC(0);
#undef WV_PQC
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemsetAsync(idx->flCtr.p, 0, 2 * sizeof(uint32_t), s));
        k_flag_list<<<(unsigned)((nq + 255) / 256), 256, 0, s>>>(pflag, (int)nq, idx->qsList.as<int32_t>(),
                                                                  idx->flCtr.as<uint32_t>(), 0);
        HIPCHK(hipGetLastError());
        uint32_t nf = 0;
        HIPCHK(hipMemcpyAsync(&nf, idx->flCtr.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        nrep = nf;
        rep_by_query = 1;
        qlist = idx->qsList.as<int32_t>();
        idx->stats.replayed_queries += nf;
    } else if (comp == WV_COMPRESSION_PQ) {
        idx->stats.replayed_queries += (uint64_t)nq;
    }
    // query groups sized to the free HBM (two distance buffers), multiples of
    // RQ_QPB for the thread-per-row kernels
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    const int64_t have = (int64_t)(Eb0_bytes(idx) + free_b / 4);
    const int64_t budget = std::max<int64_t>(std::min<int64_t>(16ll << 30, have), 1ll << 30);
    int64_t G = std::max<int64_t>(1, std::min<int64_t>(std::max<int64_t>(nrep, 1), budget / (ld * 4)));
    if (comp != WV_COMPRESSION_PQ) {
        G = std::max<int64_t>(RQ_QPB, G / RQ_QPB * RQ_QPB);
        G = std::min<int64_t>(G, round_up(nq, RQ_QPB));
    }
    if (!rep_by_query) idx->stats.last_group_queries = (uint64_t)std::min<int64_t>(G, nq);
    rc = ensure_aux(idx);
    if (rc) return rc;
    DBuf* Eb[2] = {&idx->rE, &idx->rE2};
    DBuf* Bb[2] = {&idx->rB, &idx->rB2};
    if (nrep > 0)
        for (int b = 0; b < 2; b++) {
            HIPCHK(Eb[b]->ensure((size_t)G * ld * sizeof(float)));
            HIPCHK(Bb[b]->ensure((size_t)G * (ld / EBLK) * sizeof(float)));
        }
    const size_t lds_rep = (size_t)R * sizeof(uint64_t) + 64 * sizeof(float) + (size_t)R * sizeof(float) + 16;
    if (lds_rep > 64 * 1024)
        HIPCHK(hipFuncSetAttribute((const void*)k_replay_scan, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_rep));
    int64_t gi = 0;
    for (int64_t g0 = 0; g0 < nrep; g0 += G, gi++) {
        const int F = (int)std::min<int64_t>(G, nrep - g0);
        const int b = (int)(gi & 1);
        float* E = Eb[b]->as<float>();
        float* Bm = Bb[b]->as<float>();
        if (gi >= 2) HIPCHK(hipStreamWaitEvent(s, idx->evr[b], 0));
        const bool time_it = idx->timing && g0 == 0 && !rep_by_query;
        if (time_it) HIPCHK(hipEventRecord(idx->ev0, s));
        if (comp == WV_COMPRESSION_PQ) {
            const int m = idx->pq_m, K = idx->pq_ks;
            const size_t lds_adc = (size_t)PQ_CH * K * sizeof(float);
            dim3 grid((unsigned)F, (unsigned)((nslots + 256 * PQ_RPT - 1) / (256 * PQ_RPT)));
            if (idx->pq_adc == 2) {  // two queries per workgroup: 2 x the LUT chunk (64 KiB at ks = 256)
                dim3 grid2((unsigned)((F + 1) / 2), grid.y);
#define WV_ADC2(KCV, RPTV)                                                                                   \
    do {                                                                                                     \
        HIPCHK(hipFuncSetAttribute((const void*)k_pq_adc2<KCV, RPTV>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                   (int)(2 * lds_adc)));                                                     \
        k_pq_adc2<KCV, RPTV><<<grid2, 256, 2 * lds_adc, s>>>(idx->pq_codes, pq_g16(m), m, K, valid, nslots,    \
                                                             idx->lut.as<float>(), qlist + g0, F, wrapm, ld, E, Bm); \
    } while (0)
                if (K == 256) WV_ADC2(256, PQ_RPT);
                else WV_ADC2(0, PQ_RPT);
#undef WV_ADC2
            } else if (K == 256)
                k_pq_adc<256><<<grid, 256, lds_adc, s>>>(idx->pq_codes, pq_g16(m), m, K, valid, nslots,
                                                         idx->lut.as<float>(), qlist + g0, wrapm, ld, E, Bm);
            else
                k_pq_adc<0><<<grid, 256, lds_adc, s>>>(idx->pq_codes, pq_g16(m), m, K, valid, nslots,
                                                       idx->lut.as<float>(), qlist + g0, wrapm, ld, E, Bm);
        } else if (comp == WV_COMPRESSION_RQ8) {
            rc = rq_dist(idx, s, valid, g0, F, ld, E, Bm);
            if (rc) return rc;
        } else if (comp == WV_COMPRESSION_SQ) {
            dim3 grid((unsigned)((F + RQ_QPB - 1) / RQ_QPB), (unsigned)(ld / 256));
            k_sq_dist<<<grid, 256, 0, s>>>(idx->sq_codes, idx->sq_meta, idx->sq_Dq, valid, nslots,
                                           idx->sqq.as<uint4>(), idx->sqm.as<uint2>(), g0, F, wrapm, idx->sq_a2,
                                           idx->sq_ab, idx->sq_ib2, ld, E, Bm);
        } else {  // BQ
            dim3 grid((unsigned)((F + RQ_QPB - 1) / RQ_QPB), (unsigned)(ld / 256));
            k_bq_dist<<<grid, 256, 0, s>>>(idx->codes, idx->cap, idx->words, valid, nslots, idx->qcodes.as<uint64_t>(),
                                           nq, g0, F, ld, E, Bm);
        }
        HIPCHK(hipGetLastError());
        if (time_it) HIPCHK(hipEventRecord(idx->ev1, s));
        HIPCHK(hipEventRecord(idx->evd[b], s));
        HIPCHK(hipStreamWaitEvent(idx->aux, idx->evd[b], 0));
        // the worker heap (addResult == insertToHeap) in id order, extracted ascending
        // (rows by list position, or by query for the PQ candidate path's flagged list)
        const int64_t ao = rep_by_query ? 0 : g0;
        k_replay_scan<<<F, 64, lds_rep, idx->aux>>>(E, Bm, valid, nslots, ld, qlist + g0, F, R, idx->id_base, nullptr,
                                                    nullptr, nullptr, 1, rep_by_query, R,
                                                    idx->ascI.as<uint64_t>() + ao * R, idx->ascD.as<float>() + ao * R,
                                                    idx->ascN.as<int32_t>() + ao, 0, 0, nullptr, nullptr, nullptr, 0);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(idx->evr[b], idx->aux));
    }
    for (int b = 0; b < 2 && b < gi; b++) HIPCHK(hipStreamWaitEvent(s, idx->evr[b], 0));
    qlist = idx->ident.as<int32_t>();
    HIPCHK(idx->cslot.ensure((size_t)nq * R * sizeof(uint32_t)));
    HIPCHK(idx->cn.ensure((size_t)nq * sizeof(int32_t)));
    const size_t lds_f = (size_t)R * (sizeof(uint64_t) + sizeof(float)) + 16;
    if (lds_f > 64 * 1024)
        HIPCHK(hipFuncSetAttribute((const void*)k_pq_finish, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_f));
    k_pq_finish<<<(unsigned)nq, 64, lds_f, s>>>(idx->ascI.as<uint64_t>(), idx->ascD.as<float>(), idx->ascN.as<int32_t>(),
                                                qlist, (int)nq, R, k, rescore, idx->id_base, o_ids, o_d, o_n,
                                                idx->cslot.as<uint32_t>(), idx->cn.as<int32_t>(), rescore ? trim : 0);
    HIPCHK(hipGetLastError());
    if (rescore) {
        HIPCHK(idx->candE.ensure((size_t)nq * R * sizeof(float)));
        const int64_t npairs = nq * R;
        const bool v5 = idx->variant == WV_VARIANT_AVX512;
#define WV_RS(M, V) k_rescore<M, V><<<(unsigned)((npairs + 63) / 64), 64, 0, s>>>(idx->X, idx->dpad, Qn, idx->dims, idx->cslot.as<uint32_t>(), (int)nq, R, idx->candE.as<float>())
        switch (idx->metric) {
        case WV_METRIC_L2_SQUARED: if (v5) WV_RS(L2, AVX512); else WV_RS(L2, AVX256); break;
        case WV_METRIC_DOT: if (v5) WV_RS(DOT, AVX512); else WV_RS(DOT, AVX256); break;
        case WV_METRIC_COSINE_DOT: if (v5) WV_RS(COSINE, AVX512); else WV_RS(COSINE, AVX256); break;
        default: WV_RS(HAMMING, AVX256); break;
        }
#undef WV_RS
        HIPCHK(hipGetLastError());
        const size_t lds_q = (size_t)(k + 1) * (sizeof(uint64_t) + sizeof(float)) + 16;
        if (lds_q > 64 * 1024)
            HIPCHK(hipFuncSetAttribute((const void*)k_pq_rescore_final, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_q));
        k_pq_rescore_final<<<(unsigned)nq, 64, lds_q, s>>>(idx->cslot.as<uint32_t>(), idx->candE.as<float>(),
                                                           idx->cn.as<int32_t>(), qlist, (int)nq, R, k, idx->id_base,
                                                           o_ids, o_d, o_n);
        HIPCHK(hipGetLastError());
    }
    if (idx->timing) {
        HIPCHK(hipStreamSynchronize(s));
        float ms = 0.f;
        hipEventElapsedTime(&ms, idx->ev0, idx->ev1);
        idx->stats.last_select_ms = ms;
    }
    return WV_OK;
}

// the PQ index behind SearchByVector: hnsw.flatSearch with limit =
// max(rescore_limit, k) when rescoring (the caller's ef), else k
static int search_pq(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k,
                     const uint32_t* valid, uint64_t* o_ids, float* o_d, int32_t* o_n) {
    const int rescore = idx->pq_rescore ? 1 : 0;
    const int R = rescore && idx->rescore_limit > k ? idx->rescore_limit : k;
    return search_hnsw(idx, s, d_qraw, nq, qd, k, R, 0, rescore, valid, o_ids, o_d, o_n);
}

// searchTimeEF (hnsw/search.go:44-76)
static int hnsw_search_ef(const wv_index* idx, int k) {
    int ef = idx->hnsw_ef;
    if (ef < 1) {  // autoEfFromK
        ef = k * idx->ef_factor;
        if (ef > idx->ef_max) ef = idx->ef_max;
        else if (ef < idx->ef_min) ef = idx->ef_min;
        if (k > ef) ef = k;
        return ef;
    }
    return ef < k ? k : ef;
}

// hnsw.SearchByVector's flat branch for a compressed index: limit / trim / rescore
static int search_hnsw_flat(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k,
                            const uint32_t* valid, uint64_t* o_ids, float* o_d, int32_t* o_n) {
    const bool sqrq = idx->compression == WV_COMPRESSION_SQ || idx->rq_bits != 0;
    // shouldRescore (search.go:182-189); a PQ index created with pq_rescore = 0 counts as doNotRescore
    bool rescore = idx->hnsw_rescore != 0 && !(sqrq && idx->rescore_limit == 0);
    if (idx->compression == WV_COMPRESSION_PQ && !idx->pq_rescore) rescore = false;
    const int limit = rescore ? hnsw_search_ef(idx, k) : k;  // flat_search.go:31-33
    const int trim = (sqrq && idx->rescore_limit >= k) ? idx->rescore_limit : 0;
    return search_hnsw(idx, s, d_qraw, nq, qd, k, limit, trim, rescore ? 1 : 0, valid, o_ids, o_d, o_n);
}

// ---------------------------------------------------------------------------
// scalar quantizer (compressionhelpers/scalar_quantization.go)
// ---------------------------------------------------------------------------
// a, b -> the float32 constants of the distance (NewScalarQuantizer :93-95),
// codes for the current capacity, every stored row encoded
static int sq_set(wv_index* idx, float a, float b) {
    const float codes2 = 65025.0f;  // codes * codes
    float t = a * a;
    idx->sq_a2 = t / codes2;
    t = a * b;
    idx->sq_ab = t / 255.0f;
    t = b * b;
    idx->sq_ib2 = t * (float)idx->dims;
    idx->sq_a = a;
    idx->sq_b = b;
    idx->sq_Dq = (int)round_up(idx->dims, 16);
    if (!idx->sq_codes && idx->cap > 0) {
        HIPCHK(hipMalloc(&idx->sq_codes, (size_t)idx->cap * idx->sq_Dq));
        HIPCHK(hipMalloc(&idx->sq_meta, (size_t)idx->cap * sizeof(uint2)));
        HIPCHK(hipMemsetAsync(idx->sq_codes, 0, (size_t)idx->cap * idx->sq_Dq, idx->stream));
        HIPCHK(hipMemsetAsync(idx->sq_meta, 0, (size_t)idx->cap * sizeof(uint2), idx->stream));
    }
    idx->sq_ready = 1;
    if (idx->hiwater > 0) {
        k_sq_encode<0><<<(unsigned)((idx->hiwater + 3) / 4), 256, 0, idx->stream>>>(
            idx->X, idx->dpad, idx->hiwater, idx->dims, nullptr, idx->sq_Dq, a, b, idx->sq_codes, idx->sq_meta);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(idx->stream));
    return WV_OK;
}

extern "C" int wv_index_sq_fit(wv_index* idx, int64_t training_limit) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->compression != WV_COMPRESSION_SQ) return set_err(WV_ERR_INVALID, "sq_fit: index is not SQ-compressed");
    if (idx->npresent == 0 || idx->dims == 0)  // hnsw/compress.go:34-36
        return set_err(WV_ERR_INVALID, "compress command cannot be executed before inserting some data");
    std::vector<int64_t> rows;
    for (int64_t sl = 0; sl < idx->hiwater; sl++) {
        if (!idx->h_present[sl]) continue;
        rows.push_back(sl);
        if (training_limit > 0 && (int64_t)rows.size() >= training_limit) break;
    }
    // NewScalarQuantizer (:73-97): b = data[0][0]; a grows with every new
    // minimum (a += b - x) or sets to the new range (a = x - b), in float32
    const int d = idx->dims;
    // one copy of the slot range holding the sample (padded rows, dpad stride)
    const int64_t span = rows.back() + 1;
    std::vector<float> buf((size_t)span * idx->dpad);
    HIPCHK(hipMemcpy(buf.data(), idx->X, buf.size() * sizeof(float), hipMemcpyDeviceToHost));
    float a = 0.f, b = 0.f;
    for (size_t i = 0; i < rows.size(); i++) {
        const float* row = buf.data() + (size_t)rows[i] * idx->dpad;
        if (i == 0) b = row[0];
        for (int j = 0; j < d; j++) {
            const float x = row[j];
            if (x < b) {
                const float t = b - x;
                a = a + t;
                b = x;
            } else if (x - b > a) {
                a = x - b;
            }
        }
    }
    return sq_set(idx, a, b);
}

extern "C" int wv_index_sq_restore(wv_index* idx, float a, float b) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->compression != WV_COMPRESSION_SQ) return set_err(WV_ERR_INVALID, "sq_restore: index is not SQ-compressed");
    if (a == 0.f) return set_err(WV_ERR_INVALID, "invalid range value while restoring SQ settings");
    if (idx->dims == 0) return set_err(WV_ERR_INVALID, "sq_restore: dimensions not set yet");
    return sq_set(idx, a, b);
}

extern "C" int wv_index_sq_info(wv_index* idx, float* out) {
    if (!idx || !out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    out[0] = idx->sq_a;
    out[1] = idx->sq_b;
    out[2] = (float)idx->sq_ready;
    out[3] = (float)(idx->dims + 8);
    return WV_OK;
}

extern "C" int wv_index_sq_codes(wv_index* idx, uint8_t* out, int64_t n) {
    if (!idx || !out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (!idx->sq_ready) return set_err(WV_ERR_QUANTIZER, "quantizer not initialized");
    if (n < 0 || n > idx->cap) return set_err(WV_ERR_INVALID, "sq_codes: n out of range");
    const int Dq = idx->sq_Dq, d = idx->dims, nch = Dq / 16;
    std::vector<uint8_t> tiles((size_t)round_up(std::max<int64_t>(n, 1), 256) * Dq);
    std::vector<uint2> meta((size_t)std::max<int64_t>(n, 1));
    HIPCHK(hipMemcpy(tiles.data(), idx->sq_codes, std::min<size_t>(tiles.size(), (size_t)idx->cap * Dq), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(meta.data(), idx->sq_meta, (size_t)n * sizeof(uint2), hipMemcpyDeviceToHost));
    for (int64_t r = 0; r < n; r++) {
        uint8_t* o = out + r * (d + 8);
        for (int e = 0; e < d; e++) {
            const int c = e / 16;
            o[e] = tiles[((size_t)((r >> 8) * nch + c) * 256 + (r & 255)) * 16 + (e & 15)];
        }
        const uint32_t v[2] = {meta[r].x, meta[r].y};
        for (int w = 0; w < 2; w++)
            for (int i = 0; i < 4; i++) o[d + 4 * w + i] = (uint8_t)(v[w] >> (24 - 8 * i));  // big endian
    }
    return WV_OK;
}

// ---------------------------------------------------------------------------
// rotational quantization: flat "rq-8" / "rq-1" (flat/quantizer.go:85-99)
// ---------------------------------------------------------------------------
static constexpr uint64_t kDefaultFastRotationSeed = 0x535ab5105169b1dfULL;  // fast_rotation.go:27

// NewFastRotation (fast_rotation.go:72-90) -> per-round gather tables, and the
// rq-1 rounding vector (binary_rotational_quantization.go:52-56); then the code
// store for the current capacity.
static int rq_init(wv_index* idx) {
    const int in_dim = (idx->rq_bits == 1 && idx->dims < 256) ? 256 : idx->dims;  // minCodeBits
    int D = 64;
    while (D < in_dim) D += 64;
    if (D > RQ_MAXD) return set_err(WV_ERR_UNSUPPORTED, "rq: output dimension %d > %d", D, RQ_MAXD);
    std::vector<uint16_t> src((size_t)RQ_ROUNDS * D);
    std::vector<float> sign((size_t)RQ_ROUNDS * D), rnd((size_t)D);
    GoPCG r{kDefaultFastRotationSeed, 0x385ab5285169b1acULL};
    std::vector<int> perm((size_t)D);
    for (int rd = 0; rd < RQ_ROUNDS; rd++) {
        for (int i = 0; i < D; i++) perm[i] = i;  // rng.Perm(n): Shuffle with uint64n
        for (int i = D - 1; i > 0; i--) std::swap(perm[i], perm[(size_t)r.u64n((uint64_t)(i + 1))]);
        std::vector<float> sg((size_t)D);
        for (int i = 0; i < D; i++) sg[i] = r.f64() < 0.5 ? -1.0f : 1.0f;  // randomSigns
        // swap (I, J): new[I] = sign[I] * old[J], new[J] = sign[J] * old[I]
        for (int p = 0; p < D / 2; p++) {
            const int a = perm[2 * p], b = perm[2 * p + 1];
            src[(size_t)rd * D + a] = (uint16_t)b;
            src[(size_t)rd * D + b] = (uint16_t)a;
        }
        for (int i = 0; i < D; i++) sign[(size_t)rd * D + i] = sg[i];
    }
    if (idx->rq_bits == 1) {
        GoPCG rr{kDefaultFastRotationSeed, 0x4f8ebf70e130707fULL};
        for (int i = 0; i < D; i++) {  // rng.Float32(): float32(Uint32()<<8>>8) / 2^24
            const uint32_t u = (uint32_t)(rr.next_u64() >> 32);
            rnd[i] = (float)((u << 8) >> 8) / 16777216.0f;
        }
    }
    HIPCHK(hipMalloc(&idx->rq_src, src.size() * sizeof(uint16_t)));
    HIPCHK(hipMalloc(&idx->rq_sign, sign.size() * sizeof(float)));
    HIPCHK(hipMalloc(&idx->rq_round, rnd.size() * sizeof(float)));
    HIPCHK(hipMemcpy(idx->rq_src, src.data(), src.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(idx->rq_sign, sign.data(), sign.size() * sizeof(float), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(idx->rq_round, rnd.data(), rnd.size() * sizeof(float), hipMemcpyHostToDevice));
    idx->rq_D = D;
    idx->rq_ready = 1;
    if (idx->cap > 0) {  // store already sized (reserve): allocate the codes for it
        const size_t cb = idx->rq_bits == 8 ? (size_t)idx->cap * D : (size_t)(D / 64) * idx->cap * sizeof(uint64_t);
        HIPCHK(hipMalloc(&idx->rq_codes, cb));
        HIPCHK(hipMalloc(&idx->rq_meta, (size_t)idx->cap * sizeof(float4)));
        HIPCHK(hipMemset(idx->rq_codes, 0, cb));
        HIPCHK(hipMemset(idx->rq_meta, 0, (size_t)idx->cap * sizeof(float4)));
    }
    return WV_OK;
}

// encode nq prepared query rows (idx->qn, normalised for cosine) into idx->rqq / rqm
static int rq_encode_queries(wv_index* idx, hipStream_t s, int64_t nq) {
    const int64_t nq32 = round_up(nq, RQ_QPB);
    const size_t qb = idx->rq_bits == 8 ? (size_t)nq32 * idx->rq_D : (size_t)nq32 * 5 * (idx->rq_D / 64) * sizeof(uint64_t);
    HIPCHK(idx->rqq.ensure(qb));
    HIPCHK(idx->rqm.ensure((size_t)nq32 * sizeof(float4)));
    if (nq32 > nq) {  // padded group members: zero codes (their results are never written)
        HIPCHK(hipMemsetAsync(idx->rqq.p, 0, qb, s));
        HIPCHK(hipMemsetAsync(idx->rqm.p, 0, (size_t)nq32 * sizeof(float4), s));
    }
    launch_rq_encode(idx, s, idx->qn.as<float>(), idx->dpad, nq, nullptr, 1, idx->rqq.p, 0, idx->rqm.as<float4>());
    HIPCHK(hipGetLastError());
    return WV_OK;
}

// quantized distances of queries [q0, q0 + F) (q0 % RQ_QPB == 0) -> E [F][ld], bmin
static int rq_dist(wv_index* idx, hipStream_t s, const uint32_t* valid, int64_t q0, int F, int64_t ld, float* E,
                   float* bmin) {
    const int64_t nslots = idx->hiwater;
    const float fl2 = idx->metric == WV_METRIC_L2_SQUARED ? 1.f : 0.f;
    const float fcos = idx->metric == WV_METRIC_COSINE_DOT ? 1.f : 0.f;
    dim3 grid((unsigned)((F + RQ_QPB - 1) / RQ_QPB), (unsigned)(ld / 256));
    if (idx->rq_bits == 8)
        k_rq8_dist<<<grid, 256, 0, s>>>(reinterpret_cast<const uint4*>(idx->rq_codes), idx->rq_meta, idx->rq_D, valid,
                                        nslots, idx->rqq.as<uint4>(), idx->rqm.as<float4>(), q0, F, fl2, fcos, ld, E,
                                        bmin);
    else
        k_rq1_dist<<<grid, 256, 0, s>>>(reinterpret_cast<const uint64_t*>(idx->rq_codes), idx->cap, idx->rq_meta,
                                        idx->rq_D / 64, valid, nslots, idx->rqq.as<uint64_t>(), idx->rqm.as<float4>(),
                                        q0, F, fl2, fcos, ld, E, bmin);
    HIPCHK(hipGetLastError());
    return WV_OK;
}

// flat.searchByVectorQuantized (flat/index.go:460-532) for rq-8 / rq-1: exact
// quantized distances + block minima (k_rq*_dist), the R-heap replayed in id
// order (k_replay_scan, extracted ascending = reversed pop order), fp32
// rescoring of the candidates (k_rescore_ids) and the k-heap fed in pop order
// (k_bq_final with asc = 1).
static int search_rq(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k,
                     const uint32_t* valid, uint64_t* o_ids, float* o_d, int32_t* o_n) {
    if (qd != idx->dims)  // SingleDist of the rescoring (distancer/errors.go:16)
        return set_err(WV_ERR_VECTOR_LENGTH, "%lld vs %d: vector lengths don't match", (long long)qd, idx->dims);
    if (k <= 0) return set_err(WV_ERR_INVALID, "k must be positive (reference heap Top() on empty queue)");
    if (!idx->rq_ready) return set_err(WV_ERR_QUANTIZER, "quantizer not initialized");
    const int R = idx->rescore_limit > k ? idx->rescore_limit : k;  // searchTimeRescore (:413-421)
    if (R > 8192) return set_err(WV_ERR_UNSUPPORTED, "rescore limit %d > 8192", R);
    const int64_t nq_pad = round_up(nq, QB);
    int rc = prepare_queries(idx, s, d_qraw, nq, nq_pad);
    if (rc) return rc;
    rc = rq_encode_queries(idx, s, nq);
    if (rc) return rc;
    idx->stats.queries += (uint64_t)nq;
    idx->stats.batches++;
    idx->stats.replayed_queries += (uint64_t)nq;
    HIPCHK(idx->ident.ensure((size_t)nq * sizeof(int32_t)));
    {
        std::vector<int32_t> id((size_t)nq);
        for (int64_t i = 0; i < nq; i++) id[i] = (int32_t)i;
        HIPCHK(hipMemcpyAsync(idx->ident.p, id.data(), (size_t)nq * sizeof(int32_t), hipMemcpyHostToDevice, s));
    }
    const int32_t* qlist = idx->ident.as<int32_t>();
    const int64_t nslots = idx->hiwater;
    const int64_t ld = std::max<int64_t>(round_up(nslots, EBLK), EBLK);
    // query groups: multiples of RQ_QPB, two distance buffers of up to
    // 16 GiB each (a quarter of the free HBM at most).  A replay wave's time
    // does not shrink with the group (one wave per query), so groups are as
    // large as memory allows.  Group i's distances (whole GPU, stream s)
    // overlap group i-1's replay (stream aux); buffer i&1 is reused once
    // replay i-2 has finished with it.
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    const int64_t have = (int64_t)(Eb0_bytes(idx) + free_b / 4);
    const int64_t budget = std::max<int64_t>(std::min<int64_t>(16ll << 30, have), 1ll << 30);
    int64_t G = (budget / (ld * 4)) / RQ_QPB * RQ_QPB;
    G = std::max<int64_t>(RQ_QPB, std::min<int64_t>(G, round_up(nq, RQ_QPB)));
    idx->stats.last_group_queries = (uint64_t)std::min<int64_t>(G, nq);
    rc = ensure_aux(idx);
    if (rc) return rc;
    DBuf* Eb[2] = {&idx->rE, &idx->rE2};
    DBuf* Bb[2] = {&idx->rB, &idx->rB2};
    for (int b = 0; b < 2; b++) {
        HIPCHK(Eb[b]->ensure((size_t)G * ld * sizeof(float)));
        HIPCHK(Bb[b]->ensure((size_t)G * (ld / EBLK) * sizeof(float)));
    }
    HIPCHK(idx->ascI.ensure((size_t)nq * R * sizeof(uint64_t)));
    HIPCHK(idx->ascD.ensure((size_t)nq * R * sizeof(float)));
    HIPCHK(idx->ascN.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(idx->candE.ensure((size_t)nq * R * sizeof(float)));
    const size_t lds_rep = (size_t)R * sizeof(uint64_t) + 64 * sizeof(float) + (size_t)R * sizeof(float) + 16;
    if (lds_rep > 64 * 1024)
        HIPCHK(hipFuncSetAttribute((const void*)k_replay_scan, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_rep));
    int64_t gi = 0;
    for (int64_t g0 = 0; g0 < nq; g0 += G, gi++) {
        const int F = (int)std::min<int64_t>(G, nq - g0);
        const int b = (int)(gi & 1);
        if (gi >= 2) HIPCHK(hipStreamWaitEvent(s, idx->evr[b], 0));
        if (idx->timing && g0 == 0) HIPCHK(hipEventRecord(idx->ev0, s));
        rc = rq_dist(idx, s, valid, g0, F, ld, Eb[b]->as<float>(), Bb[b]->as<float>());
        if (rc) return rc;
        if (idx->timing && g0 == 0) HIPCHK(hipEventRecord(idx->ev1, s));
        HIPCHK(hipEventRecord(idx->evd[b], s));
        HIPCHK(hipStreamWaitEvent(idx->aux, idx->evd[b], 0));
        k_replay_scan<<<F, 64, lds_rep, idx->aux>>>(Eb[b]->as<float>(), Bb[b]->as<float>(), valid, nslots, ld,
                                                    qlist + g0, F, R, idx->id_base, nullptr, nullptr, nullptr, 1, 0,
                                                    R, idx->ascI.as<uint64_t>() + g0 * R,
                                                    idx->ascD.as<float>() + g0 * R, idx->ascN.as<int32_t>() + g0, 0, 0,
                                                    nullptr, nullptr, nullptr, 0);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(idx->evr[b], idx->aux));
    }
    // join: the rescoring on s reads every group's heap
    for (int b = 0; b < 2 && b < gi; b++) HIPCHK(hipStreamWaitEvent(s, idx->evr[b], 0));
    idx->bq_nq = nq;
    idx->bq_R = R;
    rc = bq_rescore(idx, s, idx->ascI.as<uint64_t>(), idx->ascN.as<int32_t>(), idx->candE.as<float>());
    if (rc) return rc;
    const size_t lds_f = (size_t)k * (sizeof(uint64_t) + sizeof(float)) + 16;
    if (lds_f > 64 * 1024)
        HIPCHK(hipFuncSetAttribute((const void*)k_bq_final, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_f));
    k_bq_final<<<(unsigned)nq, 64, lds_f, s>>>(idx->ascI.as<uint64_t>(), idx->candE.as<float>(), idx->ascN.as<int32_t>(),
                                               qlist, (int)nq, R, k, 1, 0, o_ids, o_d, o_n, 1);
    HIPCHK(hipGetLastError());
    if (idx->timing) {
        HIPCHK(hipStreamSynchronize(s));
        float ms = 0.f;
        hipEventElapsedTime(&ms, idx->ev0, idx->ev1);
        idx->stats.last_select_ms = ms;
    }
    return WV_OK;
}

extern "C" int wv_index_rq_info(wv_index* idx, int32_t* out) {
    if (!idx || !out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    out[0] = idx->rq_bits;
    out[1] = idx->rq_D;
    out[2] = idx->rq_bits == 8 ? 16 + idx->rq_D : idx->rq_bits == 1 ? 8 * (1 + idx->rq_D / 64) : 0;
    out[3] = idx->rq_ready;
    return WV_OK;
}

static inline void put_be32(uint8_t* b, float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    b[0] = (uint8_t)(u >> 24); b[1] = (uint8_t)(u >> 16); b[2] = (uint8_t)(u >> 8); b[3] = (uint8_t)u;
}

// codes of slots [0, n) in the reference's compressed-bucket formats:
// rq-8 RQCode (rotational_quantization.go:95-155, BE floats + bytes),
// rq-1 RQOneBitCode words (binary_rotational_quantization.go:92-148, LE u64)
extern "C" int wv_index_rq_codes(wv_index* idx, void* out, int64_t n) {
    if (!idx || !out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (!idx->rq_ready) return set_err(WV_ERR_QUANTIZER, "quantizer not initialized");
    if (n < 0 || n > idx->cap) return set_err(WV_ERR_INVALID, "rq_codes: n out of range");
    HIPCHK(hipStreamSynchronize(idx->stream));
    const int D = idx->rq_D, W = D / 64;
    std::vector<float4> meta((size_t)std::max<int64_t>(n, 1));
    if (n) HIPCHK(hipMemcpy(meta.data(), idx->rq_meta, (size_t)n * sizeof(float4), hipMemcpyDeviceToHost));
    if (idx->rq_bits == 8) {
        const int64_t ntile = (n + 255) / 256;
        std::vector<uint8_t> tiled((size_t)std::max<int64_t>(ntile * 256 * D, 1));
        if (n) HIPCHK(hipMemcpy(tiled.data(), idx->rq_codes, (size_t)ntile * 256 * D, hipMemcpyDeviceToHost));
        uint8_t* o = (uint8_t*)out;
        const int nch = D / 16;
        for (int64_t s = 0; s < n; s++) {
            uint8_t* c = o + (size_t)s * (16 + D);
            put_be32(c + 0, meta[s].x);
            put_be32(c + 4, meta[s].y);
            put_be32(c + 8, meta[s].z);
            put_be32(c + 12, meta[s].w);
            for (int ch = 0; ch < nch; ch++)
                memcpy(c + 16 + ch * 16, &tiled[((size_t)((s >> 8) * nch + ch) * 256 + (s & 255)) * 16], 16);
        }
    } else {
        std::vector<uint64_t> words((size_t)W * std::max<int64_t>(n, 1));
        if (n)
            HIPCHK(hipMemcpy2D(words.data(), (size_t)n * sizeof(uint64_t), idx->rq_codes, (size_t)idx->cap * sizeof(uint64_t),
                               (size_t)n * sizeof(uint64_t), W, hipMemcpyDeviceToHost));
        uint64_t* o = (uint64_t*)out;
        for (int64_t s = 0; s < n; s++) {
            uint32_t st, sq;
            memcpy(&st, &meta[s].x, 4);
            memcpy(&sq, &meta[s].y, 4);
            o[(size_t)s * (1 + W)] = ((uint64_t)sq << 32) | st;
            for (int w = 0; w < W; w++) o[(size_t)s * (1 + W) + 1 + w] = words[(size_t)w * n + s];
        }
    }
    return WV_OK;
}

// quantized distances (the distancer the scan uses) of nq queries against
// slots [0, n): out [nq][n], +inf for slots without a vector
extern "C" int wv_index_rq_distances(wv_index* idx, const float* queries, int64_t nq, int64_t d, float* out,
                                     int64_t n) {
    if (!idx || !out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (!idx->rq_ready) return set_err(WV_ERR_QUANTIZER, "quantizer not initialized");
    if (d != idx->dims) return set_err(WV_ERR_VECTOR_LENGTH, "vector lengths don't match");
    if (n < 0 || n > idx->hiwater || nq <= 0) return set_err(WV_ERR_INVALID, "rq_distances: bad sizes");
    hipStream_t s = idx->stream;
    HIPCHK(idx->qraw.ensure((size_t)nq * d * sizeof(float)));
    HIPCHK(hipMemcpyAsync(idx->qraw.p, queries, (size_t)nq * d * sizeof(float), hipMemcpyHostToDevice, s));
    int rc = prepare_queries(idx, s, idx->qraw.as<float>(), nq, round_up(nq, QB));
    if (rc) return rc;
    rc = rq_encode_queries(idx, s, nq);
    if (rc) return rc;
    const int64_t ld = std::max<int64_t>(round_up(idx->hiwater, EBLK), EBLK);
    const int64_t nq32 = round_up(nq, RQ_QPB);
    DBuf E, B;
    HIPCHK(E.ensure((size_t)nq32 * ld * sizeof(float)));
    HIPCHK(B.ensure((size_t)nq32 * (ld / EBLK) * sizeof(float)));
    rc = rq_dist(idx, s, idx->present, 0, (int)nq, ld, E.as<float>(), B.as<float>());
    if (rc) return rc;
    if (n > 0)
        HIPCHK(hipMemcpy2DAsync(out, (size_t)n * sizeof(float), E.p, (size_t)ld * sizeof(float), (size_t)n * sizeof(float),
                                nq, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    E.release();
    B.release();
    return WV_OK;
}

// ---------------------------------------------------------------------------
// exact search on the block-key path (qs_kernels.hip).
// Queries already prepared (idx->qn, qn2).  Outputs [nq][kout]; mode 1 leaves
// flags (nonzero = not proven) for the caller, mode 0 replays them.  No host
// synchronisation: the eps inputs, flag lists and counts stay on the device.
// ---------------------------------------------------------------------------
// the block-key replay of listed queries: k_blk_replay_par (8 waves per query,
// k < 64) or k_blk_replay (one wave per query).  list/count: device list and
// its length at counters[1] (or nlist when counters == nullptr); max_list =
// host bound of the list length (grid sizing).
// the pooled block-key replay (k_rp_*) serves this k and key row length
// (the only block-key form that can record insertions)
static bool blk_pooled(const wv_index* idx, int k, int64_t nb) {
    const int64_t nch = (nb + RP_CH - 1) / RP_CH;
    return k < 448 && nch <= RP_MAXCH && ((idx->replay_par == 2 && k < 64) || idx->replay_par == 3);
}

static int launch_blk_replay(wv_index* idx, hipStream_t s, const float* key, int64_t ldk, int64_t nb, const float* eps,
                             const float4* qinfo, const uint32_t* valid, const float* Qn, const int32_t* list,
                             const uint32_t* counters, int nlist, int64_t max_list, int k, int kout, uint64_t* oi,
                             float* od, int32_t* on, const uint64_t* in_i, const float* in_d, const int32_t* in_n,
                             int extract, int by_list, uint64_t* rec_i = nullptr, float* rec_d = nullptr,
                             int32_t* rec_n = nullptr, int rec_cap = 0) {
    const int metric = idx->metric == WV_METRIC_L2_SQUARED ? L2 : idx->metric == WV_METRIC_DOT ? DOT : COSINE;
    const bool v5 = idx->variant == WV_VARIANT_AVX512;
    const int64_t nch = (nb + RP_CH - 1) / RP_CH;
    if (max_list <= 0) return WV_OK;
    // pooled form by default for k < 64 (few flagged queries, latency-bound);
    // many flagged queries with large k (integer data, C2) replay faster in the
    // one-wave kernel, which visits only blocks under the true heap top
    const int RS = k < 64 ? 2 : k < 192 ? 4 : k < 448 ? 8 : 0;
    if (blk_pooled(idx, k, nb)) {
        // pooled form: bounds + candidate pool (8 waves per query), exact
        // distances over the whole grid, one-wave heap per query
        const int64_t pool_cap = idx->rp_pool;
        const int64_t g1 = std::min<int64_t>(max_list, 256);
        HIPCHK(idx->qsScratch.ensure((size_t)g1 * nch * 64 * sizeof(float)));
        HIPCHK(idx->rpBlk.ensure((size_t)pool_cap * sizeof(uint32_t)));
        HIPCHK(idx->rpLb.ensure((size_t)pool_cap * sizeof(float)));
        HIPCHK(idx->rpQ.ensure((size_t)pool_cap * sizeof(int32_t)));
        HIPCHK(idx->rpE.ensure((size_t)pool_cap * 32 * sizeof(float)));
        HIPCHK(idx->rpVm.ensure((size_t)pool_cap * sizeof(uint32_t)));
        HIPCHK(idx->rpOff.ensure((size_t)max_list * sizeof(int32_t)));
        HIPCHK(idx->rpTot.ensure((size_t)max_list * sizeof(int32_t)));
        HIPCHK(idx->rpCtr.ensure(sizeof(uint32_t)));
        HIPCHK(hipMemsetAsync(idx->rpCtr.p, 0, sizeof(uint32_t), s));
#define WV_RPB(RSV, M) k_rp_bounds<RSV, M><<<(unsigned)g1, 512, 0, s>>>(key, ldk, nb, eps, qinfo, list, counters, nlist, k, in_d, in_n, idx->qsScratch.as<float>(), idx->rpBlk.as<uint32_t>(), idx->rpLb.as<float>(), idx->rpQ.as<int32_t>(), idx->rpCtr.as<uint32_t>(), pool_cap, idx->rpOff.as<int32_t>(), idx->rpTot.as<int32_t>(), by_list)
#define WV_RPBS(M) do { if (RS == 2) WV_RPB(2, M); else if (RS == 4) WV_RPB(4, M); else WV_RPB(8, M); } while (0)
        switch (metric) {
        case L2: WV_RPBS(L2); break;
        case DOT: WV_RPBS(DOT); break;
        default: WV_RPBS(COSINE); break;
        }
#undef WV_RPBS
#undef WV_RPB
        HIPCHK(hipGetLastError());
#define WV_RPE(M, V) k_rp_exact<M, V><<<1024, 256, 0, s>>>(idx->X, idx->dpad, valid, idx->hiwater, Qn, idx->dims, list, idx->rpBlk.as<uint32_t>(), idx->rpQ.as<int32_t>(), idx->rpCtr.as<uint32_t>(), pool_cap, idx->rpE.as<float>(), idx->rpVm.as<uint32_t>())
        switch (metric) {
        case L2: if (v5) WV_RPE(L2, AVX512); else WV_RPE(L2, AVX256); break;
        case DOT: if (v5) WV_RPE(DOT, AVX512); else WV_RPE(DOT, AVX256); break;
        default: if (v5) WV_RPE(COSINE, AVX512); else WV_RPE(COSINE, AVX256); break;
        }
#undef WV_RPE
        HIPCHK(hipGetLastError());
        const size_t hlds = (size_t)k * (sizeof(uint64_t) + sizeof(float)) + 64 * sizeof(float) + RPW * 32 * sizeof(float) + 16;
        const int64_t g3 = std::min<int64_t>(max_list, 2048);
#define WV_RPH(M, V)                                                                                            \
    do {                                                                                                        \
        if (hlds > 64 * 1024) HIPCHK(hipFuncSetAttribute((const void*)k_rp_heap<M, V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)hlds)); \
        k_rp_heap<M, V><<<(unsigned)g3, 64, hlds, s>>>(key, ldk, nb, eps, qinfo, idx->X, idx->dpad, valid, idx->hiwater, Qn, idx->dims, list, counters, nlist, k, kout, idx->id_base, oi, od, on, in_i, in_d, in_n, extract, by_list, idx->rpBlk.as<uint32_t>(), idx->rpLb.as<float>(), idx->rpE.as<float>(), idx->rpVm.as<uint32_t>(), idx->rpOff.as<int32_t>(), idx->rpTot.as<int32_t>(), rec_i, rec_d, rec_n, rec_cap); \
    } while (0)
        switch (metric) {
        case L2: if (v5) WV_RPH(L2, AVX512); else WV_RPH(L2, AVX256); break;
        case DOT: if (v5) WV_RPH(DOT, AVX512); else WV_RPH(DOT, AVX256); break;
        default: if (v5) WV_RPH(COSINE, AVX512); else WV_RPH(COSINE, AVX256); break;
        }
#undef WV_RPH
        HIPCHK(hipGetLastError());
        return WV_OK;
    }
    if (rec_i) return set_err(WV_ERR_UNSUPPORTED, "recorded replay needs the pooled block-key replay (k < 64)");
    if (k < 64 && nch <= RP_MAXCH && idx->replay_par) {
        const int64_t grid = std::min<int64_t>(max_list, 256);
        HIPCHK(idx->qsScratch.ensure((size_t)grid * nch * 64 * sizeof(float)));
#define WV_RPP(M, V) k_blk_replay_par<M, V><<<(unsigned)grid, 512, 0, s>>>(key, ldk, nb, eps, qinfo, idx->X, idx->dpad, valid, idx->hiwater, Qn, idx->dims, list, counters, nlist, k, kout, idx->id_base, oi, od, on, in_i, in_d, in_n, extract, by_list, idx->qsScratch.as<float>())
        switch (metric) {
        case L2: if (v5) WV_RPP(L2, AVX512); else WV_RPP(L2, AVX256); break;
        case DOT: if (v5) WV_RPP(DOT, AVX512); else WV_RPP(DOT, AVX256); break;
        default: if (v5) WV_RPP(COSINE, AVX512); else WV_RPP(COSINE, AVX256); break;
        }
#undef WV_RPP
        HIPCHK(hipGetLastError());
        return WV_OK;
    }
    const size_t rlds = (size_t)k * sizeof(uint64_t) + 64 * sizeof(float) + (size_t)k * sizeof(float) + 16 + 16 * 64 * sizeof(float);
    if (rlds > 160 * 1024) return set_err(WV_ERR_UNSUPPORTED, "k %d too large for the replay heap", k);
#define WV_RP(M, V)                                                                                             \
    do {                                                                                                        \
        if (rlds > 64 * 1024) HIPCHK(hipFuncSetAttribute((const void*)k_blk_replay<M, V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)rlds)); \
        k_blk_replay<M, V><<<(unsigned)max_list, 64, rlds, s>>>(key, ldk, nb, eps, qinfo, idx->X, idx->dpad, valid, idx->hiwater, Qn, idx->dims, list, counters, nlist, k, kout, idx->id_base, oi, od, on, in_i, in_d, in_n, extract, by_list); \
    } while (0)
    switch (metric) {
    case L2: if (v5) WV_RP(L2, AVX512); else WV_RP(L2, AVX256); break;
    case DOT: if (v5) WV_RP(DOT, AVX512); else WV_RP(DOT, AVX256); break;
    default: if (v5) WV_RP(COSINE, AVX512); else WV_RP(COSINE, AVX256); break;
    }
#undef WV_RP
    HIPCHK(hipGetLastError());
    return WV_OK;
}

static int qs_R(int k) { return k + 1 <= 64 ? 2 : k + 1 <= 192 ? 4 : k + 1 <= 448 ? 8 : 0; }

// phase 0: the whole search.  Sharded two-phase form (mode 1, one query chunk):
// phase 1 = block keys + local candidate selection, topA [nq][k+1] = this
// shard's k+1 smallest block-key A values (eps in idx->qsEps); phase 2 = the
// global threshold from every shard's topA / eps (gA [W][nq][k+1], gE [W][nq],
// k_blk_gthresh), exact distances, overflow pass.
static int search_qs(wv_index* idx, hipStream_t s, int64_t nq, int k, int mode, const uint32_t* valid,
                     uint64_t* o_ids, float* o_d, int32_t* o_n, int32_t* o_flags, int phase = 0,
                     float* topA = nullptr, const float* gA = nullptr, const float* gE = nullptr, int W = 0) {
    const int kout = mode == 1 ? k + 1 : k;
    const int NK = idx->dpb / 16;
    const int RB = qs_rb(NK);
    const int R = qs_R(k);
    const int L = 64 * (R - 1);
    const int64_t nslots = std::max<int64_t>(1, (idx->hiwater + 32 * RB - 1) / (32 * RB));
    const int64_t nb = nslots * RB;  // 32-row blocks scanned = key row length
    const int64_t ldk = nb;
    // query chunks of 256-multiples whose key rows fit 16 GiB (10M rows: 13k queries per chunk)
    const int64_t qmax = std::max<int64_t>(QS_QPB, ((16ll << 30) / (ldk * 4)) / QS_QPB * QS_QPB);
    const int64_t qc = std::min<int64_t>(round_up(nq, QS_QPB), qmax);
    idx->stats.last_group_queries = (uint64_t)std::min<int64_t>(qc, nq);  // the timed block-key launch
    HIPCHK(idx->qsQb.ensure((size_t)qc * idx->dpb * sizeof(uint16_t)));
    HIPCHK(idx->qsInfo.ensure((size_t)qc * sizeof(float4)));
    HIPCHK(idx->qsKey.ensure((size_t)qc * ldk * sizeof(float)));
    HIPCHK(idx->qsCand.ensure((size_t)qc * std::max(L, 448) * sizeof(uint32_t)));  // 448: the overflow pass
    HIPCHK(idx->qsNc.ensure((size_t)qc * sizeof(int32_t)));
    HIPCHK(idx->qsEps.ensure((size_t)qc * sizeof(float)));
    HIPCHK(idx->qsCap.ensure((size_t)qc * sizeof(float)));
    HIPCHK(idx->qsList.ensure((size_t)2 * qc * sizeof(int32_t)));
    if (!o_flags || phase) HIPCHK(idx->qsFlags.ensure((size_t)qc * sizeof(int32_t)));
    if (phase && qc < nq) return set_err(WV_ERR_UNSUPPORTED, "two-phase shard search: batch exceeds one query chunk");
    const size_t rlds = (size_t)k * sizeof(uint64_t) + 64 * sizeof(float) + (size_t)k * sizeof(float) + 16 + 16 * 64 * sizeof(float);
    if (mode == 0 && rlds > 160 * 1024) return set_err(WV_ERR_UNSUPPORTED, "k %d too large for the replay heap", k);
    // error-bound constants: reference-order fp32 (gamma_{dpb+8}) and the MFMA's
    // fp32 accumulation over NK chained 16-deep products (u' = 2^-22)
    const double u4 = 2.384185791015625e-07;
    const double hdep = NK + 16.0;
    const float gacc = (float)(hdep * u4 / (1.0 - hdep * u4));
    const float gd = (float)gamma_n(idx->dpb + 8);
    const int metric = idx->metric == WV_METRIC_L2_SQUARED ? L2 : idx->metric == WV_METRIC_DOT ? DOT : COSINE;
    const bool v5 = idx->variant == WV_VARIANT_AVX512;
    const float* Qn_all = idx->qn.as<float>();
    if (phase != 2) {  // phase 2 keeps phase 1's block-key timing; the total spans both
        idx->timed = 0;
        idx->timed_total = 0;
        if (idx->timing) HIPCHK(hipEventRecord(idx->evt0, s));
    }
    for (int64_t c0 = 0; c0 < nq; c0 += qc) {
        const int64_t cn = std::min<int64_t>(qc, nq - c0);
        const int64_t cn_pad = round_up(cn, QS_QPB);
        if (c0 == 0) { idx->qs_last_nq = cn == nq ? cn : 0; idx->qs_last_nb = nb; idx->qs_last_ldk = ldk; }
        const float* Qn = Qn_all + c0 * idx->dpad;
        float4* qinfo = idx->qsInfo.as<float4>();
        if (phase != 2)
        k_query_split<<<(unsigned)((cn_pad + 3) / 4), 256, 0, s>>>(Qn, idx->dpad, idx->dpb, cn, cn_pad,
                                                                   idx->qsQb.as<uint16_t>(), qinfo);
        // ---- block keys (the dominant kernel) ----
        QsArgs a;
        a.Xb = reinterpret_cast<const unsigned char*>(idx->Xb);
        a.xnorm2 = idx->xnorm2;
        a.valid = valid;
        a.Qb = reinterpret_cast<const unsigned char*>(idx->qsQb.p);
        a.key = idx->qsKey.as<float>();
        a.ldk = ldk;
        a.nslots = nslots;
        a.dbg = idx->sel_dbg;
        // k_qs_blockkey_w4 for d > 768: 128-query workgroups, a 32-row block in two
        // column parts per ring step: dpb 1024 -> 4 slots of 32 KiB, 1536 -> 3 of 48 KiB
        const bool w4 = idx->dpb > QS_W4_DPB;
        const int w4_nb = NK == 64 ? 4 : 3;
        a.nqg = (int)(cn_pad / (w4 ? 128 : QS_QPB));
        int64_t nspans = 256 / std::gcd(256, a.nqg);
        while ((int64_t)a.nqg * nspans < 256) nspans *= 2;
        if (idx->spans_opt > 0) nspans = idx->spans_opt;
        {   // a span's plane bytes (+ one tile of slack) must stay below 4 GiB (32-bit buffer offsets)
            const int64_t slot_b = (int64_t)RB * 32 * idx->dpb * 2;
            const int64_t max_sps = ((1ll << 32) - 2 * 256ll * idx->dpb * 2) / slot_b;
            nspans = std::max<int64_t>(nspans, (nslots + max_sps - 1) / max_sps);
        }
        nspans = std::max<int64_t>(1, std::min<int64_t>(nspans, nslots));
        const int64_t sps = (nslots + nspans - 1) / nspans;
        a.slots_per_span = (int)sps;
        a.nspans = (int)((nslots + sps - 1) / sps);
        const bool l2 = metric == L2;
        const size_t lds = w4 ? (size_t)w4_nb * (NK / 4) * 2048 + 256 + (l2 ? (size_t)4 * 4 * 128 : 0)
                              : (size_t)QS_NBUF * RB * NK * 1024 + 512 + (l2 ? (size_t)8 * 4 * RB * 128 : 0);
        dim3 grid((unsigned)((int64_t)a.nqg * a.nspans));
        if (phase != 2) {
        const bool time_it = idx->timing && c0 == 0;
        if (time_it) HIPCHK(hipEventRecord(idx->ev0, s));
#define WV_QS(NKV, L2V)                                                                                        \
    do {                                                                                                       \
        HIPCHK(hipFuncSetAttribute((const void*)k_qs_blockkey<NKV, L2V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
        k_qs_blockkey<NKV, L2V><<<grid, 512, lds, s>>>(a);                                                     \
    } while (0)
#define WV_QS3(NKV, L2V, D)                                                                                    \
    do {                                                                                                       \
        HIPCHK(hipFuncSetAttribute((const void*)k_qs_blockkey<NKV, L2V, D>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
        k_qs_blockkey<NKV, L2V, D><<<grid, 512, lds, s>>>(a);                                                  \
    } while (0)
#define WV_QSN(L2V)                                    \
    switch (NK) {                                      \
    case 8: WV_QS(8, L2V); break;                      \
    case 16: WV_QS(16, L2V); break;                    \
    case 24: WV_QS(24, L2V); break;                    \
    case 32: WV_QS(32, L2V); break;                    \
    case 40: WV_QS(40, L2V); break;                    \
    default: WV_QS(48, L2V); break;                    \
    }
#define WV_QSW(NKV, L2V, NBV)                                                                                  \
    do {                                                                                                       \
        HIPCHK(hipFuncSetAttribute((const void*)k_qs_blockkey_w4<NKV, L2V, 2, NBV>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
        k_qs_blockkey_w4<NKV, L2V, 2, NBV><<<grid, 256, lds, s>>>(a);                                          \
    } while (0)
#define WV_QSWN(L2V)                                   \
    if (NK == 64) WV_QSW(64, L2V, 4); else WV_QSW(96, L2V, 3);
        if (w4) {
            if (l2) { WV_QSWN(true); } else { WV_QSWN(false); }
#ifdef WV_QS_DBG  // timing experiments (k_qs_blockkey DBG bits), not in the product build
        } else if (idx->sel_dbg > 0 && !l2 && NK == 48) {
            switch (idx->sel_dbg) {
            case 1: WV_QS3(48, false, 1); break;
            case 2: WV_QS3(48, false, 2); break;
            case 3: WV_QS3(48, false, 3); break;
            case 4: WV_QS3(48, false, 4); break;
            case 5: WV_QS3(48, false, 5); break;
            case 6: WV_QS3(48, false, 6); break;
            default: WV_QS3(48, false, 7); break;
            }
#endif
        } else if (l2) { WV_QSN(true); } else { WV_QSN(false); }
#undef WV_QSN
#undef WV_QS3
#undef WV_QS
#undef WV_QSWN
#undef WV_QSW
        HIPCHK(hipGetLastError());
        if (time_it) { HIPCHK(hipEventRecord(idx->ev1, s)); idx->timed = 1; }
        idx->stats.mfma_launches++;
        }
        // ---- candidate blocks, exact rows, proof ----
        int32_t* flags = phase ? idx->qsFlags.as<int32_t>() : o_flags ? o_flags + c0 : idx->qsFlags.as<int32_t>();
        int32_t* olist = idx->qsList.as<int32_t>() + qc;  // second half: the overflow list
        // select / exact pass RV over all queries (list == nullptr) or over the listed ones
        auto sel = [&](int RV, const int32_t* list, const uint32_t* cnt, float* tA) {
            const unsigned gw = (unsigned)((cn + 3) / 4);
#define WV_SELR(RV) k_blk_select<RV><<<gw, 256, 0, s>>>(a.key, ldk, nb, (int)cn, k, metric, qinfo, idx->qsmax, idx->d_maxn2, gd, gacc, idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(), flags, idx->qsEps.as<float>(), list, cnt, tA, idx->qsCap.as<float>())
            if (RV == 2) WV_SELR(2); else if (RV == 4) WV_SELR(4); else WV_SELR(8);
#undef WV_SELR
        };
        // phase 2 cuts the lists with the global threshold: the local cap no longer bounds them
        const float* capv = (idx->exact_cap && phase == 0) ? idx->qsCap.as<float>() : nullptr;
        auto exa = [&](int RV, const int32_t* list, const uint32_t* cnt, const float* eb = nullptr, int64_t ldE = 0) {
#define WV_EXR(RV, M, V) k_blk_exact<RV, M, V><<<(unsigned)cn, 256, 0, s>>>(idx->X, idx->dpad, valid, idx->hiwater, Qn, idx->dims, idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(), (int)cn, k, kout, idx->id_base, o_ids + c0 * kout, o_d + c0 * kout, o_n + c0, flags, list, cnt, eb, ldE, capv)
#define WV_EXM(RV)                                                          \
    switch (metric) {                                                       \
    case L2: if (v5) WV_EXR(RV, L2, AVX512); else WV_EXR(RV, L2, AVX256); break;   \
    case DOT: if (v5) WV_EXR(RV, DOT, AVX512); else WV_EXR(RV, DOT, AVX256); break; \
    default: if (v5) WV_EXR(RV, COSINE, AVX512); else WV_EXR(RV, COSINE, AVX256); break; \
    }
            if (RV == 2) { WV_EXM(2); } else if (RV == 4) { WV_EXM(4); } else { WV_EXM(8); }
#undef WV_EXM
#undef WV_EXR
        };
        if (phase != 2) sel(R, nullptr, nullptr, phase == 1 ? topA : nullptr);
        HIPCHK(hipGetLastError());
        if (phase == 1) continue;
        if (phase == 2)  // the global threshold cuts this shard's candidate lists
            k_blk_gthresh<<<(unsigned)((cn + 3) / 4), 256, 0, s>>>(gA, gE, W, (int)cn, k, metric, qinfo, a.key, ldk,
                                                                  idx->qsCand.as<uint32_t>(), L, idx->qsNc.as<int32_t>(),
                                                                  idx->qsEps.as<float>(), flags);
        const size_t bm_lds = (size_t)32 * (idx->dpad + 4) * sizeof(float);
        // (bmE holds cn*L*32 floats: above a 4 GiB budget, or past the 2^23
        // queries k_inv_scatter's packed (q << 9 | j) can name, the
        // candidate-major k_blk_exact computes the distances itself)
        if (idx->exact_bm && bm_lds <= 64 * 1024 && nb < (1ll << 31) && cn < (1ll << 23) &&
            (int64_t)cn * L * 32 * 4 <= (4ll << 30)) {
            // block-major exact distances: invert the candidate lists per block
            const int64_t ldE = (int64_t)L * 32;
            HIPCHK(idx->bmCnt.ensure((size_t)nb * sizeof(uint32_t)));
            HIPCHK(idx->bmOff.ensure((size_t)(nb + 1) * sizeof(uint32_t)));
            HIPCHK(idx->bmPairs.ensure((size_t)cn * L * sizeof(uint32_t)));
            HIPCHK(idx->bmE.ensure((size_t)cn * ldE * sizeof(float)));
            HIPCHK(hipMemsetAsync(idx->bmCnt.p, 0, (size_t)nb * sizeof(uint32_t), s));
            const unsigned gw = (unsigned)((cn + 3) / 4);
            k_inv_count<<<gw, 256, 0, s>>>(idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(), flags, (int)cn, L,
                                           idx->bmCnt.as<uint32_t>());
            k_inv_scan<<<1, 1024, 0, s>>>(idx->bmCnt.as<uint32_t>(), nb, idx->bmOff.as<uint32_t>());
            k_inv_scatter<<<gw, 256, 0, s>>>(idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(), flags, (int)cn, L,
                                             idx->bmOff.as<uint32_t>(), idx->bmCnt.as<uint32_t>(),
                                             idx->bmPairs.as<uint32_t>());
#define WV_BM(M, V) k_exact_bm<M, V><<<(unsigned)nb, 256, bm_lds, s>>>(idx->X, idx->dpad, idx->hiwater, Qn, idx->dims, idx->bmOff.as<uint32_t>(), idx->bmPairs.as<uint32_t>(), ldE, idx->bmE.as<float>())
            switch (metric) {
            case L2: if (v5) WV_BM(L2, AVX512); else WV_BM(L2, AVX256); break;
            case DOT: if (v5) WV_BM(DOT, AVX512); else WV_BM(DOT, AVX256); break;
            default: if (v5) WV_BM(COSINE, AVX512); else WV_BM(COSINE, AVX256); break;
            }
#undef WV_BM
            HIPCHK(hipGetLastError());
            exa(R, nullptr, nullptr, idx->bmE.as<float>(), ldE);
        } else {
            exa(R, nullptr, nullptr);
        }
        HIPCHK(hipGetLastError());
        if (R < 8) {  // candidate lists that overflowed (flag 2): again with the 448-block lists
            HIPCHK(hipMemsetAsync(idx->qscount + 3, 0, sizeof(uint32_t), s));
            k_flag_list<<<(unsigned)((cn + 255) / 256), 256, 0, s>>>(flags, (int)cn, olist, idx->qscount + 2, 2);
            sel(8, olist, idx->qscount + 2, nullptr);
            exa(8, olist, idx->qscount + 2);
            HIPCHK(hipGetLastError());
        }
        if (idx->qs_force_flag) HIPCHK(hipMemsetAsync(flags, 1, (size_t)cn * sizeof(int32_t), s));
        if (phase == 2 && o_flags)
            HIPCHK(hipMemcpyAsync(o_flags + c0, flags, (size_t)cn * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
        if (mode == 1) continue;
        // ---- flagged queries: the exact heap replay, bounded by the block keys ----
        HIPCHK(hipMemsetAsync(idx->qscount + 1, 0, sizeof(uint32_t), s));
        k_flag_list<<<(unsigned)((cn + 255) / 256), 256, 0, s>>>(flags, (int)cn, idx->qsList.as<int32_t>(), idx->qscount, 0);
        {
            int rc = launch_blk_replay(idx, s, a.key, ldk, nb, idx->qsEps.as<float>(), qinfo, valid, Qn,
                                       idx->qsList.as<int32_t>(), idx->qscount, 0, cn, k, kout, o_ids + c0 * kout,
                                       o_d + c0 * kout, o_n + c0, nullptr, nullptr, nullptr, 1, 0);
            if (rc) return rc;
        }
    }
    if (idx->timing) {
        HIPCHK(hipEventRecord(idx->evt1, s));
        idx->timed_total = 1;
    }
    if (qc >= nq && valid == idx->present) idx->qs_keys_nq = nq;
    return WV_OK;
}

// Core batch search on device queries.  Outputs [nq][kout] device arrays.
// mode 0: kout = k, flagged queries resolved by replay; mode 1: kout = k+1,
// flags left for the caller.  n_valid = number of scan candidates.
static int search_core(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k, int mode,
                       const uint32_t* valid, int64_t n_valid, uint64_t* o_ids, float* o_d, int32_t* o_n,
                       int32_t* o_flags) {
    const int kout = mode == 1 ? k + 1 : k;
    idx->qs_keys_nq = 0;
    if (nq <= 0) return WV_OK;
    if (n_valid == 0 || idx->dims == 0) {
        HIPCHK(hipMemsetAsync(o_n, 0, (size_t)nq * sizeof(int32_t), s));
        if (o_flags) HIPCHK(hipMemsetAsync(o_flags, 0, (size_t)nq * sizeof(int32_t), s));
        return WV_OK;
    }
    if (idx->compression == WV_COMPRESSION_BQ) {
        if (mode != 0) return set_err(WV_ERR_UNSUPPORTED, "bq: shard-candidate mode not available");
        return search_bq(idx, s, d_qraw, nq, qd, k, valid, o_ids, o_d, o_n);
    }
    if (idx->rq_bits) {
        if (mode != 0) return set_err(WV_ERR_UNSUPPORTED, "rq: shard-candidate mode not available");
        return search_rq(idx, s, d_qraw, nq, qd, k, valid, o_ids, o_d, o_n);
    }
    if (idx->compression == WV_COMPRESSION_SQ) {  // SQ exists only behind hnsw: its flat branch
        if (mode != 0) return set_err(WV_ERR_UNSUPPORTED, "sq: shard-candidate mode not available");
        return search_hnsw_flat(idx, s, d_qraw, nq, qd, k, valid, o_ids, o_d, o_n);
    }
    if (idx->compression == WV_COMPRESSION_PQ && idx->pq_trained) {
        if (mode != 0) return set_err(WV_ERR_UNSUPPORTED, "pq: shard-candidate mode not available");
        return search_pq(idx, s, d_qraw, nq, qd, k, valid, o_ids, o_d, o_n);
    }
    // SingleDist length check on the first candidate: distancer/l2.go:47-50 etc.
    if (qd != idx->dims)
        return set_err(WV_ERR_VECTOR_LENGTH, "%lld vs %d: vector lengths don't match", (long long)qd, idx->dims);
    if (k <= 0) return set_err(WV_ERR_INVALID, "k must be positive (reference heap Top() on empty queue)");
    const int64_t nq_pad = round_up(nq, QS_QPB);  // 256: a block-key query group; a multiple of QB
    int rc = prepare_queries(idx, s, d_qraw, nq, nq_pad);
    if (rc) return rc;
    const float* Qn = idx->qn.as<float>();
    // block-key path (default): planes built, finite corpus, list sizes that fit
    if (idx->qs_planes && !idx->has_nonfinite && (idx->kernel_opt == 0 || idx->kernel_opt == 7) && !idx->force_replay &&
        qs_R(k) > 0 && idx->metric != WV_METRIC_HAMMING) {
        idx->stats.queries += (uint64_t)nq;
        idx->stats.batches++;
        return search_qs(idx, s, nq, k, mode, valid, o_ids, o_d, o_n, o_flags);
    }
    const int KP = k + idx->margin;
    const bool mfma_ok = KP <= 32 && idx->metric != WV_METRIC_HAMMING && !idx->force_replay;
    idx->stats.queries += (uint64_t)nq;
    idx->stats.batches++;

    HIPCHK(idx->oF.ensure((size_t)nq * sizeof(int32_t)));
    int32_t* flags = o_flags ? o_flags : idx->oF.as<int32_t>();

    if (mfma_ok) {
        // kernel 3: the f32 MFMA select (k_mfma_select3); 6: the HBM-streaming GEMV
        // select for small batches (k_gemv_select); auto picks by batch size
        int kver = idx->kernel_opt == 7 ? 0 : idx->kernel_opt;
        if (kver == 0) kver = nq <= idx->gemv_max ? 6 : 3;
        const bool gemv = kver == 6;
        // GEMV: QG queries per workgroup staged in LDS (<= 64 KiB of query rows)
        // (the smallest of 1/2/4/8 covering nq: padded query columns cost FMAs and LDS reads)
        int gqg = nq <= 1 ? 1 : nq <= 2 ? 2 : nq <= 4 ? 4 : 8;
        while (gqg > 1 && (int64_t)gqg * idx->dpad * 4 > 65536) gqg >>= 1;
        const int64_t ntiles = (idx->hiwater + BN3 - 1) / BN3;
        const int qtile = gemv ? gqg : QB;
        const int nqb = (int)(round_up(nq, qtile) / qtile);
        int qgroup = 1;
        for (int g : {4, 2, 1})
            if (nqb % g == 0) { qgroup = g; break; }
        if (idx->qgroup_opt > 0 && nqb % idx->qgroup_opt == 0) qgroup = idx->qgroup_opt;
        // ~768 workgroups for the MFMA select (2 per CU resident); keep the
        // workgroup count a multiple of 8 for the XCD mapping when possible
        const int64_t target_wg = gemv ? idx->gemv_wg : 768;
        int64_t nspans = idx->spans_opt > 0 ? idx->spans_opt : std::max<int64_t>(8, (target_wg + nqb - 1) / nqb);
        nspans = std::min<int64_t>(nspans, ntiles);
        int64_t tps = (ntiles + nspans - 1) / nspans;
        nspans = (ntiles + tps - 1) / tps;
        HIPCHK(idx->spanA.ensure((size_t)nq * nspans * KP * sizeof(float)));
        HIPCHK(idx->spanI.ensure((size_t)nq * nspans * KP * sizeof(uint32_t)));
        HIPCHK(idx->candA.ensure((size_t)nq * KP * sizeof(float)));
        HIPCHK(idx->candI.ensure((size_t)nq * KP * sizeof(uint32_t)));
        HIPCHK(idx->candE.ensure((size_t)nq * KP * sizeof(float)));
        SelectArgs a;
        a.X = idx->X; a.xnorm2 = idx->xnorm2; a.valid = valid; a.ntiles = ntiles;
        a.Q = Qn; a.qnorm2 = idx->qn2.as<float>(); a.nq = (int)nq; a.dpad = idx->dpad;
        a.tiles_per_span = (int)tps; a.nspans = (int)nspans; a.nqb = nqb; a.KP = KP; a.qgroup = qgroup;
        a.outA = idx->spanA.as<float>(); a.outI = idx->spanI.as<uint32_t>();
        a.dbg = idx->sel_dbg;
        a.opt = idx->sel_opt;
        // candidate buffer: as large as fits the LDS left by the staging ring
        const int64_t fixed = (int64_t)(NBUF3 * STG3 + QB * 2 + 4) * (int64_t)sizeof(float);
        int C = (int)std::min<int64_t>(64 - KP, std::max<int64_t>(4, (160 * 1024 - fixed) / (qtile * 8)));
        if (idx->cbuf_opt > 0) C = std::min(64 - KP, idx->cbuf_opt);
        size_t lds = (size_t)(fixed + (int64_t)qtile * C * 8);
        if (gemv) {  // a 32-row chunk adds <= 32 candidates per query: C = 64 - KP >= 32 never overflows
            C = 64 - KP;
            lds = (size_t)((int64_t)gqg * idx->dpad + (int64_t)gqg * KP * 2 + (int64_t)gqg * C * 2 + gqg * 2 + 3) * sizeof(float);
        }
        a.C = C;
        dim3 grid((unsigned)(nqb * nspans));
        if (idx->timing) HIPCHK(hipEventRecord(idx->ev0, s));
#define WV_SEL3(M)                                                                                        \
    do {                                                                                                  \
        HIPCHK(hipFuncSetAttribute((const void*)k_mfma_select3<M, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
        k_mfma_select3<M, 1><<<grid, 512, lds, s>>>(a);                                                   \
    } while (0)
#define WV_GEMV(M, G)                                                                                      \
    do {                                                                                                   \
        HIPCHK(hipFuncSetAttribute((const void*)k_gemv_select<M, G>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
        k_gemv_select<M, G><<<grid, 256, lds, s>>>(a);                                                     \
    } while (0)
#define WV_GEMVQ(M)                                          \
    do {                                                     \
        if (gqg == 8) WV_GEMV(M, 8);                         \
        else if (gqg == 4) WV_GEMV(M, 4);                    \
        else if (gqg == 2) WV_GEMV(M, 2);                    \
        else WV_GEMV(M, 1);                                  \
    } while (0)
        if (gemv) {
            switch (idx->metric) {
            case WV_METRIC_L2_SQUARED: WV_GEMVQ(L2); break;
            case WV_METRIC_DOT: WV_GEMVQ(DOT); break;
            default: WV_GEMVQ(COSINE); break;
            }
        } else {
            switch (idx->metric) {
            case WV_METRIC_L2_SQUARED: WV_SEL3(L2); break;
            case WV_METRIC_DOT: WV_SEL3(DOT); break;
            default: WV_SEL3(COSINE); break;
            }
        }
#undef WV_GEMVQ
#undef WV_GEMV
#undef WV_SEL3
        HIPCHK(hipGetLastError());
        if (idx->timing) HIPCHK(hipEventRecord(idx->ev1, s));
        idx->stats.mfma_launches++;
        int G = 1;  // GEMV: ~1024 spans per query -> merge in two levels (G groups of nspans/G)
        if (gemv)
            for (int g = 32; g >= 2; g--)
                if (nspans % g == 0 && nspans / g >= 2) { G = g; break; }
        if (gemv && G > 1) {
            HIPCHK(idx->gmA.ensure((size_t)nq * G * KP * sizeof(float)));
            HIPCHK(idx->gmI.ensure((size_t)nq * G * KP * sizeof(uint32_t)));
            k_merge_spans<2><<<(unsigned)((nq * G + 3) / 4), 256, 0, s>>>(a.outA, a.outI, (int)(nq * G), (int)(nspans / G),
                                                                           KP, idx->gmA.as<float>(), idx->gmI.as<uint32_t>());
            k_merge_spans<2><<<(unsigned)((nq + 3) / 4), 256, 0, s>>>(idx->gmA.as<float>(), idx->gmI.as<uint32_t>(), (int)nq,
                                                                       G, KP, idx->candA.as<float>(), idx->candI.as<uint32_t>());
        } else if (gemv)
            k_merge_spans<2><<<(unsigned)((nq + 3) / 4), 256, 0, s>>>(a.outA, a.outI, (int)nq, (int)nspans, KP,
                                                                       idx->candA.as<float>(), idx->candI.as<uint32_t>());
        else
            k_merge_spans<1><<<(unsigned)((nq + 3) / 4), 256, 0, s>>>(a.outA, a.outI, (int)nq, (int)nspans, KP,
                                                                       idx->candA.as<float>(), idx->candI.as<uint32_t>());
        const int64_t npairs = nq * KP;
        const bool v5 = idx->variant == WV_VARIANT_AVX512;
#define WV_RS(M, V) k_rescore<M, V><<<(unsigned)((npairs + 63) / 64), 64, 0, s>>>(idx->X, idx->dpad, Qn, idx->dims, idx->candI.as<uint32_t>(), (int)nq, KP, idx->candE.as<float>())
        switch (idx->metric) {
        case WV_METRIC_L2_SQUARED: if (v5) WV_RS(L2, AVX512); else WV_RS(L2, AVX256); break;
        case WV_METRIC_DOT: if (v5) WV_RS(DOT, AVX512); else WV_RS(DOT, AVX256); break;
        default: if (v5) WV_RS(COSINE, AVX512); else WV_RS(COSINE, AVX256); break;
        }
#undef WV_RS
        // error bound of |A - E|: 2 gamma_{d+4} * bound, +5% slack
        uint32_t mx = 0;
        HIPCHK(hipMemcpyAsync(&mx, idx->d_maxn2, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        float maxn2;
        memcpy(&maxn2, &mx, sizeof(float));
        const float eps_scale = (float)(2.0 * gamma_n(idx->dpad + 4) * 1.05 + 1e-12);
        const float eps_base = (float)(std::sqrt((double)maxn2) * (1.0 + 1e-6));
        idx->last_eps_scale = eps_scale;
        idx->last_eps_base = eps_base;
        idx->last_nq = nq;
        idx->last_KP = KP;
        k_finalize<1><<<(unsigned)((nq + 3) / 4), 256, 0, s>>>(
            idx->candA.as<float>(), idx->candI.as<uint32_t>(), idx->candE.as<float>(), idx->qn2.as<float>(), (int)nq,
            KP, k, kout, eps_scale, eps_base, idx->metric == WV_METRIC_L2_SQUARED ? L2 : DOT, idx->id_base, o_ids,
            o_d, o_n, flags);
        HIPCHK(hipGetLastError());
    } else {
        std::vector<int32_t> ones((size_t)nq, 1);
        HIPCHK(hipMemcpyAsync(flags, ones.data(), (size_t)nq * sizeof(int32_t), hipMemcpyHostToDevice, s));
    }
    if (mode == 1) {
        if (idx->timing) {
            HIPCHK(hipStreamSynchronize(s));
            float ms = 0.f;
            if (mfma_ok) hipEventElapsedTime(&ms, idx->ev0, idx->ev1);
            idx->stats.last_select_ms = ms;
        }
        return WV_OK;
    }
    // mode 0: replay the flagged queries
    std::vector<int32_t> hf((size_t)nq);
    HIPCHK(hipMemcpyAsync(hf.data(), flags, (size_t)nq * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (idx->timing && mfma_ok) {
        float ms = 0.f;
        hipEventElapsedTime(&ms, idx->ev0, idx->ev1);
        idx->stats.last_select_ms = ms;
    }
    std::vector<int32_t> ql;
    for (int64_t q = 0; q < nq; q++)
        if (hf[q]) ql.push_back((int32_t)q);
    if (!ql.empty()) {
        idx->stats.replayed_queries += ql.size();
        HIPCHK(idx->qlist.ensure(ql.size() * sizeof(int32_t)));
        HIPCHK(hipMemcpyAsync(idx->qlist.p, ql.data(), ql.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
        int rc2 = run_replay(idx, s, valid, Qn, idx->qlist.as<int32_t>(), (int)ql.size(), k, nullptr, nullptr, nullptr,
                             1, 1, kout, o_ids, o_d, o_n);
        if (rc2) return rc2;
    }
    return WV_OK;
}

// valid-slot bitmap for an allow list (present & allow); returns candidate count
static int build_valid(wv_index* idx, hipStream_t s, const uint64_t* allow, int64_t n_allow, int32_t allow_mode,
                       const uint32_t** valid_out, int64_t* n_valid) {
    if (allow_mode == 0) {
        *valid_out = idx->present;
        *n_valid = idx->npresent;
        return WV_OK;
    }
    std::vector<uint32_t> bits((size_t)std::max<int64_t>(idx->cap / 32, 1), 0);
    int64_t nv = 0;
    for (int64_t i = 0; i < n_allow; i++) {
        if (allow[i] < idx->id_base) continue;
        uint64_t sl = allow[i] - idx->id_base;
        if ((int64_t)sl >= idx->cap || !idx->h_present[sl]) continue;
        if (!(bits[sl >> 5] & (1u << (sl & 31)))) { bits[sl >> 5] |= 1u << (sl & 31); nv++; }
    }
    HIPCHK(idx->valid.ensure(bits.size() * sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(idx->valid.p, bits.data(), bits.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    *valid_out = idx->valid.as<uint32_t>();
    *n_valid = nv;
    return WV_OK;
}

extern "C" int wv_index_search_by_vector_batch(wv_index* idx, const float* queries, int64_t nq, int64_t d, int32_t k,
                                               const uint64_t* allow_ids, int64_t n_allow, int32_t allow_mode,
                                               uint64_t* out_ids, float* out_dists, int32_t* out_counts) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    hipStream_t s = idx->stream;
    if (allow_mode == 1 && n_allow == 0) {  // flat/index.go:590-594
        for (int64_t q = 0; q < nq; q++) out_counts[q] = 0;
        return WV_OK;
    }
    const uint32_t* valid = nullptr;
    int64_t n_valid = 0;
    int rc = build_valid(idx, s, allow_ids, n_allow, allow_mode, &valid, &n_valid);
    if (rc) return rc;
    if (n_valid == 0 || idx->dims == 0) {
        for (int64_t q = 0; q < nq; q++) out_counts[q] = 0;
        return WV_OK;
    }
    const int kk = std::max(k, 1);
    HIPCHK(idx->qraw.ensure((size_t)nq * d * sizeof(float)));
    HIPCHK(idx->oIds.ensure((size_t)nq * kk * sizeof(uint64_t)));
    HIPCHK(idx->oD.ensure((size_t)nq * kk * sizeof(float)));
    HIPCHK(idx->oN.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(hipMemcpyAsync(idx->qraw.p, queries, (size_t)nq * d * sizeof(float), hipMemcpyHostToDevice, s));
    rc = search_core(idx, s, idx->qraw.as<float>(), nq, d, k, 0, valid, n_valid, idx->oIds.as<uint64_t>(),
                     idx->oD.as<float>(), idx->oN.as<int32_t>(), nullptr);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(out_ids, idx->oIds.p, (size_t)nq * k * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out_dists, idx->oD.p, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out_counts, idx->oN.p, (size_t)nq * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

extern "C" int wv_index_hnsw_flat_search(wv_index* idx, const float* queries, int64_t nq, int64_t d, int32_t k,
                                         const uint64_t* allow_ids, int64_t n_allow, int32_t allow_mode,
                                         uint64_t* out_ids, float* out_dists, int32_t* out_counts) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->compression == WV_COMPRESSION_NONE)
        return set_err(WV_ERR_UNSUPPORTED, "hnsw flat search: index is not compressed (use SearchByVector)");
    hipStream_t s = idx->stream;
    if (allow_mode == 1 && n_allow == 0) {
        for (int64_t q = 0; q < nq; q++) out_counts[q] = 0;
        return WV_OK;
    }
    const uint32_t* valid = nullptr;
    int64_t n_valid = 0;
    int rc = build_valid(idx, s, allow_ids, n_allow, allow_mode, &valid, &n_valid);
    if (rc) return rc;
    if (n_valid == 0 || idx->dims == 0 || nq <= 0) {
        for (int64_t q = 0; q < nq; q++) out_counts[q] = 0;
        return WV_OK;
    }
    const int kk = std::max(k, 1);
    HIPCHK(idx->qraw.ensure((size_t)nq * d * sizeof(float)));
    HIPCHK(idx->oIds.ensure((size_t)nq * kk * sizeof(uint64_t)));
    HIPCHK(idx->oD.ensure((size_t)nq * kk * sizeof(float)));
    HIPCHK(idx->oN.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(hipMemcpyAsync(idx->qraw.p, queries, (size_t)nq * d * sizeof(float), hipMemcpyHostToDevice, s));
    rc = search_hnsw_flat(idx, s, idx->qraw.as<float>(), nq, d, k, valid, idx->oIds.as<uint64_t>(),
                          idx->oD.as<float>(), idx->oN.as<int32_t>());
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(out_ids, idx->oIds.p, (size_t)nq * k * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out_dists, idx->oD.p, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out_counts, idx->oN.p, (size_t)nq * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

// flat.SearchByVectorDistance (flat/index.go:699-761): recursiveSearch runs once
// with totalLimit = 100 (common/search_by_dist_params.go DefaultSearchByDist-
// InitialLimit); the for loop has no post statement, so later iterations only
// advance the params until MaxLimitReached.
extern "C" int wv_index_search_by_vector_distance(wv_index* idx, const float* query, int64_t d, float target,
                                                  int64_t max_limit, const uint64_t* allow_ids, int64_t n_allow,
                                                  int32_t allow_mode, uint64_t* out_ids, float* out_dists,
                                                  int32_t* out_count) {
    (void)max_limit;
    const int total_limit = 100;
    std::vector<uint64_t> ids(total_limit);
    std::vector<float> dd(total_limit);
    int32_t n = 0;
    int rc = wv_index_search_by_vector_batch(idx, query, 1, d, total_limit, allow_ids, n_allow, allow_mode, ids.data(),
                                             dd.data(), &n);
    if (rc) return rc;
    int m = 0;
    for (int i = 0; i < n && i < total_limit; i++) {
        double diff = std::fabs((double)dd[i] - (double)target);
        if (dd[i] <= target || diff <= 1e-6) { out_ids[m] = ids[i]; out_dists[m] = dd[i]; m++; }
        else break;
    }
    *out_count = m;
    return WV_OK;
}

extern "C" int wv_index_search_device(wv_index* idx, const float* d_queries, int64_t nq, int64_t d, int32_t k,
                                      int32_t mode, uint64_t* d_ids, float* d_dists, int32_t* d_counts,
                                      int32_t* d_flags, void* stream) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (mode == 1 && !d_flags) return set_err(WV_ERR_INVALID, "mode 1 needs d_flags");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    hipStream_t s = (hipStream_t)stream;  // NULL: the null stream (ordered with the caller's default-stream work)
    int rc = search_core(idx, s, d_queries, nq, d, k, mode, idx->present, idx->npresent, d_ids, d_dists, d_counts,
                         mode == 1 ? d_flags : nullptr);
    if (rc) return rc;
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

extern "C" int wv_index_replay(wv_index* idx, const float* d_queries, int64_t nq, int64_t d, int32_t k,
                               const int32_t* h_qlist, int32_t nlist, const uint64_t* h_in_ids,
                               const float* h_in_dists, const int32_t* h_in_len, int32_t extract,
                               uint64_t* h_out_ids, float* h_out_dists, int32_t* h_out_len) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (k <= 0 || nlist < 0) return set_err(WV_ERR_INVALID, "invalid k / list");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    hipStream_t s = idx->stream;
    if (nlist == 0) return WV_OK;
    const bool have_data = idx->dims != 0 && idx->npresent > 0;
    if (have_data && d != idx->dims)
        return set_err(WV_ERR_VECTOR_LENGTH, "%lld vs %d: vector lengths don't match", (long long)d, idx->dims);
    HIPCHK(idx->hI.ensure((size_t)nlist * k * sizeof(uint64_t) * 2));
    HIPCHK(idx->hD.ensure((size_t)nlist * k * sizeof(float) * 2));
    HIPCHK(idx->hN.ensure((size_t)nlist * sizeof(int32_t) * 2));
    HIPCHK(idx->qlist.ensure((size_t)nlist * sizeof(int32_t)));
    uint64_t* inI = idx->hI.as<uint64_t>();
    uint64_t* outI = inI + (size_t)nlist * k;
    float* inD = idx->hD.as<float>();
    float* outD = inD + (size_t)nlist * k;
    int32_t* inN = idx->hN.as<int32_t>();
    int32_t* outN = inN + nlist;
    if (h_in_len) {
        HIPCHK(hipMemcpyAsync(inI, h_in_ids, (size_t)nlist * k * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(inD, h_in_dists, (size_t)nlist * k * sizeof(float), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(inN, h_in_len, (size_t)nlist * sizeof(int32_t), hipMemcpyHostToDevice, s));
    } else {
        HIPCHK(hipMemsetAsync(inN, 0, (size_t)nlist * sizeof(int32_t), s));
    }
    HIPCHK(hipMemcpyAsync(idx->qlist.p, h_qlist, (size_t)nlist * sizeof(int32_t), hipMemcpyHostToDevice, s));
    const float* Qn = nullptr;
    if (have_data) {
        const int64_t nq_pad = round_up(nq, QB);
        int rc = prepare_queries(idx, s, d_queries, nq, nq_pad);
        if (rc) return rc;
        Qn = idx->qn.as<float>();
    }
    // list-ordered output rows (out_by_query = 0); an empty shard passes the
    // heaps through unchanged (zero tiles scanned)
    int rc2 = run_replay(idx, s, idx->present, Qn, idx->qlist.as<int32_t>(), nlist, k, inI, inD, h_in_len ? inN : nullptr,
                         extract, 0, k, outI, outD, outN);
    if (rc2) return rc2;
    HIPCHK(hipMemcpyAsync(h_out_ids, outI, (size_t)nlist * k * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(h_out_dists, outD, (size_t)nlist * k * sizeof(float), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(h_out_len, outN, (size_t)nlist * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

// wv_index_replay on device buffers (no host hops, stream-ordered).  With the
// block keys of this index's last search over the same nq queries still valid
// (qs_keys_nq), the scan visits only blocks that can insert (k_blk_replay);
// otherwise every row's exact distance is computed (run_replay).
// sharded two-phase exact search (weaviate_amd/sharded.py): phase 1 on the
// block-key path only (WV_ERR_UNSUPPORTED otherwise: the caller uses mode 1)
extern "C" int wv_index_shard_phase1(wv_index* idx, const float* d_queries, int64_t nq, int64_t d, int32_t k,
                                     float* d_topA, float* d_eps, void* stream) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (!d_topA || !d_eps) return set_err(WV_ERR_INVALID, "nil buffer");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    hipStream_t s = (hipStream_t)stream;
    idx->qs_keys_nq = 0;
    idx->qs_phase_nq = 0;
    const bool qs = idx->compression == WV_COMPRESSION_NONE && idx->qs_planes && !idx->has_nonfinite &&
                    (idx->kernel_opt == 0 || idx->kernel_opt == 7) && !idx->force_replay && qs_R(k) > 0 &&
                    idx->metric != WV_METRIC_HAMMING && idx->dims != 0 && idx->npresent > 0 && nq > 0;
    if (!qs) return set_err(WV_ERR_UNSUPPORTED, "two-phase shard search: not on the block-key path");
    if (d != idx->dims)
        return set_err(WV_ERR_VECTOR_LENGTH, "%lld vs %d: vector lengths don't match", (long long)d, idx->dims);
    if (k <= 0) return set_err(WV_ERR_INVALID, "k must be positive (reference heap Top() on empty queue)");
    int rc = prepare_queries(idx, s, d_queries, nq, round_up(nq, QS_QPB));
    if (rc) return rc;
    idx->stats.queries += (uint64_t)nq;
    idx->stats.batches++;
    rc = search_qs(idx, s, nq, k, 1, idx->present, nullptr, nullptr, nullptr, nullptr, 1, d_topA);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(d_eps, idx->qsEps.p, (size_t)nq * sizeof(float), hipMemcpyDeviceToDevice, s));
    idx->qs_phase_nq = nq;
    idx->qs_phase_k = k;
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

extern "C" int wv_index_shard_phase2(wv_index* idx, int32_t world, int64_t nq, const float* d_topA_all,
                                     const float* d_eps_all, int32_t k, uint64_t* d_ids, float* d_dists,
                                     int32_t* d_counts, int32_t* d_flags, void* stream) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (!d_topA_all || !d_eps_all || !d_ids || !d_dists || !d_counts || !d_flags)
        return set_err(WV_ERR_INVALID, "nil buffer");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    hipStream_t s = (hipStream_t)stream;
    if (idx->qs_phase_nq != nq || idx->qs_phase_k != k || world < 1)
        return set_err(WV_ERR_INVALID, "shard phase 2 without a matching phase 1 (nq %lld, k %d)", (long long)nq, k);
    idx->qs_phase_nq = 0;
    int rc = search_qs(idx, s, nq, k, 1, idx->present, d_ids, d_dists, d_counts, d_flags, 2, nullptr, d_topA_all,
                       d_eps_all, world);
    if (rc) return rc;
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

// the cross-shard replay of every query with d_flags[q] != 0, list built on the
// device; states and results indexed by query.  Needs this index's block keys
// of the same batch (wv_index_search_device mode 1 or the two phases).
extern "C" int wv_index_replay_flags_device(wv_index* idx, const float* d_queries, int64_t nq, int64_t d, int32_t k,
                                            const int32_t* d_flags, const uint64_t* d_in_ids, const float* d_in_dists,
                                            const int32_t* d_in_len, int32_t extract, uint64_t* d_out_ids,
                                            float* d_out_dists, int32_t* d_out_len, void* stream) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (k <= 0 || nq < 0 || !d_flags || !d_out_ids || !d_out_dists || !d_out_len)
        return set_err(WV_ERR_INVALID, "invalid arguments");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    hipStream_t s = (hipStream_t)stream;
    if (nq == 0) return WV_OK;
    const bool have_data = idx->dims != 0 && idx->npresent > 0;
    if (have_data && d != idx->dims)
        return set_err(WV_ERR_VECTOR_LENGTH, "%lld vs %d: vector lengths don't match", (long long)d, idx->dims);
    HIPCHK(idx->flCtr.ensure(2 * sizeof(uint32_t)));
    HIPCHK(idx->qsList.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(hipMemsetAsync(idx->flCtr.p, 0, 2 * sizeof(uint32_t), s));
    k_flag_list<<<(unsigned)((nq + 255) / 256), 256, 0, s>>>(d_flags, (int)nq, idx->qsList.as<int32_t>(),
                                                              idx->flCtr.as<uint32_t>(), 0);
    HIPCHK(hipGetLastError());
    if (!have_data || idx->qs_keys_nq != nq) {
        // no block keys of this batch (empty shard, non-finite rows, k or batch
        // off the block-key path): every row's exact distance + the id-ordered
        // heap (run_replay, states and results by query); one host sync for the
        // list length
        uint32_t nl = 0;
        HIPCHK(hipMemcpyAsync(&nl, idx->flCtr.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (nl == 0) return WV_OK;
        const float* Qn = nullptr;
        if (have_data) {
            int rc = prepare_queries(idx, s, d_queries, nq, round_up(nq, QB));
            if (rc) return rc;
            Qn = idx->qn.as<float>();
        }
        int rc = run_replay(idx, s, idx->present, Qn, idx->qsList.as<int32_t>(), (int)nl, k, d_in_ids, d_in_dists,
                            d_in_len, extract, 1, k, d_out_ids, d_out_dists, d_out_len, 1);
        if (rc) return rc;
        if (!stream) HIPCHK(hipStreamSynchronize(s));
        return WV_OK;
    }
    int rc = launch_blk_replay(idx, s, idx->qsKey.as<float>(), idx->qs_last_ldk, idx->qs_last_nb, idx->qsEps.as<float>(),
                               idx->qsInfo.as<float4>(), idx->present, idx->qn.as<float>(), idx->qsList.as<int32_t>(),
                               idx->flCtr.as<uint32_t>(), 0, nq, k, k, d_out_ids, d_out_dists, d_out_len, d_in_ids,
                               d_in_dists, d_in_len, extract, 0);
    if (rc) return rc;
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

// parallel cross-shard replay (weaviate_amd/sharded.py): this shard's replay of
// the listed queries from heap states d_in_* (by list position), recording every
// insertion (ids, dists [nlist][cap], counts [nlist], cap + 1 = overflow)
extern "C" int wv_index_replay_record_device(wv_index* idx, const float* d_queries, int64_t nq, int64_t d, int32_t k,
                                             const int32_t* d_qlist, int32_t nlist, const uint64_t* d_in_ids,
                                             const float* d_in_dists, const int32_t* d_in_len, int32_t cap,
                                             uint64_t* d_rec_ids, float* d_rec_dists, int32_t* d_rec_n, void* stream) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (k <= 0 || nlist < 0 || cap < 1) return set_err(WV_ERR_INVALID, "invalid arguments");
    if (nlist == 0) return WV_OK;
    if (!d_qlist || !d_rec_ids || !d_rec_dists || !d_rec_n) return set_err(WV_ERR_INVALID, "nil buffer");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    hipStream_t s = (hipStream_t)stream;
    if (nlist == 0) return WV_OK;
    const bool have_data = idx->dims != 0 && idx->npresent > 0;
    if (!have_data) {
        HIPCHK(hipMemsetAsync(d_rec_n, 0, (size_t)nlist * sizeof(int32_t), s));
        return WV_OK;
    }
    if (d != idx->dims)
        return set_err(WV_ERR_VECTOR_LENGTH, "%lld vs %d: vector lengths don't match", (long long)d, idx->dims);
    HIPCHK(idx->hI.ensure((size_t)nlist * k * sizeof(uint64_t)));
    HIPCHK(idx->hD.ensure((size_t)nlist * k * sizeof(float)));
    HIPCHK(idx->hN.ensure((size_t)nlist * sizeof(int32_t)));
    if (idx->qs_keys_nq != nq || !blk_pooled(idx, k, idx->qs_last_nb)) {
        // no block keys of this batch (or k outside the pooled replay): the
        // all-rows exact replay records the same insertions
        int rc = prepare_queries(idx, s, d_queries, nq, round_up(nq, QB));
        if (rc) return rc;
        rc = run_replay(idx, s, idx->present, idx->qn.as<float>(), d_qlist, nlist, k, d_in_ids, d_in_dists, d_in_len, 0,
                        0, k, idx->hI.as<uint64_t>(), idx->hD.as<float>(), idx->hN.as<int32_t>(), 0, d_rec_ids,
                        d_rec_dists, d_rec_n, cap);
        if (rc) return rc;
        if (!stream) HIPCHK(hipStreamSynchronize(s));
        return WV_OK;
    }
    int rc = launch_blk_replay(idx, s, idx->qsKey.as<float>(), idx->qs_last_ldk, idx->qs_last_nb, idx->qsEps.as<float>(),
                               idx->qsInfo.as<float4>(), idx->present, idx->qn.as<float>(), d_qlist, nullptr, nlist,
                               nlist, k, k, idx->hI.as<uint64_t>(), idx->hD.as<float>(), idx->hN.as<int32_t>(), d_in_ids,
                               d_in_dists, d_in_len, 0, 1, d_rec_ids, d_rec_dists, d_rec_n, cap);
    if (rc) return rc;
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

extern "C" int wv_heap_merge_records(int32_t device, int32_t nlist, int32_t k, int32_t world, int32_t cap,
                                     const uint64_t* d_st_ids, const float* d_st_dists, const int32_t* d_st_n,
                                     const uint64_t* d_rec_ids, const float* d_rec_dists, const int32_t* d_rec_n,
                                     uint64_t* d_out_ids, float* d_out_dists, int32_t* d_out_n,
                                     int32_t* d_unresolved, void* stream) {
    if (k <= 0 || nlist < 0 || world < 1 || cap < 1) return set_err(WV_ERR_INVALID, "invalid arguments");
    if (nlist == 0) return WV_OK;
    HIPCHK(hipSetDevice(device));
    hipStream_t s = (hipStream_t)stream;
    const size_t lds = (size_t)k * (sizeof(uint64_t) + sizeof(float)) + 16;
    if (lds > 64 * 1024)
        HIPCHK(hipFuncSetAttribute((const void*)k_heap_merge_records, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    k_heap_merge_records<<<(unsigned)nlist, 64, lds, s>>>(nlist, k, world, cap, d_st_ids, d_st_dists, d_st_n, d_rec_ids,
                                                          d_rec_dists, d_rec_n, d_out_ids, d_out_dists, d_out_n,
                                                          d_unresolved);
    HIPCHK(hipGetLastError());
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

extern "C" int wv_index_replay_device(wv_index* idx, const float* d_queries, int64_t nq, int64_t d, int32_t k,
                                      const int32_t* d_qlist, int32_t nlist, const uint64_t* d_in_ids,
                                      const float* d_in_dists, const int32_t* d_in_len, int32_t extract,
                                      uint64_t* d_out_ids, float* d_out_dists, int32_t* d_out_len, void* stream) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (k <= 0 || nlist < 0) return set_err(WV_ERR_INVALID, "invalid k / list");
    if (nlist > 0 && (!d_qlist || !d_out_ids || !d_out_dists || !d_out_len)) return set_err(WV_ERR_INVALID, "nil buffer");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    hipStream_t s = (hipStream_t)stream;  // NULL: the null stream (ordered with the caller's default-stream work)
    if (nlist == 0) return WV_OK;
    const bool have_data = idx->dims != 0 && idx->npresent > 0;
    if (have_data && d != idx->dims)
        return set_err(WV_ERR_VECTOR_LENGTH, "%lld vs %d: vector lengths don't match", (long long)d, idx->dims);
    const size_t rlds = (size_t)k * sizeof(uint64_t) + 64 * sizeof(float) + (size_t)k * sizeof(float) + 16 + 16 * 64 * sizeof(float);
    const bool keyed = have_data && idx->qs_keys_nq == nq && rlds <= 160 * 1024;
    if (keyed) {
        const float* Qn = idx->qn.as<float>();  // the prepared rows of that batch
        return launch_blk_replay(idx, s, idx->qsKey.as<float>(), idx->qs_last_ldk, idx->qs_last_nb,
                                 idx->qsEps.as<float>(), idx->qsInfo.as<float4>(), idx->present, Qn, d_qlist, nullptr,
                                 nlist, nlist, k, k, d_out_ids, d_out_dists, d_out_len, d_in_ids, d_in_dists, d_in_len,
                                 extract, 1);
    }
    const float* Qn = nullptr;
    if (have_data) {
        int rc = prepare_queries(idx, s, d_queries, nq, round_up(nq, QB));
        if (rc) return rc;
        Qn = idx->qn.as<float>();
    }
    // run_replay reads in-state when in_n != nullptr; list-ordered outputs
    return run_replay(idx, s, idx->present, Qn, d_qlist, nlist, k, d_in_ids, d_in_dists, d_in_len, extract, 0, k,
                      d_out_ids, d_out_dists, d_out_len);
}

extern "C" int wv_merge_shards(int32_t device, int32_t nshards, int64_t nq, int32_t k, const uint64_t* d_ids,
                               const float* d_dists, const int32_t* d_counts, const int32_t* d_flags,
                               uint64_t* d_out_ids, float* d_out_dists, int32_t* d_out_counts, int32_t* d_out_flags,
                               void* stream) {
    HIPCHK(hipSetDevice(device));
    const int64_t n = (int64_t)nshards * (k + 1);
    hipStream_t s = (hipStream_t)stream;
    unsigned grid = (unsigned)((nq + 3) / 4);
    if (n <= 64) k_merge_shards<1><<<grid, 256, 0, s>>>(nshards, nq, k, d_ids, d_dists, d_counts, d_flags, d_out_ids, d_out_dists, d_out_counts, d_out_flags);
    else if (n <= 128) k_merge_shards<2><<<grid, 256, 0, s>>>(nshards, nq, k, d_ids, d_dists, d_counts, d_flags, d_out_ids, d_out_dists, d_out_counts, d_out_flags);
    else if (n <= 256) k_merge_shards<4><<<grid, 256, 0, s>>>(nshards, nq, k, d_ids, d_dists, d_counts, d_flags, d_out_ids, d_out_dists, d_out_counts, d_out_flags);
    else if (n <= 512) k_merge_shards<8><<<grid, 256, 0, s>>>(nshards, nq, k, d_ids, d_dists, d_counts, d_flags, d_out_ids, d_out_dists, d_out_counts, d_out_flags);
    else return set_err(WV_ERR_UNSUPPORTED, "merge: nshards*(k+1) > 512");
    HIPCHK(hipGetLastError());
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

// ---------------------------------------------------------------------------
// stateless distancer entry points
// ---------------------------------------------------------------------------
extern "C" int wv_distance_batch(int32_t device, int32_t metric, int32_t variant, const float* a, const float* b,
                                 int64_t n, int64_t d, float* out) {
    HIPCHK(hipSetDevice(device));
    if (n <= 0) return WV_OK;
    const int v = wv_resolve_variant(variant);
    const int ld = (int)round_up(d, 4);  // 16-byte aligned rows for the float4 loads
    DBuf A, B, O;
    HIPCHK(A.ensure((size_t)n * ld * sizeof(float)));
    HIPCHK(B.ensure((size_t)n * ld * sizeof(float)));
    HIPCHK(O.ensure((size_t)n * sizeof(float)));
    HIPCHK(hipMemcpy2D(A.p, ld * sizeof(float), a, d * sizeof(float), d * sizeof(float), n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy2D(B.p, ld * sizeof(float), b, d * sizeof(float), d * sizeof(float), n, hipMemcpyHostToDevice));
    unsigned grid = (unsigned)((n + 255) / 256);
#define WV_DP(M, V) k_distance_pairs<M, V><<<(unsigned)((n + 63) / 64), 64>>>(A.as<float>(), B.as<float>(), n, (int)d, ld, O.as<float>())
    const bool v5 = v == WV_VARIANT_AVX512;
    switch (metric) {
    case WV_METRIC_L2_SQUARED: if (v5) WV_DP(L2, AVX512); else WV_DP(L2, AVX256); break;
    case WV_METRIC_DOT: if (v5) WV_DP(DOT, AVX512); else WV_DP(DOT, AVX256); break;
    case WV_METRIC_COSINE_DOT: if (v5) WV_DP(COSINE, AVX512); else WV_DP(COSINE, AVX256); break;
    case WV_METRIC_HAMMING: WV_DP(HAMMING, AVX256); break;
    default: A.release(); B.release(); O.release(); return set_err(WV_ERR_INVALID, "unknown metric %d", metric);
    }
#undef WV_DP
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(out, O.p, (size_t)n * sizeof(float), hipMemcpyDeviceToHost);
    A.release(); B.release(); O.release();
    if (e != hipSuccess) return set_err(WV_ERR_HIP, "distance_batch: %s", hipGetErrorString(e));
    return WV_OK;
}

extern "C" int wv_hamming_bitwise_batch(int32_t device, const uint64_t* a, const uint64_t* b, int64_t n,
                                        int64_t words, float* out) {
    HIPCHK(hipSetDevice(device));
    if (n <= 0) return WV_OK;
    DBuf A, B, O;
    HIPCHK(A.ensure((size_t)n * words * 8));
    HIPCHK(B.ensure((size_t)n * words * 8));
    HIPCHK(O.ensure((size_t)n * 4));
    HIPCHK(hipMemcpy(A.p, a, (size_t)n * words * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(B.p, b, (size_t)n * words * 8, hipMemcpyHostToDevice));
    k_hamming_pairs<<<(unsigned)((n + 255) / 256), 256>>>(A.as<uint64_t>(), B.as<uint64_t>(), n, (int)words,
                                                          O.as<float>());
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(out, O.p, (size_t)n * 4, hipMemcpyDeviceToHost);
    A.release(); B.release(); O.release();
    if (e != hipSuccess) return set_err(WV_ERR_HIP, "hamming: %s", hipGetErrorString(e));
    return WV_OK;
}

extern "C" int wv_bq_encode_batch(int32_t device, const float* vecs, int64_t n, int64_t d, uint64_t* out_codes) {
    HIPCHK(hipSetDevice(device));
    if (n <= 0) return WV_OK;
    const int64_t words = (d + 63) / 64;
    DBuf A, O;
    HIPCHK(A.ensure((size_t)n * d * 4));
    HIPCHK(O.ensure((size_t)n * words * 8));
    HIPCHK(hipMemcpy(A.p, vecs, (size_t)n * d * 4, hipMemcpyHostToDevice));
    k_bq_encode<<<(unsigned)((n * words + 255) / 256), 256>>>(A.as<float>(), n, (int)d, (int)d, O.as<uint64_t>());
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(out_codes, O.p, (size_t)n * words * 8, hipMemcpyDeviceToHost);
    A.release(); O.release();
    if (e != hipSuccess) return set_err(WV_ERR_HIP, "bq_encode: %s", hipGetErrorString(e));
    return WV_OK;
}

extern "C" int wv_normalize_batch(int32_t device, const float* vecs, int64_t n, int64_t d, float* out) {
    HIPCHK(hipSetDevice(device));
    if (n <= 0) return WV_OK;
    DBuf A, O;
    HIPCHK(A.ensure((size_t)n * d * 4));
    HIPCHK(O.ensure((size_t)n * d * 4));
    HIPCHK(hipMemcpy(A.p, vecs, (size_t)n * d * 4, hipMemcpyHostToDevice));
    k_normalize_rows<<<(unsigned)((n + 3) / 4), 256>>>(A.as<float>(), n, (int)d, O.as<float>(), (int)d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(out, O.p, (size_t)n * d * 4, hipMemcpyDeviceToHost);
    A.release(); O.release();
    if (e != hipSuccess) return set_err(WV_ERR_HIP, "normalize: %s", hipGetErrorString(e));
    return WV_OK;
}

extern "C" int wv_gen_device(int32_t device, int32_t kind, uint64_t seed, uint64_t row0, int64_t rows, int64_t d,
                             float* d_out, void* stream) {
    HIPCHK(hipSetDevice(device));
    int64_t n = rows * d;
    if (n <= 0) return WV_OK;
    k_gen<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(kind, seed, row0, rows, (int)d, d_out);
    HIPCHK(hipGetLastError());
    if (!stream) HIPCHK(hipStreamSynchronize(nullptr));
    return WV_OK;
}

// LSM segment restore (host-only; uses add_rows_locked / wv_index_delete above)
#include "lsm_segment.hip"

// Iterate, QueryVectorDistancer, Preload, UpdateUserConfig, CompressionStats
#include "vector_index.hip"

// micro-batcher of concurrent single-query SearchByVector calls
#include "batcher.hip"
