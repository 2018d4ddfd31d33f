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
#include "rt_index.h"
#include <cpuid.h>
#include <functional>
#include <map>

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string g_err;

int set_err(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}


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
// dims fixed (config or first Add, initializeDimensionsAndRQ flat/index.go:338-360)
static void set_dims(wv_index* idx, int64_t d) {
    idx->dims = (int)d;
    idx->dpad = (int)round_up(d, BK);
    idx->dpb = (int)round_up(d, 128);
    if (idx->dpb > QS_W4_DPB) idx->dpb = (int)round_up(d, 512);  // 512-column ring parts
    idx->qs_planes = (idx->use_qs && idx->dpb <= QS_MAX_DPB) ? 1 : 0;
    // int8 plane: 128-column multiples up to 768 (two blocks per ring slot),
    // 256-column multiples above (one block per slot), <= 48 KiB per slot
    idx->dpb8 = (int)(d <= 768 ? round_up(d, 128) : round_up(d, 256));
    idx->q8_planes = (idx->qs_planes && d > 384 && idx->dpb8 <= 1536) ? 1 : 0;
    // above 1536 dims: int8 planes only (no bf16 plane), 512-column multiples up
    // to 3072 -- two column parts of 16 / 20 / 24 chunks per block (k_q8_blockkey_cp);
    // 1024-column multiples up to 6144 -- 4 / 5 / 6 parts of 16 chunks
    idx->q8_only = (idx->use_qs && !idx->qs_planes && d > 1536 && round_up(d, 1024) <= Q8_WIDE_DPB) ? 1 : 0;
    if (idx->q8_only) {
        idx->dpb8 = (int)(round_up(d, 512) <= Q8_MAX_DPB ? round_up(d, 512) : round_up(d, 1024));
        idx->q8_planes = 1;
    }
    if (idx->compression == WV_COMPRESSION_BQ) {  // +-1 code plane: 7..24 words (448..1536 bits)
        const int w = (int)((d + 63) / 64), bits = 64 * w;
        idx->dpb8b = (w >= 7 && w <= 24) ? (int)(bits <= 768 ? round_up(bits, 128) : round_up(bits, 256)) : 0;
    }
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
    idx->id_base0 = cfg->id_base;
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
    if (e == hipSuccess) e = hipMalloc(&idx->qmax8, 4 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(idx->qmax8, 0, 4 * sizeof(uint32_t));
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
    // rq with the dimension configured: the (seeded, dimension-only) rotation
    // now rather than at the first Add, so an empty shard can answer a search
    if (idx->rq_bits && idx->dims > 0) {
        const int rc = rq_init(idx);
        if (rc) {
            wv_index_destroy(idx);
            return rc;
        }
    }
    *out = idx;
    return WV_OK;
}

extern "C" void wv_index_destroy(wv_index* idx) {
    if (!idx) return;
    if (idx->sub) wv_index_destroy(idx->sub);
    hipSetDevice(idx->device);
    batcher_free(idx, idx->batcher);
    if (idx->stream) hipStreamSynchronize(idx->stream);
    if (idx->g_exec) hipGraphExecDestroy(idx->g_exec);
    if (idx->g_graph) hipGraphDestroy(idx->g_graph);
    for (DBuf* b : {&idx->stage, &idx->slots, &idx->qraw, &idx->qn, &idx->qn2, &idx->spanA, &idx->spanI, &idx->candA,
                    &idx->candI, &idx->candE, &idx->oIds, &idx->oD, &idx->oN, &idx->oF, &idx->valid, &idx->qlist,
                    &idx->hI, &idx->hD, &idx->hN, &idx->rE, &idx->rB, &idx->qcodes, &idx->bqmin, &idx->cslot,
                    &idx->cn, &idx->ident, &idx->lut, &idx->ascI, &idx->ascD, &idx->ascN, &idx->rqq, &idx->rqm,
                    &idx->rE2, &idx->rB2, &idx->gmA, &idx->gmI, &idx->qsQb, &idx->qsInfo, &idx->qsKey, &idx->qsCand,
                    &idx->qsNc, &idx->qsEps, &idx->qsFlags, &idx->qsList, &idx->qsScratch, &idx->rpBlk, &idx->rpLb,
                    &idx->rpQ, &idx->rpE, &idx->rpVm, &idx->rpOff, &idx->rpTot, &idx->rpCtr, &idx->flCtr,
                    &idx->q8Qb, &idx->q8Scale, &idx->q8Info, &idx->q8Blk})
        b->release();
    if (idx->aux) hipStreamSynchronize(idx->aux);
    for (hipEvent_t e : {idx->evd[0], idx->evd[1], idx->evr[0], idx->evr[1]})
        if (e) hipEventDestroy(e);
    if (idx->aux) hipStreamDestroy(idx->aux);
    if (idx->sq_codes) hipFree(idx->sq_codes);
    if (idx->sq_meta) hipFree(idx->sq_meta);
    idx->sqq.release();
    idx->sqm.release();
    if (idx->pq8_X8) hipFree(idx->pq8_X8);
    if (idx->pq8_sb) hipFree(idx->pq8_sb);
    if (idx->pq8_n2) hipFree(idx->pq8_n2);
    if (idx->X) hipFree(idx->X);
    if (idx->xnorm2) hipFree(idx->xnorm2);
    if (idx->present) hipFree(idx->present);
    if (idx->d_maxn2) hipFree(idx->d_maxn2);
    if (idx->codes) hipFree(idx->codes);
    if (idx->pq_centers) hipFree(idx->pq_centers);
    if (idx->pq_codes) hipFree(idx->pq_codes);
    if (idx->Xb) hipFree(idx->Xb);
    if (idx->qsmax) hipFree(idx->qsmax);
    if (idx->X8) hipFree(idx->X8);
    if (idx->bq8) hipFree(idx->bq8);
    if (idx->sb8) hipFree(idx->sb8);
    if (idx->qmax8) hipFree(idx->qmax8);
    if (idx->qscount) hipFree(idx->qscount);
    for (void* p : {(void*)idx->rq_src, (void*)idx->rq_sign, (void*)idx->rq_round, idx->rq_codes, (void*)idx->rq_meta,
                    (void*)idx->rq1_pm})
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
    note_mutation(idx);
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
    unsigned char* x8 = nullptr;
    float* sb8 = nullptr;
    unsigned char* b8 = nullptr;
    void* rqc = nullptr;
    float4* rqm = nullptr;
    unsigned char* rpm = nullptr;
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
    if (idx->compression == WV_COMPRESSION_BQ && idx->dpb8b > 0)
        WV_STEP("bq +-1 plane", alloc((void**)&b8, (size_t)nc * idx->dpb8b));
    if (idx->qs_planes) WV_STEP("bf16 block-key plane", alloc((void**)&xb, qs_b));
    if (idx->q8_planes) {
        WV_STEP("int8 block-key plane", alloc((void**)&x8, (size_t)nc * idx->dpb8));
        WV_STEP("int8 block scales", alloc((void**)&sb8, (size_t)(nc / 32) * sizeof(float)));
    }
    if (idx->rq_ready) {
        WV_STEP("rq codes", alloc(&rqc, rq_cb));
        WV_STEP("rq meta", alloc((void**)&rqm, (size_t)nc * RQ_META_B));
        if (idx->rq_bits == 1) WV_STEP("rq-1 +-1 plane", alloc((void**)&rpm, (size_t)nc * idx->rq_D));
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
    if (b8) {  // 256-row tiles: the old tiles are a prefix
        WV_STEP("memset", hipMemsetAsync(b8, 0, (size_t)nc * idx->dpb8b, s));
        if (oc > 0 && idx->bq8)
            WV_STEP("copy", hipMemcpyAsync(b8, idx->bq8, (size_t)oc * idx->dpb8b, hipMemcpyDeviceToDevice, s));
    }
    if (x8) {  // 256-row tiles: the old tiles are a prefix
        WV_STEP("memset", hipMemsetAsync(x8, 0, (size_t)nc * idx->dpb8, s));
        WV_STEP("memset", hipMemsetAsync(sb8, 0, (size_t)(nc / 32) * sizeof(float), s));
        if (oc > 0 && idx->X8) {
            WV_STEP("copy", hipMemcpyAsync(x8, idx->X8, (size_t)oc * idx->dpb8, hipMemcpyDeviceToDevice, s));
            WV_STEP("copy", hipMemcpyAsync(sb8, idx->sb8, (size_t)(oc / 32) * sizeof(float), hipMemcpyDeviceToDevice, s));
        }
    }
    if (rqc) {
        WV_STEP("memset", hipMemsetAsync(rqc, 0, rq_cb, s));
        WV_STEP("memset", hipMemsetAsync(rqm, 0, (size_t)nc * RQ_META_B, s));
        if (rpm) {  // 256-row tiles: the old tiles are a prefix
            WV_STEP("memset", hipMemsetAsync(rpm, 0, (size_t)nc * idx->rq_D, s));
            if (oc > 0 && idx->rq1_pm)
                WV_STEP("copy", hipMemcpyAsync(rpm, idx->rq1_pm, (size_t)oc * idx->rq_D, hipMemcpyDeviceToDevice, s));
        }
        if (oc > 0 && idx->rq_codes) {
            if (idx->rq_bits == 8)  // tiles of 256 rows are contiguous: the old tiles are a prefix
                WV_STEP("copy", hipMemcpyAsync(rqc, idx->rq_codes, (size_t)oc * idx->rq_D, hipMemcpyDeviceToDevice, s));
            else
                WV_STEP("copy", hipMemcpy2DAsync(rqc, (size_t)nc * sizeof(uint64_t), idx->rq_codes,
                                                 (size_t)oc * sizeof(uint64_t), (size_t)oc * sizeof(uint64_t),
                                                 idx->rq_D / 64, hipMemcpyDeviceToDevice, s));
            WV_STEP("copy", hipMemcpyAsync(rqm, idx->rq_meta, (size_t)oc * sizeof(float4), hipMemcpyDeviceToDevice, s));
            if (idx->rq_bits == 8)  // the code sums behind the meta
                WV_STEP("copy", hipMemcpyAsync(reinterpret_cast<uint32_t*>(rqm + nc), rq_csum(idx),
                                               (size_t)oc * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
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
    swap_in(idx->X8, x8);
    swap_in(idx->bq8, b8);
    swap_in(idx->sb8, sb8);
    if (rqc) {
        if (idx->rq_codes) hipFree(idx->rq_codes);
        idx->rq_codes = rqc;
        swap_in(idx->rq_meta, rqm);
        swap_in(idx->rq1_pm, rpm);
    }
    swap_in(idx->pq_codes, pc);
    swap_in(idx->sq_codes, sqc);
    swap_in(idx->sq_meta, sqmt);
    idx->cap = nc;
    idx->h_present.resize((size_t)nc, 0);
    if (idx->pq8_X8) {  // the PQ reconstruction plane is reallocated and rebuilt at the next search
        hipFree(idx->pq8_X8); hipFree(idx->pq8_sb); hipFree(idx->pq8_n2);
        idx->pq8_X8 = nullptr; idx->pq8_sb = nullptr; idx->pq8_n2 = nullptr;
        idx->pq8_cap = 0;
    }
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
void launch_pq_encode(wv_index* idx, int64_t n, const uint32_t* d_slots) {
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
void launch_rq_encode(wv_index* idx, hipStream_t s, const float* rows, int64_t ld, int64_t n,
                             const uint32_t* d_slots, int query, void* codes, int64_t cap, float4* meta,
                             uint32_t* csum, unsigned char* pm) {
    if (n <= 0) return;
    const size_t lds = 2 * (size_t)idx->rq_D * sizeof(float);
    const bool v5 = idx->variant == WV_VARIANT_AVX512;
#define WV_RQE(B, V, Q) k_rq_encode<B, V, Q><<<(unsigned)n, 256, lds, s>>>(rows, ld, n, idx->dims, d_slots, idx->rq_D, idx->rq_src, idx->rq_sign, idx->rq_round, codes, cap, meta, csum, pm)
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
        launch_rq_encode(idx, idx->stream, idx->X, idx->dpad, n, d_slots, 0, idx->rq_codes, idx->cap, idx->rq_meta,
                         idx->rq_bits == 8 ? rq_csum(idx) : nullptr, idx->rq1_pm);
    if (idx->compression == WV_COMPRESSION_BQ) {  // Preload: quantizer.Encode of the stored row (flat/index.go:376)
        const int64_t nt = n * idx->words;
        k_bq_encode_rows<<<(unsigned)((nt + 255) / 256), 256, 0, idx->stream>>>(idx->X, idx->dpad, n, idx->dims, d_slots,
                                                                                 idx->codes, idx->cap);
        if (idx->bq8) {  // the +-1 plane of the same codes (integer-MFMA block minima)
            const int64_t nu = n * (idx->dpb8b / 4);
            k_bq_unpack8<<<(unsigned)((nu + 255) / 256), 256, 0, idx->stream>>>(idx->codes, idx->cap, idx->words, n,
                                                                                d_slots, idx->dpb8b, idx->bq8);
        }
    }
}

// the int8 plane of every 32-row block holding one of the written slots
// (host slot list): each block is re-quantised whole (its scale is the
// block's max |x|), after the rows themselves were stored
static int requant_blocks(wv_index* idx, const uint32_t* h_slots, int64_t n) {
    if (idx->compression == WV_COMPRESSION_PQ && idx->pq_trained && n > 0) {
        const auto mm = std::minmax_element(h_slots, h_slots + n);
        pq8_mark(idx, (int64_t)*mm.first, (int64_t)*mm.second + 1);
    }
    if (!idx->q8_planes || n <= 0) return WV_OK;
    std::vector<uint32_t> blk((size_t)n);
    for (int64_t i = 0; i < n; i++) blk[(size_t)i] = h_slots[i] >> 5;
    std::sort(blk.begin(), blk.end());
    blk.erase(std::unique(blk.begin(), blk.end()), blk.end());
    HIPCHK(idx->q8Blk.ensure(blk.size() * sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(idx->q8Blk.p, blk.data(), blk.size() * sizeof(uint32_t), hipMemcpyHostToDevice, idx->stream));
    k_block_q8<<<(unsigned)blk.size(), 256, 0, idx->stream>>>(idx->X, idx->dpad, idx->dims, idx->dpb8,
                                                              idx->q8Blk.as<uint32_t>(), 0, idx->X8, idx->sb8,
                                                              idx->qmax8);
    HIPCHK(hipGetLastError());
    // the host list is read by the copy: keep it alive until the stream passes it
    HIPCHK(hipStreamSynchronize(idx->stream));
    return WV_OK;
}

// host mirror of the device non-finite flag (rows with NaN/Inf route the exact
// search to the all-rows path); called after a synchronised Add
static int refresh_nonfinite(wv_index* idx) {
    if (!(idx->qs_planes || idx->q8_only) || idx->has_nonfinite) return WV_OK;
    uint32_t f = 0;
    // bf16 plane builder's flag, or k_block_q8's on the int8-only planes
    HIPCHK(hipMemcpy(&f, idx->q8_only ? idx->qmax8 + 2 : idx->qsmax + 2, sizeof(uint32_t), hipMemcpyDeviceToHost));
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
    invalidate_batch(idx); note_mutation(idx);
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
        rc = requant_blocks(idx, hslots.data(), (int64_t)m);
        if (rc) return rc;
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
    invalidate_batch(idx); note_mutation(idx);
    rc = ensure_capacity(idx, s0 + n);
    if (rc) return rc;
    std::vector<uint32_t> hs((size_t)n);
    for (int64_t i = 0; i < n; i++) hs[i] = (uint32_t)(s0 + i);
    HIPCHK(idx->slots.ensure((size_t)n * sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(idx->slots.p, hs.data(), (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice, idx->stream));
    launch_prepare(idx, d_vecs, n, idx->slots.as<uint32_t>());
    HIPCHK(hipGetLastError());
    rc = requant_blocks(idx, hs.data(), n);
    if (rc) return rc;
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
    invalidate_batch(idx); note_mutation(idx);
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
    note_mutation(idx);
    if (k == "graph") { idx->graph_opt = value ? 1 : 0; return WV_OK; }
    if (k == "sel_filter") { idx->sel_filter = value ? 1 : 0; return WV_OK; }
    if (k == "batch_window_us") { if (value < 0 || value > 1000000) return set_err(WV_ERR_INVALID, "batch_window_us out of range"); idx->batch_window_us = value; return WV_OK; }
    if (k == "exact_multi") { idx->exact_multi = value ? 1 : 0; return WV_OK; }
    if (k == "gemv_wg") { if (value < 8 || value > 65536) return set_err(WV_ERR_INVALID, "gemv_wg out of range"); idx->gemv_wg = (int)value; return WV_OK; }
    if (k == "gemv_max") { if (value < 0 || value > 4096) return set_err(WV_ERR_INVALID, "gemv_max out of range"); idx->gemv_max = (int)value; return WV_OK; }
    if (k == "batch_max") { if (value < 1) return set_err(WV_ERR_INVALID, "batch_max out of range"); idx->batch_max = value; return WV_OK; }
    if (k == "margin") { if (value < 2 || value > 30) return set_err(WV_ERR_INVALID, "margin out of range"); idx->margin = (int)value; }
    else if (k == "force_replay") idx->force_replay = (int)value;
    else if (k == "spans") idx->spans_opt = (int)value;
    else if (k == "replay_dbg") idx->replay_dbg = value != 0;  // diagnostics: k_blk_replay clock totals (printf)
    else if (k == "pq_adc3") {  // 2: k_pq_adc4 (16-byte LUT reads, default), 1: k_pq_adc3, 0: k_pq_adc2
#ifdef WV_PQ_DBG  // 3, 4, 5: timing experiments (wrong results), debug builds only
        if (value < 0 || value > 5) return set_err(WV_ERR_INVALID, "pq_adc3 must be 0..5");
#else
        if (value < 0 || value > 2) return set_err(WV_ERR_INVALID, "pq_adc3 must be 0, 1 or 2");
#endif
        idx->pq_adc3 = (int)value;
    }
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
    else if (k == "q8_bm") idx->q8_bm = value ? 1 : 0;
    else if (k == "pq8") idx->pq8_opt = value ? 1 : 0;
    else if (k == "q8_gemv") idx->q8_gemv = value ? 1 : 0;
    else if (k == "q8_live") idx->q8_live = value ? 1 : 0;
    else if (k == "q8_prio") idx->q8_prio = value ? 1 : 0;
    else if (k == "sel_split_max") idx->sel_split_max = value;
    else if (k == "rq_mfma") idx->rq_mfma = value ? 1 : 0;
    else if (k == "q8_bm_min") idx->q8_bm_min = value;
    else if (k == "rq_serial") idx->rq_serial = (int)value;
    else if (k == "exact_cap") idx->exact_cap = value ? 1 : 0;
    else if (k == "exact_filter") idx->exact_filter = value ? 1 : 0;  // 0: every candidate row gets its exact distance
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
    else if (k == "q8") idx->q8_opt = value ? 1 : 0;  // int8 block keys (default 1) or bf16 (0)
    else if (k == "q8_filter") idx->q8_filter = value ? 1 : 0;
    else if (k == "q8_stag") idx->q8_stag = value ? 1 : 0;  // staggered epilogues of the int8 key kernel
    else if (k == "q8_pf") {  // int8 key kernel: A-fragment prefetch distance
        if (value != 1 && value != 2) return set_err(WV_ERR_INVALID, "q8_pf must be 1 or 2");
        idx->q8_pf = (int)value;
    }
    else if (k == "q8_shape") {  // int8 key kernel MFMA shape
        if (value != 16 && value != 32) return set_err(WV_ERR_INVALID, "q8_shape must be 16 or 32");
        idx->q8_shape = (int)value;
    }
    else if (k == "bq8") idx->bq8_opt = value ? 1 : 0;      // BQ block minima on the integer MFMA (1) or VALU (0)
    else if (k == "pqa") idx->pqa = value ? 1 : 0;
    else if (k == "sel_lower") idx->sel_lower = value ? 1 : 0;  // per-query allow lists share one block-key launch
    else if (k == "pqa_alone") idx->pqa_alone = value ? 1 : 0;  // unresolved per-query lists searched alone
    else if (k == "pqa_keys") idx->pqa_keys = value ? 1 : 0;    // per-query masked int8 keys
    else if (k == "bq_fast") idx->bq_fast = value ? 1 : 0;  // replay-free BQ answers when ties cannot matter
    else if (k == "rp_few") idx->rp_few = value;  // replay lists up to this long (device-counted) take the one-launch form
    else if (k == "batch_rows") idx->batch_rows = value ? 1 : 0;  // batcher: dense lists as slot bitmaps
    else if (k == "pqa_split_max") idx->pqa_split_max = std::max<int64_t>(value, 0);  // sparse lists searched alone
    else if (k == "pqa_budget_mb") idx->pqa_budget_mb = std::max<int64_t>(value, 1);
    else if (k == "scan_window") idx->scan_window = value ? 1 : 0;  // allow lists scan their slot span only
    else if (k == "gather_max") {  // sparse allow lists up to this many rows: gathered sub-index search
        if (value < 0 || value > (1ll << 28)) return set_err(WV_ERR_INVALID, "gather_max out of range");
        idx->gather_max = value;
    }  // int8 keys: row bound from the int8 plane (1) or bf16 (0)
    else if (k == "q8_R") {
        if (value != 0 && value != 2 && value != 4 && value != 8) return set_err(WV_ERR_INVALID, "q8_R must be 0, 2, 4 or 8");
        idx->q8_R = (int)value;
    }
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
    if (idx->stats.last_route == WV_ROUTE_RQ8_INT8) {  // rq: the exact 32-row minima themselves, eps 0
        if (q < 0 || q >= idx->rq_dbg_nq) return set_err(WV_ERR_INVALID, "debug_blockkeys: no such query");
        *nb = idx->rq_dbg_nb;
        if (!A) return WV_OK;
        HIPCHK(hipStreamSynchronize(idx->stream));
        HIPCHK(hipMemcpy(A, idx->qsKey.as<float>() + q * idx->rq_dbg_nb, (size_t)idx->rq_dbg_nb * sizeof(float),
                         hipMemcpyDeviceToHost));
        if (eps) *eps = 0.f;
        return WV_OK;
    }
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
double gamma_n(int n) {
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
int run_replay(wv_index* idx, hipStream_t s, const uint32_t* valid, const float* Qn, const int32_t* d_qlist,
                      int nlist, int k, const uint64_t* in_i, const float* in_d, const int32_t* in_n, int extract,
                      int out_by_query, int kout, uint64_t* oi, float* od, int32_t* on, int by_query,
                      uint64_t* rec_i, float* rec_d, int32_t* rec_n, int rec_cap) {
    const int64_t nslots = idx->hiwater;
    const int64_t ld = std::max<int64_t>(round_up(nslots, EBLK), EBLK);
    int64_t G = std::max<int64_t>(1, std::min<int64_t>(nlist, (2ll << 30) / (ld * 4)));
    HIPCHK(idx->rE.ensure((size_t)G * ld * sizeof(float)));
    HIPCHK(idx->rB.ensure((size_t)G * (ld / EBLK) * sizeof(float)));
    if (replay_scan_lds(k) > 160 * 1024)
        return set_err(WV_ERR_INVALID, "k=%d exceeds the exact replay heap limit of %d results", k,
                       (int)((160 * 1024 - 272) / 12));
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
        HIPCHK(launch_replay_scan(k, (unsigned)F, s, idx->rE.as<float>(), idx->rB.as<float>(), valid,
                                  Qn ? nslots : (int64_t)0, ld, d_qlist + g0, F, k, idx->id_base,
                                  in_n ? in_i + ioff * k : (const uint64_t*)nullptr,
                                  in_n ? in_d + ioff * k : (const float*)nullptr,
                                  in_n ? in_n + ioff : (const int32_t*)nullptr, extract, (int)(out_by_query || by_query),
                                  kout, oi + ooff * (raw ? k : kout), od + ooff * (raw ? k : kout), on + ooff, by_query,
                                  by_query, rec_n ? rec_i + g0 * rec_cap : (uint64_t*)nullptr,
                                  rec_n ? rec_d + g0 * rec_cap : (float*)nullptr, rec_n ? rec_n + g0 : (int32_t*)nullptr,
                                  rec_cap));
    }
    return WV_OK;
}

// prepare padded (and for cosine exactly normalised) query rows + norms
// (overwrites idx->qn: the block keys / shard phase of an earlier batch no longer apply)
int prepare_queries(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t nq_pad) {
    invalidate_batch(idx);
    HIPCHK(idx->qn.ensure((size_t)nq_pad * idx->dpad * sizeof(float)));
    HIPCHK(idx->qn2.ensure((size_t)nq_pad * sizeof(float)));
    float* Qn = idx->qn.as<float>();
    // the padding rows [nq, nq_pad) are zeroed by the same launch
    if (idx->metric == WV_METRIC_COSINE_DOT)
        k_normalize_rows<<<(unsigned)((nq_pad + 3) / 4), 256, 0, s>>>(d_qraw, nq, idx->dims, Qn, idx->dpad, nq_pad);
    else
        k_copy_pad_rows<<<(unsigned)((nq_pad * idx->dpad + 255) / 256), 256, 0, s>>>(d_qraw, nq, idx->dims, Qn,
                                                                                   idx->dpad, nq_pad);
    k_row_norm2<<<(unsigned)((nq_pad + 3) / 4), 256, 0, s>>>(Qn, nq_pad, idx->dpad, idx->qn2.as<float>());
    HIPCHK(hipGetLastError());
    return WV_OK;
}

// the block-key route (search_qs) serves this index and k
static bool qs_route(const wv_index* idx, int k) {
    return (idx->qs_planes || idx->q8_only) && !idx->has_nonfinite && (idx->kernel_opt == 0 || idx->kernel_opt == 7) &&
           !idx->force_replay && qs_R_flat(k) > 0 && idx->metric != WV_METRIC_HAMMING;
}

// Core batch search on device queries.  Outputs [nq][kout] device arrays.
// mode 0: kout = k, flagged queries resolved by replay; mode 1: kout = k+1,
// flags left for the caller.  n_valid = number of scan candidates.
static int search_core(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k, int mode,
                       const uint32_t* valid, int64_t n_valid, uint64_t* o_ids, float* o_d, int32_t* o_n,
                       int32_t* o_flags) {
    const int kout = mode == 1 ? k + 1 : k;
    idx->qs_keys_nq = 0;
    idx->stats.last_route = WV_ROUTE_NONE;
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
    if (qs_route(idx, k)) {
        idx->stats.queries += (uint64_t)nq;
        idx->stats.batches++;
        return search_qs(idx, s, nq, k, mode, valid, o_ids, o_d, o_n, o_flags);
    }
    if (idx->pqa_valid) return set_err(WV_ERR_UNSUPPORTED, "per-query allow lists: block-key route only");
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
        idx->stats.last_route = gemv ? WV_ROUTE_GEMV : WV_ROUTE_F32_SELECT;
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

// valid-slot bitmap for an allow list (present & allow), built on the device
// from the id list.  windowed: only the words of the allowed slot span
// [lo, hi) are written (flat/index.go:590-608 seeks to allow.Min() and stops
// past allow.Max()) and the caller scans only that span (ScanWindow); else the
// whole bitmap up to hiwater.  Returns the candidate count (one host sync)
// and the span.
static int build_valid(wv_index* idx, hipStream_t s, const uint64_t* allow, int64_t n_allow, int32_t allow_mode,
                       const uint32_t** valid_out, int64_t* n_valid, int64_t* lo_out = nullptr,
                       int64_t* hi_out = nullptr, bool windowed = false) {
    if (lo_out) { *lo_out = 0; *hi_out = idx->hiwater; }
    if (allow_mode == 0) {
        *valid_out = idx->present;
        *n_valid = idx->npresent;
        return WV_OK;
    }
    int64_t lo = INT64_MAX, hi = -1;
    for (int64_t i = 0; i < n_allow; i++) {
        if (allow[i] < idx->id_base) continue;
        const uint64_t sl = allow[i] - idx->id_base;
        if ((int64_t)sl >= idx->hiwater) continue;
        lo = std::min<int64_t>(lo, (int64_t)sl);
        hi = std::max<int64_t>(hi, (int64_t)sl + 1);
    }
    *valid_out = idx->present;
    *n_valid = 0;
    if (hi <= lo) return WV_OK;
    HIPCHK(idx->valid.ensure((size_t)std::max<int64_t>(idx->cap / 32, 1) * sizeof(uint32_t)));
    HIPCHK(idx->allowIds.ensure((size_t)n_allow * sizeof(uint64_t) + 8));
    HIPCHK(idx->allowCnt.ensure(sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(idx->allowIds.p, allow, (size_t)n_allow * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    // every word a kernel of the (windowed) scan reads: whole 256-row tiles
    // from the window start (lo rounded down) to the span end rounded up
    const int64_t w0 = windowed ? (lo / 256 * 256) >> 5 : 0;
    const int64_t w1 = round_up(windowed ? hi : idx->hiwater, 256) >> 5;
    HIPCHK(hipMemsetAsync(idx->valid.as<uint32_t>() + w0, 0, (size_t)(w1 - w0) * sizeof(uint32_t), s));
    HIPCHK(hipMemsetAsync(idx->allowCnt.p, 0, sizeof(uint32_t), s));
    k_allow_bits<<<(unsigned)((n_allow + 255) / 256), 256, 0, s>>>(idx->allowIds.as<uint64_t>(), n_allow, idx->id_base,
                                                                    idx->hiwater, idx->present,
                                                                    idx->valid.as<uint32_t>(), idx->allowCnt.as<uint32_t>());
    HIPCHK(hipGetLastError());
    uint32_t nv = 0;
    HIPCHK(hipMemcpyAsync(&nv, idx->allowCnt.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    *valid_out = idx->valid.as<uint32_t>();
    *n_valid = nv;
    if (lo_out) { *lo_out = lo; *hi_out = hi; }
    return WV_OK;
}

// The allow-list bitmap of one shard of a filtered multi-shard search
// (multi.hip): present & allow over the whole allocation (every word a kernel
// may read, zero where no allowed row is), in idx->valid; *n_valid = its
// population (one host sync).  The ids of other shards are skipped by range.
int shard_filter_bitmap(wv_index* idx, hipStream_t s, const uint64_t* allow, int64_t n_allow, const uint32_t** valid,
                        int64_t* n_valid) {
    const int64_t words = std::max<int64_t>(idx->cap / 32, 1);
    HIPCHK(idx->valid.ensure((size_t)words * sizeof(uint32_t)));
    HIPCHK(hipMemsetAsync(idx->valid.p, 0, (size_t)words * sizeof(uint32_t), s));
    *valid = idx->valid.as<uint32_t>();
    *n_valid = 0;
    if (n_allow <= 0 || idx->hiwater == 0) return WV_OK;
    HIPCHK(idx->allowIds.ensure((size_t)n_allow * sizeof(uint64_t) + 8));
    HIPCHK(idx->allowCnt.ensure(sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(idx->allowIds.p, allow, (size_t)n_allow * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(idx->allowCnt.p, 0, sizeof(uint32_t), s));
    k_allow_bits<<<(unsigned)((n_allow + 255) / 256), 256, 0, s>>>(idx->allowIds.as<uint64_t>(), n_allow, idx->id_base,
                                                                    idx->hiwater, idx->present,
                                                                    idx->valid.as<uint32_t>(), idx->allowCnt.as<uint32_t>());
    HIPCHK(hipGetLastError());
    uint32_t nv = 0;
    HIPCHK(hipMemcpyAsync(&nv, idx->allowCnt.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    *n_valid = nv;
    return WV_OK;
}

// A search over the slot span [lo, hi) of the store only: the stored-row
// arrays are offset to lo (a multiple of 256: whole tiles of the tiled planes)
// and the index reads as one of hi - lo slots with id_base + lo, so every
// kernel of the path scans only the span.  Exact fp32 and BQ indexes (their
// layouts are row- or 256-row-tile-major); restored on scope exit.
struct ScanWindow {
    wv_index* idx;
    int64_t lo;
    float* X; float* xnorm2; uint32_t* present; uint16_t* Xb; unsigned char* X8; float* sb8;
    uint64_t* codes; unsigned char* bq8; int64_t hiwater; uint64_t id_base;
    ScanWindow(wv_index* i, int64_t lo_, int64_t hi_) : idx(i), lo(lo_) {
        X = idx->X; xnorm2 = idx->xnorm2; present = idx->present; Xb = idx->Xb; X8 = idx->X8; sb8 = idx->sb8;
        codes = idx->codes; bq8 = idx->bq8; hiwater = idx->hiwater; id_base = idx->id_base;
        idx->hiwater = hi_ - lo;
        if (lo == 0) return;
        idx->X += lo * idx->dpad;
        idx->xnorm2 += lo;
        idx->present += lo / 32;
        if (idx->Xb) idx->Xb += lo * idx->dpb;
        if (idx->X8) { idx->X8 += lo * idx->dpb8; idx->sb8 += lo / 32; }
        if (idx->codes) idx->codes += lo;  // word-major, stride cap
        if (idx->bq8) idx->bq8 += lo * idx->dpb8b;
        idx->id_base += (uint64_t)lo;
    }
    ~ScanWindow() {
        idx->X = X; idx->xnorm2 = xnorm2; idx->present = present; idx->Xb = Xb; idx->X8 = X8; idx->sb8 = sb8;
        idx->codes = codes; idx->bq8 = bq8; idx->hiwater = hiwater; idx->id_base = id_base;
    }
};

static bool window_ok(const wv_index* idx) {
    return idx->compression == WV_COMPRESSION_NONE || idx->compression == WV_COMPRESSION_BQ;
}

// The allowed rows (slots ascending = the reference cursor's id order) as a
// sub-index: fp32 rows, norms and bf16 plane rows gathered, the int8 plane
// re-quantised per sub-index block; the parent's residual maxima bound the
// gathered bf16 rows.  Same metric, variant and exact-path options.
static int subindex_build(wv_index* idx, hipStream_t s, const std::vector<uint32_t>& slots) {
    const int64_t n = (int64_t)slots.size();
    if (!idx->sub) {
        wv_config c{};
        c.metric = idx->metric;
        c.dims = idx->dims;
        c.compression = WV_COMPRESSION_NONE;
        c.rescore_limit = -1;
        c.device = idx->device;
        c.variant = idx->variant;
        c.id_base = 0;
        c.root_path = idx->root_path.c_str();
        int rc = wv_index_create(&c, &idx->sub);
        if (rc) return rc;
    }
    wv_index* sb = idx->sub;
    sb->use_qs = idx->use_qs;
    set_dims(sb, idx->dims);
    sb->kernel_opt = idx->kernel_opt; sb->q8_opt = idx->q8_opt; sb->q8_R = idx->q8_R; sb->q8_filter = idx->q8_filter;
    sb->q8_stag = idx->q8_stag; sb->q8_shape = idx->q8_shape; sb->q8_pf = idx->q8_pf; sb->exact_filter = idx->exact_filter; sb->exact_bm = idx->exact_bm; sb->q8_bm = idx->q8_bm; sb->q8_gemv = idx->q8_gemv; sb->q8_live = idx->q8_live; sb->q8_prio = idx->q8_prio; sb->sel_split_max = idx->sel_split_max; sb->q8_bm_min = idx->q8_bm_min;
    sb->exact_cap = idx->exact_cap; sb->replay_par = idx->replay_par; sb->rp_few = idx->rp_few; sb->margin = idx->margin;
    sb->gemv_max = idx->gemv_max; sb->gemv_wg = idx->gemv_wg; sb->exact_multi = idx->exact_multi;
    sb->force_replay = idx->force_replay; sb->qs_force_flag = idx->qs_force_flag; sb->timing = idx->timing;
    sb->hiwater = 0;
    sb->npresent = 0;
    int rc = ensure_capacity(sb, round_up(std::max<int64_t>(n, 1), 256));
    if (rc) return rc;
    HIPCHK(idx->subSlots.ensure((size_t)n * sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(idx->subSlots.p, slots.data(), (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    const int64_t n_pad = round_up(n, 256);
    {
        const int64_t per = idx->dpad / 4 + (sb->qs_planes ? idx->dpb / 8 : 0) + 1;
        const int64_t nt = n_pad * per;
        k_gather_rows<<<(unsigned)((nt + 255) / 256), 256, 0, s>>>(idx->X, idx->xnorm2, idx->dpad,
                                                                    sb->qs_planes ? idx->Xb : nullptr, idx->dpb,
                                                                    idx->subSlots.as<uint32_t>(), n, n_pad, sb->X,
                                                                    sb->xnorm2, sb->Xb);
        HIPCHK(hipGetLastError());
    }
    std::vector<uint32_t> bits((size_t)(sb->cap / 32), 0);
    for (int64_t i = 0; i < n; i++) bits[(size_t)(i >> 5)] |= 1u << (i & 31);
    HIPCHK(hipMemcpyAsync(sb->present, bits.data(), bits.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(sb->d_maxn2, idx->d_maxn2, sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(sb->qsmax, idx->qsmax, 4 * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    if (sb->q8_planes) {
        HIPCHK(hipMemsetAsync(sb->qmax8, 0, 4 * sizeof(uint32_t), s));
        k_block_q8<<<(unsigned)(n_pad / 32), 256, 0, s>>>(sb->X, sb->dpad, sb->dims, sb->dpb8, nullptr, 0, sb->X8, sb->sb8,
                                                          sb->qmax8);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(s));  // the host bitmap and slot list are read by the copies
    sb->hiwater = n;
    sb->npresent = n;
    sb->has_nonfinite = idx->has_nonfinite;
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
    int64_t n_valid = 0, lo = 0, hi = 0;
    if (allow_mode == 1 && idx->compression == WV_COMPRESSION_NONE && idx->qs_planes && n_allow <= idx->gather_max &&
        idx->dims != 0 && d == idx->dims) {
        // a sparse allow list: its rows as a sub-index (cost follows the list, not its span)
        std::vector<uint32_t> slots;
        slots.reserve((size_t)n_allow);
        for (int64_t i = 0; i < n_allow; i++) {
            if (allow_ids[i] < idx->id_base) continue;
            const uint64_t sl = allow_ids[i] - idx->id_base;
            if ((int64_t)sl < idx->hiwater && idx->h_present[sl]) slots.push_back((uint32_t)sl);
        }
        std::sort(slots.begin(), slots.end());
        slots.erase(std::unique(slots.begin(), slots.end()), slots.end());
        if (slots.empty()) {
            for (int64_t q = 0; q < nq; q++) out_counts[q] = 0;
            return WV_OK;
        }
        const int64_t span = (int64_t)slots.back() + 1 - (int64_t)slots.front() / 256 * 256;
        if ((int64_t)slots.size() * 8 <= span) {
            int rc = subindex_build(idx, s, slots);
            if (rc) return rc;
            const int kk = std::max(k, 1);
            HIPCHK(idx->qraw.ensure((size_t)nq * d * sizeof(float)));
            HIPCHK(idx->oIds.ensure((size_t)nq * kk * sizeof(uint64_t)));
            HIPCHK(idx->oD.ensure((size_t)nq * kk * sizeof(float)));
            HIPCHK(idx->oN.ensure((size_t)nq * sizeof(int32_t)));
            HIPCHK(hipMemcpyAsync(idx->qraw.p, queries, (size_t)nq * d * sizeof(float), hipMemcpyHostToDevice, s));
            wv_index* sb = idx->sub;
            rc = search_core(sb, s, idx->qraw.as<float>(), nq, d, k, 0, sb->present, sb->npresent,
                             idx->oIds.as<uint64_t>(), idx->oD.as<float>(), idx->oN.as<int32_t>(), nullptr);
            if (rc) return rc;
            if (k > 0)
                k_remap_ids<<<(unsigned)((nq * k + 255) / 256), 256, 0, s>>>(idx->oIds.as<uint64_t>(),
                                                                             idx->oN.as<int32_t>(), nq, k,
                                                                             idx->subSlots.as<uint32_t>(), idx->id_base);
            HIPCHK(hipGetLastError());
            idx->stats.last_route = sb->stats.last_route;
            idx->stats.last_scan_rows = (uint64_t)sb->hiwater;
            idx->stats.queries += (uint64_t)nq;
            idx->stats.batches++;
            HIPCHK(hipMemcpyAsync(out_ids, idx->oIds.p, (size_t)nq * k * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(out_dists, idx->oD.p, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(out_counts, idx->oN.p, (size_t)nq * sizeof(int32_t), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            return WV_OK;
        }
    }
    const bool windowed = allow_mode == 1 && idx->scan_window && window_ok(idx);
    int rc = build_valid(idx, s, allow_ids, n_allow, allow_mode, &valid, &n_valid, &lo, &hi, windowed);
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
    {
        // an allow list scans only its slot span (rounded down to a 256-row tile)
        const int64_t lo_t = windowed ? lo / 256 * 256 : 0;
        ScanWindow win(idx, lo_t, windowed ? hi : idx->hiwater);
        idx->stats.last_scan_rows = (uint64_t)idx->hiwater;
        rc = search_core(idx, s, idx->qraw.as<float>(), nq, d, k, 0, valid + lo_t / 32, n_valid,
                         idx->oIds.as<uint64_t>(), idx->oD.as<float>(), idx->oN.as<int32_t>(), nullptr);
    }
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(out_ids, idx->oIds.p, (size_t)nq * k * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out_dists, idx->oD.p, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out_counts, idx->oN.p, (size_t)nq * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

// Per-query allow lists in one call: query q is searched under its own list
// allow_ids[allow_offsets[q] .. allow_offsets[q+1]) when allow_modes[q] == 1,
// unfiltered when 0 -- the results of wv_index_search_by_vector_batch called
// per query (Weaviate's callers each bring their filter: shard_read.go:415-424
// -> flat/index.go:423-448 with its own helpers.AllowList).  On the block-key
// route the batch shares one launch: the keys run over the union of the
// queries' rows, each query's exact pass and replay over its own bitmap
// (search_qs).  Other routes: the queries grouped by identical list, one batch
// call per group.
static int multi_allow_grouped(wv_index* idx, const float* queries, int64_t nq, int64_t d, int32_t k,
                               const uint64_t* allow_ids, const int64_t* off, const int32_t* modes, uint64_t* out_ids,
                               float* out_dists, int32_t* out_counts) {
    std::map<std::pair<int, std::string>, std::vector<int64_t>> groups;
    for (int64_t q = 0; q < nq; q++) {
        std::string key;
        if (modes[q] == 1)
            key.assign(reinterpret_cast<const char*>(allow_ids + off[q]), (size_t)(off[q + 1] - off[q]) * sizeof(uint64_t));
        groups[{modes[q], key}].push_back(q);
    }
    const int64_t kk = std::max<int32_t>(k, 0), dd = std::max<int64_t>(d, 0);
    std::vector<float> qb;
    std::vector<uint64_t> ids;
    std::vector<float> ds;
    std::vector<int32_t> cnt;
    for (auto& g : groups) {
        const std::vector<int64_t>& qs = g.second;
        const int64_t n = (int64_t)qs.size();
        qb.resize((size_t)(n * dd) + 1);
        ids.resize((size_t)(n * kk) + 1);
        ds.resize((size_t)(n * kk) + 1);
        cnt.resize((size_t)n);
        for (int64_t i = 0; i < n; i++) memcpy(&qb[(size_t)(i * dd)], queries + qs[i] * dd, (size_t)dd * sizeof(float));
        const int64_t q0 = qs[0];
        int rc = wv_index_search_by_vector_batch(idx, qb.data(), n, d, k, modes[q0] ? allow_ids + off[q0] : nullptr,
                                                 modes[q0] ? off[q0 + 1] - off[q0] : 0, modes[q0], ids.data(),
                                                 ds.data(), cnt.data());
        if (rc) return rc;
        for (int64_t i = 0; i < n; i++) {
            out_counts[qs[i]] = cnt[i];
            memcpy(out_ids + qs[i] * kk, &ids[(size_t)(i * kk)], (size_t)cnt[i] * sizeof(uint64_t));
            memcpy(out_dists + qs[i] * kk, &ds[(size_t)(i * kk)], (size_t)cnt[i] * sizeof(float));
        }
    }
    return WV_OK;
}

// the select's threshold depth per query (k_blk_select mq): a block key is
// the minimum over the union's rows, this query's own with probability ~ its
// share rho of the union, so ~ (k+1) / rho blocks hold its k+1 nearest; twice
// that (unclamped; unlisted queries: k+1)
static void pqa_depths(const wv_index* idx, int64_t nq, int32_t k, const int64_t* off, const int32_t* modes,
                       std::vector<double>& m) {
    int64_t tot = 0;
    for (int64_t q = 0; q < nq; q++) tot += modes[q] ? off[q + 1] - off[q] : idx->npresent;
    const double U = (double)std::max<int64_t>(1, std::min<int64_t>(tot, idx->npresent));
    m.assign((size_t)nq, (double)(k + 1));
    for (int64_t q = 0; q < nq; q++)
        if (modes[q]) m[(size_t)q] = 2.0 * (k + 1) * std::max(1.0, U / (double)std::max<int64_t>(1, off[q + 1] - off[q]));
}

// the shared block-key launch of a multi-allow batch once the per-query
// bitmaps (bits, vq words each, ANDed with present) are on the device: union,
// search_core, results to the host; left = the queries the launch flagged
// (searched alone by the caller).  Called with idx->mu held.
static int pqa_run(wv_index* idx, hipStream_t s, const float* queries, int64_t nq, int64_t d, int32_t k, int64_t vq,
                   uint32_t* bits, uint64_t* out_ids, float* out_dists, int32_t* out_counts,
                   std::vector<int64_t>& left) {
    uint32_t* uni = idx->pqaUnion.as<uint32_t>();
    HIPCHK(hipMemsetAsync(uni, 0, (size_t)std::max<int64_t>(idx->cap / 32, vq) * sizeof(uint32_t), s));
    k_pqa_union<<<(unsigned)((vq + 255) / 256), 256, 0, s>>>(bits, vq, nq, uni);
    HIPCHK(hipGetLastError());
    HIPCHK(idx->qraw.ensure((size_t)nq * d * sizeof(float)));
    HIPCHK(idx->oIds.ensure((size_t)nq * k * sizeof(uint64_t)));
    HIPCHK(idx->oD.ensure((size_t)nq * k * sizeof(float)));
    HIPCHK(idx->oN.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(hipMemcpyAsync(idx->qraw.p, queries, (size_t)nq * d * sizeof(float), hipMemcpyHostToDevice, s));
    idx->stats.last_scan_rows = (uint64_t)idx->hiwater;
    idx->pqa_valid = bits;
    idx->pqa_vq = vq;
    idx->pqa_m = idx->pqaM.as<int32_t>();
    // the queries the shared launch leaves unresolved (flags) are searched
    // alone afterwards (a sparse list's own gathered sub-index or window)
    // instead of by the one-wave replay inside the launch, which walks every
    // block key of the union for one query (35 ms at 1M rows, 2 % lists)
    HIPCHK(idx->oF.ensure((size_t)nq * sizeof(int32_t)));
    int32_t* dflags = idx->pqa_alone ? idx->oF.as<int32_t>() : nullptr;
    int rc = search_core(idx, s, idx->qraw.as<float>(), nq, d, k, 0, uni, idx->npresent, idx->oIds.as<uint64_t>(),
                         idx->oD.as<float>(), idx->oN.as<int32_t>(), dflags);
    idx->pqa_valid = nullptr;
    idx->pqa_vq = 0;
    idx->pqa_m = nullptr;
    if (rc) return rc;
    std::vector<int32_t> hf(dflags ? (size_t)nq : 0);
    HIPCHK(hipMemcpyAsync(out_ids, idx->oIds.p, (size_t)nq * k * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out_dists, idx->oD.p, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out_counts, idx->oN.p, (size_t)nq * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (dflags) HIPCHK(hipMemcpyAsync(hf.data(), dflags, (size_t)nq * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (int64_t q = 0; q < (int64_t)hf.size(); q++)
        if (hf[(size_t)q]) left.push_back(q);
    idx->stats.replayed_queries += (uint64_t)left.size();
    return WV_OK;
}


static thread_local bool t_pqa_nosplit = false;

extern "C" int wv_index_search_by_vector_batch_multi_allow(wv_index* idx, const float* queries, int64_t nq, int64_t d,
                                                           int32_t k, const uint64_t* allow_ids,
                                                           const int64_t* allow_offsets, const int32_t* allow_modes,
                                                           uint64_t* out_ids, float* out_dists, int32_t* out_counts);

// the queries qs of a multi-allow batch as their own batch -- grouped by list
// (shared == false: one-query-list calls) or shared (the one-launch path, no
// further split) -- results scattered back into the batch's outputs
static int multi_allow_subset(wv_index* idx, const float* queries, int64_t d, int32_t k, const uint64_t* allow_ids,
                              const int64_t* allow_offsets, const int32_t* allow_modes, const std::vector<int64_t>& qs,
                              bool shared, uint64_t* out_ids, float* out_dists, int32_t* out_counts) {
    const int64_t kk = std::max<int32_t>(k, 0);
    const int64_t n = (int64_t)qs.size();
    std::vector<float> qb((size_t)(n * d) + 1);
    std::vector<int64_t> off((size_t)n + 1, 0);
    std::vector<int32_t> modes((size_t)n);
    std::vector<uint64_t> aid;
    for (int64_t i = 0; i < n; i++) {
        const int64_t q = qs[(size_t)i];
        memcpy(&qb[(size_t)(i * d)], queries + q * d, (size_t)d * sizeof(float));
        modes[(size_t)i] = allow_modes[q];
        if (allow_modes[q]) aid.insert(aid.end(), allow_ids + allow_offsets[q], allow_ids + allow_offsets[q + 1]);
        off[(size_t)i + 1] = (int64_t)aid.size();
    }
    aid.push_back(0);  // a valid pointer when every list is empty
    std::vector<uint64_t> oi((size_t)(n * kk) + 1);
    std::vector<float> od((size_t)(n * kk) + 1);
    std::vector<int32_t> oc((size_t)n);
    int rc;
    if (!shared) {
        rc = multi_allow_grouped(idx, qb.data(), n, d, k, aid.data(), off.data(), modes.data(), oi.data(), od.data(),
                                 oc.data());
    } else {
        t_pqa_nosplit = true;
        rc = wv_index_search_by_vector_batch_multi_allow(idx, qb.data(), n, d, k, aid.data(), off.data(), modes.data(),
                                                         oi.data(), od.data(), oc.data());
        t_pqa_nosplit = false;
    }
    if (rc) return rc;
    for (int64_t i = 0; i < n; i++) {
        const int64_t q = qs[(size_t)i];
        out_counts[q] = oc[(size_t)i];
        memcpy(out_ids + q * kk, &oi[(size_t)(i * kk)], (size_t)oc[(size_t)i] * sizeof(uint64_t));
        memcpy(out_dists + q * kk, &od[(size_t)(i * kk)], (size_t)oc[(size_t)i] * sizeof(float));
    }
    return WV_OK;
}

extern "C" int wv_index_search_by_vector_batch_multi_allow(wv_index* idx, const float* queries, int64_t nq, int64_t d,
                                                           int32_t k, const uint64_t* allow_ids,
                                                           const int64_t* allow_offsets, const int32_t* allow_modes,
                                                           uint64_t* out_ids, float* out_dists, int32_t* out_counts) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (nq < 0) return set_err(WV_ERR_INVALID, "negative batch");
    if (nq == 0) return WV_OK;
    if (!allow_offsets || !allow_modes || !out_counts || (d > 0 && !queries))
        return set_err(WV_ERR_INVALID, "nil argument");
    for (int64_t q = 0; q < nq; q++) {
        if (allow_modes[q] != 0 && allow_modes[q] != 1) return set_err(WV_ERR_INVALID, "allow mode %d", allow_modes[q]);
        if (allow_offsets[q] < 0 || allow_offsets[q + 1] < allow_offsets[q])
            return set_err(WV_ERR_INVALID, "allow offsets not ascending at %lld", (long long)q);
        if (allow_modes[q] == 1 && allow_offsets[q + 1] > allow_offsets[q] && !allow_ids)
            return set_err(WV_ERR_INVALID, "nil allow ids");
    }
    std::unique_lock<std::mutex> g(idx->mu);
    const int64_t vq = round_up(std::max<int64_t>(idx->hiwater, 1), 256) / 32;  // words per query bitmap
    const int64_t qmax = std::max<int64_t>(1, (idx->pqa_budget_mb << 20) / (vq * (int64_t)sizeof(uint32_t)));
    const bool fast = idx->pqa && nq > 1 && idx->compression == WV_COMPRESSION_NONE && !idx->rq_bits &&
                      idx->dims != 0 && d == idx->dims && k > 0 && idx->npresent > 0 && qs_route(idx, k);
    if (!fast) {
        g.unlock();
        return multi_allow_grouped(idx, queries, nq, d, k, allow_ids, allow_offsets, allow_modes, out_ids, out_dists,
                                   out_counts);
    }
    std::vector<double> md;
    pqa_depths(idx, nq, k, allow_offsets, allow_modes, md);
    if (!t_pqa_nosplit && !pqa_keys_route(idx)) {  // (per-query keys serve sparse lists in the launch)
        // lists too sparse for the union's keys (deeper than the 960-block
        // lists) would end in the one-wave replay, a walk over every block
        // key: a few of them go as their own searches instead (an allow list
        // that sparse takes the gathered sub-index route)
        std::vector<int64_t> sp, dn;
        for (int64_t q = 0; q < nq; q++) (md[(size_t)q] > 960.0 ? sp : dn).push_back(q);
        if (!sp.empty() && (int64_t)sp.size() <= idx->pqa_split_max && !dn.empty()) {
            g.unlock();
            int rc = multi_allow_subset(idx, queries, d, k, allow_ids, allow_offsets, allow_modes, sp, false, out_ids,
                                        out_dists, out_counts);
            if (rc) return rc;
            return multi_allow_subset(idx, queries, d, k, allow_ids, allow_offsets, allow_modes, dn, true, out_ids,
                                      out_dists, out_counts);
        }
    }
    if (nq > qmax) {  // bitmaps past the budget: consecutive sub-batches
        g.unlock();
        for (int64_t q0 = 0; q0 < nq; q0 += qmax) {
            const int64_t n = std::min(qmax, nq - q0);
            int rc = wv_index_search_by_vector_batch_multi_allow(idx, queries + q0 * d, n, d, k, allow_ids,
                                                                 allow_offsets + q0, allow_modes + q0,
                                                                 out_ids + q0 * k, out_dists + q0 * k, out_counts + q0);
            if (rc) return rc;
        }
        return WV_OK;
    }
    HIPCHK(hipSetDevice(idx->device));
    hipStream_t s = idx->stream;
    // the unlisted queries take the present bitmap; the ids of all lists go
    // over as given (one copy), their queries found on the device
    std::vector<int32_t> q0list;
    for (int64_t q = 0; q < nq; q++)
        if (allow_modes[q] == 0) q0list.push_back((int32_t)q);
    const int64_t nids = allow_offsets[nq] - allow_offsets[0];
    HIPCHK(idx->pqaBits.ensure((size_t)(nq * vq) * sizeof(uint32_t)));
    HIPCHK(idx->pqaUnion.ensure((size_t)std::max<int64_t>(idx->cap / 32, vq) * sizeof(uint32_t)));
    // pqaQ: [nq + 1] offsets (int64), [nq] modes, [n0] unlisted queries
    HIPCHK(idx->pqaQ.ensure((size_t)(nq + 1) * sizeof(int64_t) + (size_t)(2 * nq + 2) * sizeof(int32_t)));
    HIPCHK(idx->pqaIds.ensure((size_t)(nids + 1) * sizeof(uint64_t)));
    std::vector<int32_t> hm((size_t)nq);
    for (int64_t q = 0; q < nq; q++) hm[(size_t)q] = (int32_t)std::min(960.0, std::ceil(md[(size_t)q]));
    // 448-block lists, 960 when a query wants more (k_blk_exact<16>)
    idx->pqa_R = *std::max_element(hm.begin(), hm.end()) > 448 ? 16 : 8;
    HIPCHK(idx->pqaM.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(hipMemcpyAsync(idx->pqaM.p, hm.data(), (size_t)nq * sizeof(int32_t), hipMemcpyHostToDevice, s));
    int64_t* d_off = idx->pqaQ.as<int64_t>();
    int32_t* d_modes = reinterpret_cast<int32_t*>(d_off + nq + 1);
    int32_t* d_q0 = d_modes + nq + 1;
    uint32_t* bits = idx->pqaBits.as<uint32_t>();
    HIPCHK(hipMemsetAsync(bits, 0, (size_t)(nq * vq) * sizeof(uint32_t), s));
    HIPCHK(hipMemcpyAsync(d_off, allow_offsets, (size_t)(nq + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_modes, allow_modes, (size_t)nq * sizeof(int32_t), hipMemcpyHostToDevice, s));
    if (!q0list.empty()) {
        HIPCHK(hipMemcpyAsync(d_q0, q0list.data(), q0list.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
        const int64_t n = (int64_t)q0list.size() * vq;
        k_pqa_present<<<(unsigned)std::min<int64_t>((n + 255) / 256, 4096), 256, 0, s>>>(
            idx->present, vq, d_q0, (int64_t)q0list.size(), bits);
        HIPCHK(hipGetLastError());
    }
    if (nids > 0) {
        HIPCHK(hipMemcpyAsync(idx->pqaIds.p, allow_ids + allow_offsets[0], (size_t)nids * sizeof(uint64_t),
                              hipMemcpyHostToDevice, s));
        k_pqa_bits<<<(unsigned)((nids + 255) / 256), 256, 0, s>>>(idx->pqaIds.as<uint64_t>(), d_off, d_modes, nq,
                                                                  idx->id_base, idx->hiwater, idx->present, vq, bits);
        HIPCHK(hipGetLastError());
    }
    std::vector<int64_t> left;
    int rc = pqa_run(idx, s, queries, nq, d, k, vq, bits, out_ids, out_dists, out_counts, left);
    if (rc || left.empty()) return rc;
    g.unlock();
    return multi_allow_subset(idx, queries, d, k, allow_ids, allow_offsets, allow_modes, left, false, out_ids, out_dists,
                              out_counts);
}

// bitmap allow lists -> id lists (absolute doc ids), for the paths that take lists
static void bits_to_lists(const uint32_t* bits, int64_t words, const int32_t* modes, int64_t nq,
                          std::vector<uint64_t>& ids, std::vector<int64_t>& off, const std::vector<char>* want) {
    ids.clear();
    off.assign((size_t)nq + 1, 0);
    for (int64_t q = 0; q < nq; q++) {
        if (modes[q] && (!want || (*want)[(size_t)q]))
            for (int64_t w = 0; w < words; w++)
                for (uint32_t v = bits[q * words + w]; v; v &= v - 1)
                    ids.push_back((uint64_t)(w * 32 + __builtin_ctz(v)));
        off[(size_t)q + 1] = (int64_t)ids.size();
    }
    ids.push_back(0);
}

// The shared multi-allow launch from per-query bitmaps, whatever their host
// form: off = the lists' size prefix sums (the select depths), fill writes the
// per-query device bitmaps (vq words each, ANDed with present), lists gives
// the same lists as ids (the paths that take id lists: a batch the shared
// launch does not serve, a split of too-sparse lists, the flagged queries).
// Called with g holding idx->mu; returns with it released or held.
typedef std::function<int(hipStream_t, int64_t, uint32_t*, const int32_t*)> PqaFill;
typedef std::function<void(std::vector<uint64_t>&, std::vector<int64_t>&, const std::vector<char>*)> PqaLists;
static int pqa_bitmap_core(wv_index* idx, std::unique_lock<std::mutex>& g, const float* queries, int64_t nq, int64_t d,
                           int32_t k, const int32_t* allow_modes, const std::vector<int64_t>& off, const PqaFill& fill,
                           const PqaLists& lists, uint64_t* out_ids, float* out_dists, int32_t* out_counts) {
    auto by_lists = [&](const std::vector<int64_t>* qs) -> int {
        g.unlock();
        std::vector<uint64_t> ids;
        std::vector<int64_t> lo;
        std::vector<char> want;  // the flagged queries' lists only
        if (qs) {
            want.assign((size_t)nq, 0);
            for (int64_t q : *qs) want[(size_t)q] = 1;
        }
        lists(ids, lo, qs ? &want : nullptr);
        if (!qs)
            return wv_index_search_by_vector_batch_multi_allow(idx, queries, nq, d, k, ids.data(), lo.data(),
                                                               allow_modes, out_ids, out_dists, out_counts);
        return multi_allow_subset(idx, queries, d, k, ids.data(), lo.data(), allow_modes, *qs, false, out_ids, out_dists,
                                  out_counts);
    };
    const int64_t vq = round_up(std::max<int64_t>(idx->hiwater, 1), 256) / 32;
    const int64_t qmax = std::max<int64_t>(1, (idx->pqa_budget_mb << 20) / (vq * (int64_t)sizeof(uint32_t) * 2));
    const bool fast = idx->pqa && nq > 1 && idx->compression == WV_COMPRESSION_NONE && !idx->rq_bits &&
                      idx->dims != 0 && d == idx->dims && k > 0 && idx->npresent > 0 && qs_route(idx, k) && nq <= qmax;
    std::vector<double> md;
    if (fast) pqa_depths(idx, nq, k, off.data(), allow_modes, md);
    bool split = false;
    if (fast && !pqa_keys_route(idx)) {  // the id-list call's split of too-sparse lists (see there)
        int64_t nsp = 0;
        for (int64_t q = 0; q < nq; q++) nsp += md[(size_t)q] > 960.0;
        split = nsp > 0 && nsp <= idx->pqa_split_max && nsp < nq;
    }
    if (!fast || split) return by_lists(nullptr);
    HIPCHK(hipSetDevice(idx->device));
    hipStream_t s = idx->stream;
    std::vector<int32_t> hm((size_t)nq);
    for (int64_t q = 0; q < nq; q++) hm[(size_t)q] = (int32_t)std::min(960.0, std::ceil(md[(size_t)q]));
    idx->pqa_R = *std::max_element(hm.begin(), hm.end()) > 448 ? 16 : 8;
    HIPCHK(idx->pqaM.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(hipMemcpyAsync(idx->pqaM.p, hm.data(), (size_t)nq * sizeof(int32_t), hipMemcpyHostToDevice, s));
    HIPCHK(idx->pqaBits.ensure((size_t)(nq * vq) * sizeof(uint32_t)));
    HIPCHK(idx->pqaUnion.ensure((size_t)std::max<int64_t>(idx->cap / 32, vq) * sizeof(uint32_t)));
    HIPCHK(idx->pqaQ.ensure((size_t)(nq + 1) * sizeof(int32_t)));
    int32_t* d_modes = idx->pqaQ.as<int32_t>();
    HIPCHK(hipMemcpyAsync(d_modes, allow_modes, (size_t)nq * sizeof(int32_t), hipMemcpyHostToDevice, s));
    uint32_t* bits = idx->pqaBits.as<uint32_t>();
    int rc = fill(s, vq, bits, d_modes);
    if (rc) return rc;
    std::vector<int64_t> left;
    rc = pqa_run(idx, s, queries, nq, d, k, vq, bits, out_ids, out_dists, out_counts, left);
    if (rc || left.empty()) return rc;
    return by_lists(&left);
}

extern "C" int wv_index_search_by_vector_batch_multi_allow_bitmap(wv_index* idx, const float* queries, int64_t nq,
                                                                  int64_t d, int32_t k, const uint32_t* allow_bits,
                                                                  int64_t words, const int32_t* allow_modes,
                                                                  uint64_t* out_ids, float* out_dists,
                                                                  int32_t* out_counts) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (nq < 0) return set_err(WV_ERR_INVALID, "negative batch");
    if (nq == 0) return WV_OK;
    if (words < 0) return set_err(WV_ERR_INVALID, "negative bitmap words");
    if (!allow_modes || !out_counts || (d > 0 && !queries)) return set_err(WV_ERR_INVALID, "nil argument");
    bool listed = false;
    for (int64_t q = 0; q < nq; q++) {
        if (allow_modes[q] != 0 && allow_modes[q] != 1) return set_err(WV_ERR_INVALID, "allow mode %d", allow_modes[q]);
        listed |= allow_modes[q] == 1;
    }
    if (listed && words > 0 && !allow_bits) return set_err(WV_ERR_INVALID, "nil allow bitmap");
    // list sizes (the select depths) from the bitmaps
    std::vector<int64_t> off((size_t)nq + 1, 0);
    for (int64_t q = 0; q < nq; q++) {
        int64_t c = 0;
        if (allow_modes[q])
            for (int64_t w = 0; w < words; w++) c += __builtin_popcount(allow_bits[q * words + w]);
        off[(size_t)q + 1] = off[(size_t)q] + c;
    }
    std::unique_lock<std::mutex> g(idx->mu);
    // the callers' words from doc id id_base & ~31 on, one strided copy (pqaIds
    // holds them), then the shift by id_base & 31 on the device
    PqaFill fill = [&](hipStream_t s, int64_t vq, uint32_t* bits, const int32_t* d_modes) -> int {
        const int64_t sw = vq + 1;  // the slot window plus the shift's spill word
        const int64_t b0 = (int64_t)(idx->id_base >> 5);
        const int64_t avail = std::max<int64_t>(0, std::min<int64_t>(sw, words - b0));
        HIPCHK(idx->pqaIds.ensure((size_t)(nq * sw) * sizeof(uint32_t) + 8));
        uint32_t* raw = reinterpret_cast<uint32_t*>(idx->pqaIds.p);
        if (avail > 0)
            HIPCHK(hipMemcpy2DAsync(raw, (size_t)sw * sizeof(uint32_t), allow_bits + b0, (size_t)words * sizeof(uint32_t),
                                    (size_t)avail * sizeof(uint32_t), (size_t)nq, hipMemcpyHostToDevice, s));
        k_pqa_from_bits<<<(unsigned)std::min<int64_t>((nq * vq + 255) / 256, 8192), 256, 0, s>>>(
            raw, sw, avail, d_modes, nq, (int)(idx->id_base & 31), idx->present, vq, bits);
        HIPCHK(hipGetLastError());
        return WV_OK;
    };
    PqaLists lists = [&](std::vector<uint64_t>& ids, std::vector<int64_t>& lo, const std::vector<char>* want) {
        bits_to_lists(allow_bits, words, allow_modes, nq, ids, lo, want);
    };
    return pqa_bitmap_core(idx, g, queries, nq, d, k, allow_modes, off, fill, lists, out_ids, out_dists, out_counts);
}

// The micro-batcher's filtered requests as slot bitmaps (batcher.hip): row q
// = rows[q].words words of bits over slots (doc id - id_base) in page-locked
// host memory the kernel reads in place (rows[q].dev); list size rows[q].n.
static int batch_search_slot_bitmaps(wv_index* idx, const float* queries, int64_t nq, int64_t d, int32_t k,
                                     const wv_batch_row* rows, uint64_t* out_ids, float* out_dists,
                                     int32_t* out_counts) {
    std::vector<int32_t> modes((size_t)nq, 1);
    std::vector<int64_t> off((size_t)nq + 1, 0);
    for (int64_t q = 0; q < nq; q++) off[(size_t)q + 1] = off[(size_t)q] + std::max<int64_t>(rows[q].n, 0);

    std::unique_lock<std::mutex> g(idx->mu);
    PqaFill fill = [&](hipStream_t s, int64_t vq, uint32_t* bits, const int32_t* d_modes) -> int {
        HIPCHK(idx->pqaIds.ensure((size_t)nq * sizeof(wv_batch_row)));
        HIPCHK(hipMemcpyAsync(idx->pqaIds.p, rows, (size_t)nq * sizeof(wv_batch_row), hipMemcpyHostToDevice, s));
        k_pqa_from_rows<<<(unsigned)std::min<int64_t>((nq * vq + 255) / 256, 8192), 256, 0, s>>>(
            reinterpret_cast<const wv_batch_row*>(idx->pqaIds.p), d_modes, nq, idx->present, vq, bits);
        HIPCHK(hipGetLastError());
        return WV_OK;
    };
    PqaLists lists = [&](std::vector<uint64_t>& ids, std::vector<int64_t>& lo, const std::vector<char>* want) {
        ids.clear();
        lo.assign((size_t)nq + 1, 0);
        for (int64_t q = 0; q < nq; q++) {
            if (!want || (*want)[(size_t)q])
                for (int64_t w = 0; w < rows[q].words; w++)
                    for (uint32_t v = rows[q].host[w]; v; v &= v - 1)
                        ids.push_back(idx->id_base + (uint64_t)(w * 32 + __builtin_ctz(v)));
            lo[(size_t)q + 1] = (int64_t)ids.size();
        }
        ids.push_back(0);
    };
    return pqa_bitmap_core(idx, g, queries, nq, d, k, modes.data(), off, fill, lists, out_ids, out_dists, out_counts);
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
    // a repeated identical call on a caller stream replays the hipGraph captured
    // on its second occurrence (uncompressed corpus; timing events become event-record nodes)
    const bool graphable = idx->graph_opt && stream && idx->compression == WV_COMPRESSION_NONE &&
                           !idx->rq_bits && nq > 0;
    if (graphable) {
        wv_index::GraphKey key;
        key.q = d_queries; key.nq = nq; key.d = d; key.k = k; key.mode = mode; key.ids = d_ids; key.dd = d_dists;
        key.cnt = d_counts; key.flags = mode == 1 ? d_flags : nullptr; key.stream = stream; key.gen = idx->mut_gen;
        if (idx->g_exec && key == idx->g_key) {
            HIPCHK(hipGraphLaunch(idx->g_exec, s));
            idx->timed = idx->g_timed;
            idx->timed_total = idx->g_timed_total;
            idx->stats.queries += idx->g_dq;
            idx->stats.batches += idx->g_db;
            idx->stats.mfma_launches += idx->g_dm;
            return WV_OK;
        }
        if (key == idx->g_seen && !idx->g_failed) {
            if (idx->g_exec) { hipGraphExecDestroy(idx->g_exec); idx->g_exec = nullptr; }
            if (idx->g_graph) { hipGraphDestroy(idx->g_graph); idx->g_graph = nullptr; }
            const wv_stats st0 = idx->stats;
            int rc = -1;
            hipGraph_t gr = nullptr;
            hipError_t ec = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
            if (ec == hipSuccess) {
                rc = search_core(idx, s, d_queries, nq, d, k, mode, idx->present, idx->npresent, d_ids, d_dists,
                                 d_counts, mode == 1 ? d_flags : nullptr);
                ec = hipStreamEndCapture(s, &gr);
            }
            hipGraphExec_t ex = nullptr;
            if (rc == 0 && ec == hipSuccess && gr && hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0) == hipSuccess) {
                idx->g_graph = gr;
                idx->g_exec = ex;
                idx->g_key = key;
                idx->g_dq = idx->stats.queries - st0.queries;
                idx->g_db = idx->stats.batches - st0.batches;
                idx->g_dm = idx->stats.mfma_launches - st0.mfma_launches;
                idx->g_timed = idx->timed;
                idx->g_timed_total = idx->timed_total;
                HIPCHK(hipGraphLaunch(ex, s));
                return WV_OK;
            }
            // not capturable (or failed): this call runs uncaptured below, and so do its repeats
            if (gr) hipGraphDestroy(gr);
            (void)hipGetLastError();
            idx->stats = st0;
            idx->g_failed = true;
        } else if (!(key == idx->g_seen)) {
            idx->g_seen = key;
            idx->g_failed = false;
        }
    }
    int rc = search_core(idx, s, d_queries, nq, d, k, mode, idx->present, idx->npresent, d_ids, d_dists, d_counts,
                         mode == 1 ? d_flags : nullptr);
    if (rc) return rc;
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
static void* batch_pinned_alloc(size_t bytes) {
    void* p = nullptr;
    return hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}
static void batch_pinned_free(void* p) { (void)hipHostFree(p); }
// page-locked rows for the batcher's allow bitmaps, mapped for kernels and
// fine-grained: the callers rewrite a row for each list and the search reads
// it in place (k_pqa_from_rows), so the device must not keep a cached copy
static uint32_t* batch_row_alloc(int64_t words, const uint32_t** dev) {
    void* p = nullptr;
    if (hipHostMalloc(&p, (size_t)std::max<int64_t>(words, 1) * sizeof(uint32_t),
                      hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess)
        return nullptr;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess) { (void)hipHostFree(p); return nullptr; }
    *dev = static_cast<const uint32_t*>(dp);
    return static_cast<uint32_t*>(p);
}
static void batch_row_free(uint32_t* p) { (void)hipHostFree(p); }
// the create-time base: id_base itself is shifted by a ScanWindow while a
// windowed search holds mu, and the callers read this without mu
static uint64_t batch_id_base(const wv_index* idx) { return idx->id_base0; }
static bool batch_rows_on(const wv_index* idx) { return idx->batch_rows.load(std::memory_order_relaxed) != 0; }
#include "batcher.hip"
