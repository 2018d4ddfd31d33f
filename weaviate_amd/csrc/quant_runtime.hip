// quant_runtime.hip -- BQ-compressed flat search and its sharded entry points,
// the product quantizer (fit, encode, search), the scalar quantizer, the
// rotational quantizers and hnsw's flat search over compressed vectors
// (see rt_index.h for the unit split).
#include "rt_index.h"

static bool bq8_route(const wv_index* idx) { return idx->bq8 != nullptr && idx->bq8_opt && idx->bq_kernel != 1; }
// rows per block minimum of the route: 32 on the integer MFMA (the block count
// rounded to whole ring slots: two blocks per slot up to 768 bits), 256 otherwise
static int64_t bq_blk(const wv_index* idx) { return bq8_route(idx) ? 32 : BQBLK; }
static int64_t bq_nblk(const wv_index* idx) {
    const int64_t nb = std::max<int64_t>((idx->hiwater + bq_blk(idx) - 1) / bq_blk(idx), 1);
    return bq8_route(idx) && idx->dpb8b <= 768 ? round_up(nb, 2) : nb;
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
    const int64_t nblk = bq_nblk(idx);
    // identity query list
    HIPCHK(idx->ident.ensure((size_t)nq * sizeof(int32_t)));
    {
        std::vector<int32_t> id((size_t)nq);
        for (int64_t i = 0; i < nq; i++) id[i] = (int32_t)i;
        HIPCHK(hipMemcpyAsync(idx->ident.p, id.data(), (size_t)nq * sizeof(int32_t), hipMemcpyHostToDevice, s));
    }
    constexpr int QPB = 16;
    // one group of block minima up to 4 GiB (the 32-row minima of the integer
    // route are 8x the 256-row ones: C4's 2048 x 195k blocks = 1.6 GB)
    *G_out = std::max<int64_t>(QPB, std::min<int64_t>(round_up(nq, QPB), ((4ll << 30) / (nblk * 4)) / QPB * QPB));
    *R_out = R;
    // the integer-MFMA minima write whole 256-query groups
    HIPCHK(idx->bqmin.ensure((size_t)round_up(*G_out, 256) * nblk * sizeof(float)));
    idx->bq_nq = nq;
    idx->bq_R = R;
    return WV_OK;
}

// the block minima on the integer matrix cores: the +-1 planes of the codes
// (k_bq_unpack8) through k_q8_blockkey<..., BQ>; hamming = (64 words - dot) / 2

static int bq_blockmin_i8(wv_index* idx, hipStream_t s, const uint32_t* valid, int64_t g0, int F, int64_t nblk,
                          float* bm) {
    const int dpb8 = idx->dpb8b;
    const int NC = dpb8 / 64;
    const int RB = dpb8 <= 768 ? 2 : 1;
    const int64_t Fp = round_up(F, 256);
    HIPCHK(idx->q8Qb.ensure((size_t)Fp * dpb8));
    HIPCHK(hipMemsetAsync(idx->q8Qb.p, 0, (size_t)Fp * dpb8, s));
    {
        const int64_t nu = (int64_t)F * (dpb8 / 4);
        k_bq_unpack8<<<(unsigned)((nu + 255) / 256), 256, 0, s>>>(idx->qcodes.as<uint64_t>() + g0, idx->bq_nq, idx->words,
                                                                  F, nullptr, dpb8, idx->q8Qb.as<unsigned char>());
    }
    Q8Args a;
    a.X8 = idx->bq8;
    a.sb = reinterpret_cast<const float*>(valid);  // any readable [nblocks] array: BQ has no scales
    a.xnorm2 = nullptr;
    a.valid = valid;
    a.Q8 = idx->q8Qb.as<unsigned char>();
    a.qscale = nullptr;
    a.key = bm;
    a.ldk = nblk;  // 32-row blocks (a multiple of RB: bq_nblk)
    a.bq_bits = 64 * idx->words;
    a.nslots = nblk / RB;
    a.nqg = (int)(Fp / 256);
    // whole rounds of one workgroup per CU
    int64_t nspans = 256 / std::gcd((int64_t)256, (int64_t)a.nqg);
    while ((int64_t)a.nqg * nspans < 256) nspans *= 2;
    {   // a span's plane bytes below 4 GiB (32-bit buffer offsets)
        const int64_t slot_b = (int64_t)RB * 32 * dpb8;
        const int64_t max_sps = ((1ll << 32) - 2 * 256ll * dpb8) / slot_b;
        nspans = std::max<int64_t>(nspans, (a.nslots + max_sps - 1) / max_sps);
    }
    nspans = std::max<int64_t>(1, std::min<int64_t>(nspans, a.nslots));
    const int64_t sps = (a.nslots + nspans - 1) / nspans;
    a.slots_per_span = (int)sps;
    a.nspans = (int)((a.nslots + sps - 1) / sps);
    const size_t lds = (size_t)3 * RB * 2 * NC * 1024 + 1024;
    dim3 grid((unsigned)((int64_t)a.nqg * a.nspans));
#define WV_BQ8(NCV, RBV)                                                                                        \
    do {                                                                                                        \
        HIPCHK(hipFuncSetAttribute((const void*)k_q8_blockkey<NCV, RBV, false, false, true>,                    \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                      \
        k_q8_blockkey<NCV, RBV, false, false, true><<<grid, 512, lds, s>>>(a);                                  \
    } while (0)
    switch (NC) {
    case 8: WV_BQ8(8, 2); break;
    case 10: WV_BQ8(10, 2); break;
    case 12: WV_BQ8(12, 2); break;
    case 16: WV_BQ8(16, 1); break;
    case 20: WV_BQ8(20, 1); break;
    default: WV_BQ8(24, 1); break;
    }
#undef WV_BQ8
    HIPCHK(hipGetLastError());
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
    const int64_t nblk = bq_nblk(idx);
    const int words = idx->words;
    const int nw = bq_nw(idx);
    const int32_t* qlist = idx->ident.as<int32_t>();
    // timing (bench roofline): the block-minima pass of the first group
    if (idx->timing && g0 == 0) HIPCHK(hipEventRecord(idx->ev0, s));
    const uint64_t* qc = idx->qcodes.as<uint64_t>();
    float* bm = idx->bqmin.as<float>();
    if (bq8_route(idx)) {
        int rc = bq_blockmin_i8(idx, s, valid, g0, F, nblk, bm);
        if (rc) return rc;
        if (idx->timing && g0 == 0) HIPCHK(hipEventRecord(idx->ev1, s));
        idx->stats.last_route = WV_ROUTE_BQ_INT8;
        return WV_OK;
    }
    idx->stats.last_route = WV_ROUTE_BQ_VALU;
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
                     int cap = 0, const int32_t* skip = nullptr) {
    const int64_t nq = idx->bq_nq;
    const int R = idx->bq_R;
    const int64_t nslots = idx->hiwater;
    const int64_t nblk = bq_nblk(idx);
    const bool b32 = bq_blk(idx) == 32;
    const int words = idx->words;
    const int nw = bq_nw(idx);
    const int32_t* qlist = idx->ident.as<int32_t>();
    const uint64_t* qc = idx->qcodes.as<uint64_t>();
    const float* bm = idx->bqmin.as<float>();
    const size_t lds_r = packed_replay_lds(R);
    if (lds_r > 160 * 1024) return set_err(WV_ERR_UNSUPPORTED, "rescore limit %d too large for the replay heap", R);
#define WV_RPB(NWV, RECV, BLKV)                                                                                 \
    do {                                                                                                        \
        if (lds_r > 64 * 1024)                                                                                  \
            HIPCHK(hipFuncSetAttribute((const void*)k_bq_replay<NWV, RECV, BLKV>,                               \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_r));                \
        k_bq_replay<NWV, RECV, BLKV><<<(unsigned)F, 64, lds_r, s>>>(idx->codes, idx->cap, words, valid, nslots, qc, nq, \
                                                              qlist + g0, F, bm, nblk, R, idx->id_base, in_ids, \
                                                              in_d, in_len, pop, out_ids, out_d, out_n, rec_ids, \
                                                              rec_d, rec_n, cap, skip);                         \
    } while (0)
#define WV_RPR(NWV, RECV)                                          \
    do {                                                           \
        if constexpr (NWV > 0) {                                   \
            if (b32) WV_RPB(NWV, RECV, 32);                        \
            else WV_RPB(NWV, RECV, BQBLK);                         \
        } else {                                                   \
            WV_RPB(NWV, RECV, BQBLK);                              \
        }                                                          \
    } while (0)
#define WV_RP(NWV) do { if (rec_n) WV_RPR(NWV, true); else WV_RPR(NWV, false); } while (0)
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
#undef WV_RPR
#undef WV_RPB
#undef WV_RP
    HIPCHK(hipGetLastError());
    return WV_OK;
}

// The replay-free answer of k_bq_fast (32-row minima, 8-24 code words, k <= 64,
// not hamming): skip[li] = 1 for every query of the group it answered (its
// candidate list then holds its m result ids)
static bool bq_fast(wv_index* idx, hipStream_t s, const uint32_t* valid, int64_t g0, int F, int k, uint64_t* out_ids,
                    int32_t* out_n, int32_t* skip, int* rc) {
    *rc = WV_OK;
    const int nw = bq_nw(idx);
    if (!idx->bq_fast || bq_blk(idx) != 32 || k > BQF_K || idx->metric == WV_METRIC_HAMMING ||
        (nw != 8 && nw != 12 && nw != 16 && nw != 24))
        return false;
    const bool v5 = idx->variant == WV_VARIANT_AVX512;
    const int32_t* qlist = idx->ident.as<int32_t>() + g0;
    const uint64_t* qc = idx->qcodes.as<uint64_t>();
    const float* Qn = idx->qn.as<float>();
#define WV_BF(NWV, M, V)                                                                                        \
    k_bq_fast<NWV, M, V><<<(unsigned)F, 256, 0, s>>>(idx->codes, idx->cap, idx->words, valid, idx->hiwater, qc,  \
                                                     idx->bq_nq, qlist, F, idx->bqmin.as<float>(), bq_nblk(idx), \
                                                     idx->bq_R, k, idx->X, idx->dpad, Qn, idx->dims, idx->id_base, \
                                                     out_ids, out_n, skip)
#define WV_BFM(NWV)                                                                                             \
    do {                                                                                                        \
        switch (idx->metric) {                                                                                  \
        case WV_METRIC_L2_SQUARED: if (v5) WV_BF(NWV, L2, AVX512); else WV_BF(NWV, L2, AVX256); break;          \
        case WV_METRIC_DOT: if (v5) WV_BF(NWV, DOT, AVX512); else WV_BF(NWV, DOT, AVX256); break;               \
        default: if (v5) WV_BF(NWV, COSINE, AVX512); else WV_BF(NWV, COSINE, AVX256); break;                    \
        }                                                                                                       \
    } while (0)
    switch (nw) {
    case 8: WV_BFM(8); break;
    case 12: WV_BFM(12); break;
    case 16: WV_BFM(16); break;
    default: WV_BFM(24); break;
    }
#undef WV_BFM
#undef WV_BF
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) *rc = set_err(WV_ERR_HIP, "k_bq_fast: %s", hipGetErrorString(e));
    return *rc == WV_OK;
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
                    int32_t* o_n, int asc = 0) {
    const size_t lds_f = (size_t)k * (sizeof(uint64_t) + sizeof(float)) + 16;
    if (lds_f > 64 * 1024)
        HIPCHK(hipFuncSetAttribute((const void*)k_bq_final, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_f));
    k_bq_final<<<(unsigned)nq, 64, lds_f, s>>>(ids, E, cnt, qlist, (int)nq, R, k, world, id_stride, o_ids, o_d, o_n, asc);
    HIPCHK(hipGetLastError());
    return WV_OK;
}

int search_bq(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k,
                     const uint32_t* valid, uint64_t* o_ids, float* o_d, int32_t* o_n) {
    int R = 0;
    int64_t G = 0;
    int rc = bq_begin(idx, s, d_qraw, nq, qd, k, &R, &G);
    if (rc) return rc;
    HIPCHK(idx->ascI.ensure((size_t)nq * R * sizeof(uint64_t)));
    HIPCHK(idx->ascD.ensure((size_t)nq * R * sizeof(float)));
    HIPCHK(idx->cn.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(idx->candE.ensure((size_t)nq * R * sizeof(float)));
    idx->bq_last_nq = G >= nq ? nq : 0;  // debug hook: a one-group batch's minima stay in bqmin
    idx->bq_last_nblk = bq_nblk(idx);
    idx->bq_last_blk = bq_blk(idx);
    for (int64_t g0 = 0; g0 < nq; g0 += G) {
        const int F = (int)std::min<int64_t>(G, nq - g0);
        rc = bq_blockmin(idx, s, valid, g0, F);
        if (rc) return rc;
        HIPCHK(idx->bqSkip.ensure((size_t)nq * sizeof(int32_t)));
        int32_t* skip = idx->bqSkip.as<int32_t>() + g0;
        const bool fast = bq_fast(idx, s, valid, g0, F, k, idx->ascI.as<uint64_t>() + g0 * R,
                                  idx->cn.as<int32_t>() + g0, skip, &rc);
        if (rc) return rc;
        rc = bq_replay(idx, s, valid, g0, F, nullptr, nullptr, nullptr, 1, idx->ascI.as<uint64_t>() + g0 * R,
                       idx->ascD.as<float>() + g0 * R, idx->cn.as<int32_t>() + g0, nullptr, nullptr, nullptr, 0,
                       fast ? skip : nullptr);
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

extern "C" int wv_index_debug_bqmin(wv_index* idx, int64_t q, float* mins, int64_t* nblk, int64_t* blk_rows) {
    if (!idx || !nblk) return set_err(WV_ERR_INVALID, "nil argument");
    if (blk_rows) *blk_rows = idx->bq_last_blk;
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->compression != WV_COMPRESSION_BQ || idx->bq_last_nq <= 0 || q < 0 || q >= idx->bq_last_nq)
        return set_err(WV_ERR_INVALID, "debug_bqmin: no such query in the last BQ batch's first group");
    *nblk = idx->bq_last_nblk;
    if (!mins) return WV_OK;
    HIPCHK(hipStreamSynchronize(idx->stream));
    HIPCHK(hipMemcpy(mins, idx->bqmin.as<float>() + q * idx->bq_last_nblk, (size_t)idx->bq_last_nblk * sizeof(float),
                     hipMemcpyDeviceToHost));
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
    const int64_t nblk = bq_nblk(idx);
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
    idx->pq8_mu_dirty = 1;  // a new codebook: mu and every block of the reconstruction plane
    pq8_mark(idx, 0, idx->hiwater);
    launch_pq_encode(idx, idx->hiwater, nullptr);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(idx->stream));
    idx->pq_trained = 1;
    return WV_OK;
}

// k-means of every segment over the n training rows T [n][dpad] (device, on
// idx's device), then Encode of every stored row.  Caller holds idx->mu.
int pq_fit_rows(wv_index* idx, const float* dT, int64_t n, uint64_t seed) {
    int rc = pq_validate(idx);
    if (rc) return rc;
    const int m = idx->pq_m, K = idx->pq_ks, ds = idx->pq_ds;
    hipStream_t s = idx->stream;
    if (n < K) return set_err(WV_ERR_INVALID, "not enough data to fit k-means");  // kmeans.go:459-461
    rc = pq_alloc(idx);
    if (rc) return rc;
    DBuf sub, asg, nbi, nbd, chg, act;
    const int64_t ldt = idx->dpad;
    float* C = idx->pq_centers;
    const size_t lds_c = (size_t)K * ds * sizeof(float);
    if (K == 1) {  // computeCentroid (kmeans.go:447-452): every row in cluster 0
        HIPCHK(asg.ensure((size_t)m * n * sizeof(uint32_t)));
        HIPCHK(hipMemsetAsync(asg.p, 0, (size_t)m * n * sizeof(uint32_t), s));
        const size_t lds_u = (size_t)K * ds * sizeof(double) + KM_T * sizeof(uint32_t) + (size_t)KM_T * ds * sizeof(float);
        k_km_update_centers<<<m, KM_T, lds_u, s>>>(dT, ldt, n, K, ds, asg.as<uint32_t>(), nullptr, C);
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
        k_km_gather_centers<<<(unsigned)((tot + 255) / 256), 256, 0, s>>>(dT, ldt, sub.as<int64_t>(), m, K, ds,
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
    k_km_assign_brute<<<rgrid, 256, lds_c, s>>>(dT, ldt, n, K, ds, C, idx->variant, nullptr, asg.as<uint32_t>());
    k_km_update_centers<<<m, KM_T, lds_u, s>>>(dT, ldt, n, K, ds, asg.as<uint32_t>(), nullptr, C);
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
        k_km_assign_prune<<<rgrid, 256, lds_c, s>>>(dT, ldt, n, K, ds, C, idx->variant, nbi.as<uint32_t>(),
                                                    nbd.as<float>(), act.as<int32_t>(), asg.as<uint32_t>(),
                                                    chg.as<unsigned long long>());
        k_km_update_centers<<<m, KM_T, lds_u, s>>>(dT, ldt, n, K, ds, asg.as<uint32_t>(), act.as<int32_t>(),
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
    sub.release(); asg.release(); nbi.release(); nbd.release(); chg.release(); act.release();
    return pq_encode_all(idx);
}

extern "C" int wv_index_pq_fit(wv_index* idx, uint64_t seed) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->compression != WV_COMPRESSION_PQ) return set_err(WV_ERR_INVALID, "pq_fit: index is not PQ-compressed");
    int rc = pq_validate(idx);
    if (rc) return rc;
    hipStream_t s = idx->stream;
    // training data: ProductQuantizer.Fit truncates to trainingLimit (:379-381)
    std::vector<uint32_t> tslots;
    for (int64_t sl = 0; sl < idx->hiwater; sl++)
        if (idx->h_present[sl]) tslots.push_back((uint32_t)sl);
    int64_t n = (int64_t)tslots.size();
    if (idx->pq_training_limit > 0 && n > idx->pq_training_limit) n = idx->pq_training_limit;
    if (n < idx->pq_ks) return set_err(WV_ERR_INVALID, "not enough data to fit k-means");  // kmeans.go:459-461
    // T = the n training rows (gathered, dpad stride)
    DBuf T;
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
    rc = pq_fit_rows(idx, T.as<float>(), n, seed);
    HIPCHK(hipStreamSynchronize(s));
    return rc;
}

// the largest batch wv_index_bq_begin takes on this shard (one block-minima group)
int64_t bq_max_batch(const wv_index* idx) {
    constexpr int QPB = 16;
    return std::max<int64_t>(QPB, ((4ll << 30) / (bq_nblk(idx) * 4)) / QPB * QPB);
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

int rq_encode_queries(wv_index* idx, hipStream_t s, int64_t nq);

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
// the compressed distances E[f][row] (+inf for invalid rows) and their 256-row
// block minima of listed queries [g0, g0 + F) (PQ: qlist positions; the
// thread-per-row SQ / RQ / BQ kernels index the query batch directly)
static int hnsw_dist(wv_index* idx, hipStream_t s, int comp, const uint32_t* valid, const int32_t* qlist, int64_t nq,
                     int64_t g0, int F, int64_t ld, float* E, float* Bm) {
    const int64_t nslots = idx->hiwater;
    const int wrapm = idx->metric == WV_METRIC_L2_SQUARED ? L2 : idx->metric == WV_METRIC_DOT ? DOT : COSINE;
    int rc = WV_OK;
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
    return rc;
}

// hnsw flat search, shared part: validation, query preparation, the
// compressor's per-query state (LUT / codes), the identity query list.
// *limit_io: the worker-heap limit (>= k on return); *comp_out: the compressor.
static int hnsw_prep(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k, int* limit_io,
                     int* comp_out) {
    int limit = *limit_io;
    int rc = WV_OK;
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
    *limit_io = limit;
    *comp_out = comp;
    if (R > 8192) return set_err(WV_ERR_UNSUPPORTED, "limit %d > 8192", R);
    const int64_t nq_pad = round_up(nq, QB);
    rc = prepare_queries(idx, s, d_qraw, nq, nq_pad);
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
    (void)R;
    return WV_OK;
}

// ---- PQ block keys on the integer matrix cores (pq_kernels.hip §3.6b) ----
static int pq8_dpb8(int d) { return d <= 768 ? (int)round_up(d, 128) : (int)round_up(d, 256); }

// l2-squared, 384 < d <= 1536 (the int8 key kernels' plane widths), a worker
// heap the 448-block candidate lists hold, key rows within 16 GiB
static bool pq8_route(const wv_index* idx, int R, int64_t nq) {
    if (!idx->pq8_opt || idx->compression != WV_COMPRESSION_PQ || !idx->pq_trained || idx->pq8_bad ||
        idx->metric != WV_METRIC_L2_SQUARED || idx->dims <= 384 || idx->dims > 1536 || R + 1 > 448 ||
        idx->hiwater <= 0)
        return false;
    const int dpb8 = pq8_dpb8(idx->dims);
    const int RB = dpb8 <= 768 ? 2 : 1;
    const int64_t nb = (idx->hiwater + 32 * RB - 1) / (32 * RB) * RB;
    return round_up(nq, QS_QPB) * nb * 4 <= (16ll << 30);
}

// the centred reconstruction plane up to date: (re)allocated with the index's
// capacity, mu from the codebook, the dirty slot range re-decoded and
// re-quantised in chunks of 2^18 rows
static int pq8_sync(wv_index* idx, hipStream_t s) {
    const int dims = idx->dims, dpad = idx->dpad, dpb8 = pq8_dpb8(dims);
    bool full = false;
    if (idx->pq8_cap != idx->cap || idx->pq8_dpb8 != dpb8 || !idx->pq8_X8) {
        if (idx->pq8_X8) hipFree(idx->pq8_X8);
        if (idx->pq8_sb) hipFree(idx->pq8_sb);
        if (idx->pq8_n2) hipFree(idx->pq8_n2);
        idx->pq8_X8 = nullptr; idx->pq8_sb = nullptr; idx->pq8_n2 = nullptr;
        idx->pq8_cap = 0;
        HIPCHK(hipMalloc(&idx->pq8_X8, (size_t)idx->cap * dpb8));
        HIPCHK(hipMalloc(&idx->pq8_sb, (size_t)(idx->cap / 32) * sizeof(float)));
        HIPCHK(hipMalloc(&idx->pq8_n2, (size_t)idx->cap * sizeof(float)));
        HIPCHK(hipMemsetAsync(idx->pq8_X8, 0, (size_t)idx->cap * dpb8, s));
        HIPCHK(hipMemsetAsync(idx->pq8_sb, 0, (size_t)(idx->cap / 32) * sizeof(float), s));
        HIPCHK(hipMemsetAsync(idx->pq8_n2, 0, (size_t)idx->cap * sizeof(float), s));
        idx->pq8_cap = idx->cap;
        idx->pq8_dpb8 = dpb8;
        full = true;
    }
    if (idx->pq8_mu_dirty) {  // mu = the per-dimension mean of the codebook
        const int m = idx->pq_m, K = idx->pq_ks, ds = idx->pq_ds;
        std::vector<float> cen((size_t)m * K * ds);
        HIPCHK(hipMemcpy(cen.data(), idx->pq_centers, cen.size() * sizeof(float), hipMemcpyDeviceToHost));
        std::vector<float> mu((size_t)dpad, 0.f);
        for (int sg = 0; sg < m; sg++)
            for (int e = 0; e < ds; e++) {
                double acc = 0.0;
                for (int c = 0; c < K; c++) acc += cen[((size_t)sg * K + c) * ds + e];
                mu[(size_t)sg * ds + e] = (float)(acc / K);
            }
        HIPCHK(idx->pq8Mu.ensure((size_t)dpad * sizeof(float)));
        HIPCHK(hipMemcpy(idx->pq8Mu.p, mu.data(), (size_t)dpad * sizeof(float), hipMemcpyHostToDevice));
        idx->pq8_mu_dirty = 0;
        full = true;
    }
    HIPCHK(idx->pq8Max.ensure(8 * sizeof(uint32_t)));
    int64_t lo = idx->pq8_lo, hi = idx->pq8_hi;
    if (full) {
        HIPCHK(hipMemsetAsync(idx->pq8Max.p, 0, 8 * sizeof(uint32_t), s));
        lo = 0;
        hi = idx->hiwater;
    }
    hi = std::min<int64_t>(hi, idx->hiwater);
    idx->pq8_lo = idx->pq8_hi = 0;
    if (hi <= lo) return WV_OK;
    const int64_t r0 = lo / 32 * 32, r1 = std::min<int64_t>(round_up(hi, 32), idx->cap);
    const int64_t chunk = 1 << 18;
    HIPCHK(idx->pq8Tmp.ensure((size_t)std::min<int64_t>(chunk, r1 - r0) * dpad * sizeof(float)));
    float* tmp = idx->pq8Tmp.as<float>();
    uint32_t* mx = idx->pq8Max.as<uint32_t>();
    for (int64_t a = r0; a < r1; a += chunk) {
        const int64_t n = std::min<int64_t>(chunk, r1 - a);
        k_pq_decode_center<<<(unsigned)((n + 3) / 4), 256, 0, s>>>(idx->pq_codes, pq_g16(idx->pq_m), idx->pq_m,
                                                                    idx->pq_ds, idx->pq_ks, idx->pq_centers,
                                                                    idx->pq8Mu.as<float>(), a, n, dims, dpad, tmp,
                                                                    idx->pq8_n2, mx);
        // k_block_q8 addresses rows absolutely: shift the chunk buffer by its first row
        k_block_q8<<<(unsigned)(n / 32), 256, 0, s>>>(tmp - a * dpad, dpad, dims, dpb8, nullptr, a / 32, idx->pq8_X8,
                                                       idx->pq8_sb, mx);
        HIPCHK(hipGetLastError());
    }
    uint32_t bad = 0;
    HIPCHK(hipMemcpyAsync(&bad, mx + 2, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    idx->pq8_bad = bad ? 1 : 0;  // a non-finite centroid: the LUT minima route from now on
    return WV_OK;
}

// keys on the centred int8 planes -> candidate 32-row blocks (eps covers the
// key's quantisation, the ADC's fp32 rounding and the centring) -> exact ADC
// of their rows below the cap -> asc (ascI / ascD / ascN) or a flag in oF
static int pq8_candidates(wv_index* idx, hipStream_t s, int64_t nq, int R, const uint32_t* valid) {
    int rc = pq8_sync(idx, s);
    if (rc) return rc;
    if (idx->pq8_bad) return set_err(WV_ERR_UNSUPPORTED, "pq8: non-finite codebook");
    const int dims = idx->dims, dpad = idx->dpad, dpb8 = idx->pq8_dpb8;
    const int m = idx->pq_m, K = idx->pq_ks;
    const int64_t nq_pad = round_up(nq, QS_QPB);
    const int RB = dpb8 <= 768 ? 2 : 1;
    const int64_t nslots = (idx->hiwater + 32 * RB - 1) / (32 * RB);
    const int64_t nb = nslots * RB;
    constexpr int RV = 8, L = 64 * (RV - 1);
    HIPCHK(idx->pq8Qc.ensure((size_t)nq_pad * dpad * sizeof(float)));
    HIPCHK(idx->qsInfo.ensure((size_t)nq_pad * sizeof(float4)));
    HIPCHK(idx->q8Qb.ensure((size_t)nq_pad * dpb8));
    HIPCHK(idx->q8Scale.ensure((size_t)nq_pad * sizeof(float)));
    HIPCHK(idx->q8Info.ensure((size_t)nq_pad * sizeof(float4)));
    HIPCHK(idx->qsKey.ensure((size_t)nq_pad * nb * sizeof(float)));
    HIPCHK(idx->qsCand.ensure((size_t)nq * L * sizeof(uint32_t)));
    HIPCHK(idx->qsNc.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(idx->qsEps.ensure((size_t)nq * sizeof(float)));
    HIPCHK(idx->qsCap.ensure((size_t)nq * sizeof(float)));
    HIPCHK(idx->qsFlags.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(idx->oF.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(idx->qsList.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(idx->flCtr.ensure(2 * sizeof(uint32_t)));
    float4* qinfo = idx->qsInfo.as<float4>();
    k_pq_center_queries<<<(unsigned)(nq_pad / 4), 256, 0, s>>>(idx->qn.as<float>(), dpad, dims, idx->pq8Mu.as<float>(),
                                                               nq, nq_pad, idx->pq8Qc.as<float>(), qinfo);
    k_query_q8<<<(unsigned)(nq_pad / 4), 256, 0, s>>>(idx->pq8Qc.as<float>(), dpad, dims, dpb8, nq, nq_pad, qinfo,
                                                      idx->q8Qb.as<unsigned char>(), idx->q8Scale.as<float>(),
                                                      idx->q8Info.as<float4>());
    HIPCHK(hipGetLastError());
    Q8Args a{};
    a.X8 = idx->pq8_X8;
    a.sb = idx->pq8_sb;
    a.xnorm2 = idx->pq8_n2;
    a.valid = valid;
    a.Q8 = idx->q8Qb.as<unsigned char>();
    a.qscale = idx->q8Scale.as<float>();
    a.key = idx->qsKey.as<float>();
    a.ldk = nb;
    a.nslots = nslots;
    a.nqg = (int)(nq_pad / QS_QPB);
    if (idx->timing) HIPCHK(hipEventRecord(idx->ev0, s));
    rc = launch_q8_keys(idx, s, a, dpb8, true);
    if (rc) return rc;
    if (idx->timing) HIPCHK(hipEventRecord(idx->ev1, s));
    idx->stats.last_group_queries = (uint64_t)nq;
    idx->stats.last_route = WV_ROUTE_PQ_INT8;
    idx->stats.mfma_launches++;
    // |A - ADC| <= eps: qs_eps's l2 form with g_d covering the plane norms'
    // fp32 sums (dpb8 terms), the ADC's (m LUT sums of ds terms, all
    // non-negative: relative error gamma_{m + ds + 3} <= (|q_c| + N)^2 terms)
    // and 2u for the centring's two roundings
    const uint32_t* mx = idx->pq8Max.as<uint32_t>();
    const float gd = (float)(gamma_n(std::max(dpb8, m + idx->pq_ds) + 8) + 2.0 * 5.9604644775390625e-08);
    const float gacc8 = 4.0001f * 5.9604645e-08f;
    const int RT = qs_R(R);
    const unsigned gw = (unsigned)((nq + 3) / 4);
#define WV_PQSEL(RTV) k_blk_select_f<RV, RTV><<<gw, 256, 0, s>>>(a.key, nb, nb, (int)nq, R, L2, idx->q8Info.as<float4>(), mx, mx + 4, gd, gacc8, idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(), idx->qsFlags.as<int32_t>(), idx->qsEps.as<float>(), nullptr, nullptr, nullptr, idx->qsCap.as<float>(), nullptr)
    if (RT == 2) WV_PQSEL(2);
    else if (RT == 4) WV_PQSEL(4);
    else
        k_blk_select<RV><<<gw, 256, 0, s>>>(a.key, nb, nb, (int)nq, R, L2, idx->q8Info.as<float4>(), mx, mx + 4, gd,
                                            gacc8, idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(),
                                            idx->qsFlags.as<int32_t>(), idx->qsEps.as<float>(), nullptr, nullptr,
                                            nullptr, idx->qsCap.as<float>(), nullptr);
#undef WV_PQSEL
    HIPCHK(hipGetLastError());
    // the int8 row bound, block-major: each listed block's codes read once
    // (k_q8_filt_bm), survivor masks for the exact ADC below
    uint32_t* fmask = nullptr;
    if (idx->q8_bm) {
        HIPCHK(idx->fMask.ensure((size_t)nq * L * sizeof(uint32_t)));
        rc = invert_lists(idx, s, idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(), idx->qsFlags.as<int32_t>(), nq,
                          L, nb);
        if (rc) return rc;
        Q8Filter f{idx->pq8_X8, idx->pq8_sb, dpb8, idx->q8Qb.as<unsigned char>(), idx->q8Scale.as<float>(),
                   idx->q8Info.as<float4>(), mx, gacc8};
        launch_q8_filt_bm(idx, s, L2, f, idx->pq8_n2, valid, nb, L, idx->qsCap.as<float>(), idx->q8Info.as<float4>(), gd,
                          idx->fMask.as<uint32_t>());
        HIPCHK(hipGetLastError());
        fmask = idx->fMask.as<uint32_t>();
    }
#define WV_PQC8(KCV, CAND, LV, FM, QL, QC) k_pq_cand8<KCV><<<(unsigned)nq, 256, 0, s>>>(idx->pq_codes, pq_g16(m), m, K, valid, idx->hiwater, idx->lut.as<float>(), CAND, LV, idx->qsNc.as<int32_t>(), idx->qsFlags.as<int32_t>(), idx->qsCap.as<float>(), R, L2, idx->id_base, idx->ascI.as<uint64_t>(), idx->ascD.as<float>(), idx->ascN.as<int32_t>(), idx->oF.as<int32_t>(), FM, QL, QC)
    if (K == 256) WV_PQC8(256, idx->qsCand.as<uint32_t>(), L, fmask, nullptr, nullptr);
    else WV_PQC8(0, idx->qsCand.as<uint32_t>(), L, fmask, nullptr, nullptr);
    HIPCHK(hipGetLastError());
    // queries whose 448-block lists overflowed (select flag 2): again with
    // 960-block lists (the sorted select over the listed queries), exact ADC of
    // every valid row of those blocks
    if (R + 1 <= 960) {
        constexpr int L16 = 64 * 15;
        HIPCHK(idx->qsCand2.ensure((size_t)nq * L16 * sizeof(uint32_t)));
        HIPCHK(hipMemsetAsync(idx->flCtr.p, 0, 2 * sizeof(uint32_t), s));
        k_flag_list<<<(unsigned)((nq + 255) / 256), 256, 0, s>>>(idx->qsFlags.as<int32_t>(), (int)nq,
                                                                  idx->qsList.as<int32_t>(), idx->flCtr.as<uint32_t>(), 2);
        k_blk_select<16><<<gw, 256, 0, s>>>(a.key, nb, nb, (int)nq, R, L2, idx->q8Info.as<float4>(), mx, mx + 4, gd,
                                            gacc8, idx->qsCand2.as<uint32_t>(), idx->qsNc.as<int32_t>(),
                                            idx->qsFlags.as<int32_t>(), idx->qsEps.as<float>(),
                                            idx->qsList.as<int32_t>(), idx->flCtr.as<uint32_t>(), nullptr,
                                            idx->qsCap.as<float>(), nullptr);
        if (K == 256) WV_PQC8(256, idx->qsCand2.as<uint32_t>(), L16, nullptr, idx->qsList.as<int32_t>(), idx->flCtr.as<uint32_t>());
        else WV_PQC8(0, idx->qsCand2.as<uint32_t>(), L16, nullptr, idx->qsList.as<int32_t>(), idx->flCtr.as<uint32_t>());
        HIPCHK(hipGetLastError());
    }
#undef WV_PQC8
    return WV_OK;
}

static int search_hnsw(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k, int limit,
                       int trim, int rescore, const uint32_t* valid, uint64_t* o_ids, float* o_d, int32_t* o_n) {
    int comp = 0;
    int rc = hnsw_prep(idx, s, d_qraw, nq, qd, k, &limit, &comp);
    if (rc) return rc;
    const int R = limit;
    const float* Qn = idx->qn.as<float>();
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
    const bool pq8 = comp == WV_COMPRESSION_PQ && pq8_route(idx, R, nq);
    if (pq8 || (comp == WV_COMPRESSION_PQ && idx->pq_cand && R + 1 <= 64)) {
      if (pq8) {
        rc = pq8_candidates(idx, s, nq, R, valid);
        if (rc) return rc;
      } else {
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
        const bool adc3 = idx->pq_adc3 && K == 256;
        if (adc3) {  // queries on the lanes: the LUT regrouped as [64-query group][segment][code][64]
            const int64_t ng = (nq + 63) / 64;
            const int64_t tot = ng * m * 256 * 64;
            HIPCHK(idx->lutg.ensure((size_t)tot * sizeof(float)));
            k_pq_lut_group<<<(unsigned)((tot + 255) / 256), 256, 0, s>>>(idx->lut.as<float>(), (int)nq, m, K, tot,
                                                                         idx->lutg.as<float>());
            HIPCHK(hipGetLastError());
        }
        if (idx->timing) HIPCHK(hipEventRecord(idx->ev0, s));
        if (adc3) {
            dim3 g3((unsigned)((nslots + PQ3_ROWS - 1) / PQ3_ROWS), (unsigned)((nq + 63) / 64));
#define WV_ADC3(DBGV) k_pq_adc3<DBGV><<<g3, 512, 0, s>>>(idx->pq_codes, pq_g16(m), m, valid, nslots, idx->lutg.as<float>(), (int)nq, wrapm, nblk, idx->rB.as<float>())
#define WV_ADC4(DBGV) k_pq_adc4<DBGV><<<g3, 512, 0, s>>>(idx->pq_codes, pq_g16(m), m, valid, nslots, \
                                   idx->lutg.as<float>(), (int)nq, wrapm, nblk, idx->rB.as<float>())
            if (idx->pq_adc3 == 2) WV_ADC4(0);
            else
#ifdef WV_PQ_DBG  // timing experiments only (wrong results), never in the product build
            if (idx->pq_adc3 == 5) WV_ADC4(1);
            else if (idx->pq_adc3 == 3) WV_ADC3(1);
            else if (idx->pq_adc3 == 4) WV_ADC3(2);
            else
#endif
            WV_ADC3(0);
#undef WV_ADC3
#undef WV_ADC4
        } else {
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
        }
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
        int32_t* const pflag = idx->oF.as<int32_t>();
#define WV_PQC(KCV) k_pq_cand<KCV><<<(unsigned)nq, 256, 0, s>>>(idx->pq_codes, pq_g16(m), m, K, valid, nslots, idx->lut.as<float>(), idx->rB.as<float>(), nblk, idx->qsCand.as<uint32_t>(), 64, idx->qsNc.as<int32_t>(), idx->qsFlags.as<int32_t>(), R, wrapm, idx->id_base, idx->ascI.as<uint64_t>(), idx->ascD.as<float>(), idx->ascN.as<int32_t>(), pflag)
        if (K == 256) WV_PQC(256);
        else WV_PQC(0);
#undef WV_PQC
        HIPCHK(hipGetLastError());
      }
        int32_t* pflag = idx->oF.as<int32_t>();
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
    int64_t gi = 0;
    for (int64_t g0 = 0; g0 < nrep; g0 += G, gi++) {
        const int F = (int)std::min<int64_t>(G, nrep - g0);
        const int b = (int)(gi & 1);
        float* E = Eb[b]->as<float>();
        float* Bm = Bb[b]->as<float>();
        if (gi >= 2) HIPCHK(hipStreamWaitEvent(s, idx->evr[b], 0));
        const bool time_it = idx->timing && g0 == 0 && !rep_by_query;
        if (time_it) HIPCHK(hipEventRecord(idx->ev0, s));
        rc = hnsw_dist(idx, s, comp, valid, qlist, nq, g0, F, ld, E, Bm);
        if (rc) return rc;
        HIPCHK(hipGetLastError());
        if (time_it) HIPCHK(hipEventRecord(idx->ev1, s));
        HIPCHK(hipEventRecord(idx->evd[b], s));
        HIPCHK(hipStreamWaitEvent(idx->aux, idx->evd[b], 0));
        // the worker heap (addResult == insertToHeap) in id order, extracted ascending
        // (rows by list position, or by query for the PQ candidate path's flagged list)
        const int64_t ao = rep_by_query ? 0 : g0;
        HIPCHK(launch_replay_scan(R, (unsigned)F, idx->aux, E, Bm, valid, nslots, ld, qlist + g0, F, R, idx->id_base,
                                  nullptr, nullptr, nullptr, 1, rep_by_query, R, idx->ascI.as<uint64_t>() + ao * R,
                                  idx->ascD.as<float>() + ao * R, idx->ascN.as<int32_t>() + ao, 0, 0, nullptr, nullptr,
                                  nullptr, 0));
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
int search_pq(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k,
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
int search_hnsw_flat(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k,
                            const uint32_t* valid, uint64_t* o_ids, float* o_d, int32_t* o_n) {
    const bool sqrq = idx->compression == WV_COMPRESSION_SQ || idx->rq_bits != 0;
    // shouldRescore (search.go:182-189); a PQ index created with pq_rescore = 0 counts as doNotRescore
    bool rescore = idx->hnsw_rescore != 0 && !(sqrq && idx->rescore_limit == 0);
    if (idx->compression == WV_COMPRESSION_PQ && !idx->pq_rescore) rescore = false;
    const int limit = rescore ? hnsw_search_ef(idx, k) : k;  // flat_search.go:31-33
    const int trim = (sqrq && idx->rescore_limit >= k) ? idx->rescore_limit : 0;
    return search_hnsw(idx, s, d_qraw, nq, qd, k, limit, trim, rescore ? 1 : 0, valid, o_ids, o_d, o_n);
}

// ---- sharded hnsw flat search over compressed vectors (weaviate_amd/sharded.py
// ShardedQuantSearch): every shard holds a contiguous id range with the same
// quantizer; the worker heap (limit R) spans the shards in id order, then the
// result heap and the rescoring follow -- the single index's search ----

// the parameters the index's own SearchByVector uses: search_pq (PQ),
// search_hnsw_flat (SQ) or search_rq (flat rq-8 / rq-1: searchByVectorQuantized,
// every worker-heap item rescored, *form = 1); BQ has ShardedBQSearch
static int quant_params(const wv_index* idx, int k, int* limit, int* trim, int* rescore, int* form) {
    *form = 0;
    if (idx->rq_bits) {
        *rescore = 1;
        *limit = idx->rescore_limit > k ? idx->rescore_limit : k;  // searchTimeRescore (flat/index.go:413-421)
        *trim = 0;
        *form = 1;
        return *limit > 8192 ? set_err(WV_ERR_UNSUPPORTED, "rescore limit %d > 8192", *limit) : WV_OK;
    }
    if (idx->compression == WV_COMPRESSION_PQ && idx->pq_trained) {
        *rescore = idx->pq_rescore ? 1 : 0;
        *limit = *rescore && idx->rescore_limit > k ? idx->rescore_limit : k;
        *trim = 0;
        return WV_OK;
    }
    if (idx->compression == WV_COMPRESSION_SQ) {
        const bool rs = idx->hnsw_rescore != 0 && idx->rescore_limit != 0;
        *rescore = rs ? 1 : 0;
        *limit = rs ? hnsw_search_ef(idx, k) : k;
        *trim = idx->rescore_limit >= k ? idx->rescore_limit : 0;
        return WV_OK;
    }
    return set_err(WV_ERR_UNSUPPORTED, "quant sharding: trained PQ, SQ or RQ indexes only");
}

// the largest batch wv_index_quant_begin takes on this shard for k at `world`
// ranks: one 16 GiB distance group, and at most 2 GiB each for the PQ lookup
// tables (nq m K floats) and the all-gathered replay records (world ranks x
// nq x (3 cap + 1) words, cap = 2R + 64), so no rank fails an allocation
// while the others wait in a collective
extern "C" int wv_index_quant_max_batch(wv_index* idx, int32_t k, int32_t world, int64_t* out) {
    if (!idx || !out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    const int64_t ld = std::max<int64_t>(round_up(idx->hiwater, EBLK), EBLK);
    int64_t mb = (16ll << 30) / (ld * 4);
    int limit = k, trim = 0, rescore = 0, form = 0;
    if (k > 0 && quant_params(idx, k, &limit, &trim, &rescore, &form) == WV_OK) {
        const int64_t cap = 2ll * limit + 64;
        mb = std::min<int64_t>(mb, (2ll << 30) / ((int64_t)std::max(world, 1) * (3 * cap + 1) * 4));
        if (idx->compression == WV_COMPRESSION_PQ && idx->pq_m > 0 && idx->pq_ks > 0)
            mb = std::min<int64_t>(mb, (2ll << 30) / ((int64_t)idx->pq_m * idx->pq_ks * 4));
    }
    *out = std::max<int64_t>(1, mb);
    return WV_OK;
}

// phase 1: query state + the compressed distances of every row of this shard to
// the whole batch (one group) and their 256-row block minima.
// out[4] = {R (worker-heap limit), block count, rescore, final form (0: h.rescore,
// 1: searchByVectorQuantized's rescoring heap)}
extern "C" int wv_index_quant_begin(wv_index* idx, const float* d_queries, int64_t nq, int64_t d, int32_t k,
                                    int64_t* out, void* stream) {
    if (!idx || !out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (nq <= 0) return set_err(WV_ERR_INVALID, "quant_begin: empty batch");
    if (k <= 0) return set_err(WV_ERR_INVALID, "k must be positive (reference heap Top() on empty queue)");
    int limit = 0, trim = 0, rescore = 0, comp = 0, form = 0;
    int rc = quant_params(idx, k, &limit, &trim, &rescore, &form);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    rc = hnsw_prep(idx, s, d_queries, nq, d, k, &limit, &comp);
    if (rc) return rc;
    const int64_t ld = std::max<int64_t>(round_up(idx->hiwater, EBLK), EBLK);
    if (nq * ld * 4 > (16ll << 30))
        return set_err(WV_ERR_UNSUPPORTED, "quant_begin: %lld queries x %lld rows exceed one 16 GiB distance group",
                       (long long)nq, (long long)ld);
    HIPCHK(idx->rE.ensure((size_t)nq * ld * sizeof(float)));
    HIPCHK(idx->rB.ensure((size_t)nq * (ld / EBLK) * sizeof(float)));
    if (idx->hiwater > 0) {
        if (idx->timing) HIPCHK(hipEventRecord(idx->ev0, s));
        rc = hnsw_dist(idx, s, comp, idx->present, idx->ident.as<int32_t>(), nq, 0, (int)nq, ld, idx->rE.as<float>(),
                       idx->rB.as<float>());
        if (rc) return rc;
        if (idx->timing) HIPCHK(hipEventRecord(idx->ev1, s));
        idx->stats.last_group_queries = (uint64_t)nq;
    } else {
        // no rows: every block minimum +inf (a finite fill would read as one row's distance)
        const int64_t nbm = nq * (ld / EBLK);
        k_fill_u32<<<(unsigned)((nbm + 255) / 256), 256, 0, s>>>(idx->rB.as<uint32_t>(), nbm, 0x7f800000u);
        HIPCHK(hipGetLastError());
    }
    idx->qt_nq = nq;
    idx->qt_ld = ld;
    idx->qt_k = k;
    idx->qt_R = limit;
    idx->qt_trim = trim;
    idx->qt_rescore = rescore;
    idx->qt_comp = comp;
    idx->qt_form = form;
    out[0] = limit;
    out[1] = ld / EBLK;
    out[2] = rescore;
    out[3] = form;
    if (!stream || (idx->timing && idx->hiwater > 0)) HIPCHK(hipStreamSynchronize(s));
    if (idx->timing && idx->hiwater > 0) {
        float ms = 0.f;
        hipEventElapsedTime(&ms, idx->ev0, idx->ev1);
        idx->stats.last_select_ms = ms;
    }
    return WV_OK;
}

// the block minima [nq][nblk] (each the compressed distance of one distinct row;
// the caller's R smallest bound the worker heap across shards)
extern "C" int wv_index_quant_blockmin(wv_index* idx, float* d_out, void* stream) {
    if (!idx || !d_out) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->qt_nq <= 0) return set_err(WV_ERR_INVALID, "quant_blockmin: no batch begun");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(d_out, idx->rB.p, (size_t)idx->qt_nq * (idx->qt_ld / EBLK) * sizeof(float),
                          hipMemcpyDeviceToDevice, s));
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

// the worker heap over this shard in id order from heap states d_in_* ([nq][R]
// layout order by query, NULL = empty): extract = 1 -> extracted ascending
// [nq][R], 0 -> the state; cap > 0 -> record every insertion in d_rec_*
static int quant_replay(wv_index* idx, hipStream_t s, const uint64_t* in_i, const float* in_d, const int32_t* in_n,
                        int extract, uint64_t* oi, float* od, int32_t* on, uint64_t* rec_i, float* rec_d,
                        int32_t* rec_n, int cap) {
    const int64_t nq = idx->qt_nq;
    const int R = idx->qt_R;
    HIPCHK(launch_replay_scan(R, (unsigned)nq, s, idx->rE.as<float>(), idx->rB.as<float>(), idx->present, idx->hiwater,
                              idx->qt_ld, idx->ident.as<int32_t>(), (int)nq, R, idx->id_base, in_i, in_d, in_n,
                              extract, 1, R, oi, od, on, 1, 1, rec_i, rec_d, rec_n, cap));
    return WV_OK;
}

extern "C" int wv_index_quant_replay(wv_index* idx, const uint64_t* d_in_ids, const float* d_in_d,
                                     const int32_t* d_in_len, int32_t extract, uint64_t* d_out_ids, float* d_out_d,
                                     int32_t* d_out_len, void* stream) {
    if (!idx || !d_out_ids || !d_out_d || !d_out_len) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->qt_nq <= 0) return set_err(WV_ERR_INVALID, "quant_replay: no batch begun");
    hipStream_t s = (hipStream_t)stream;
    int rc = quant_replay(idx, s, d_in_ids, d_in_d, d_in_len, extract ? 1 : 0, d_out_ids, d_out_d, d_out_len, nullptr,
                          nullptr, nullptr, 0);
    if (rc) return rc;
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

extern "C" int wv_index_quant_replay_record(wv_index* idx, const uint64_t* d_in_ids, const float* d_in_d,
                                            const int32_t* d_in_len, int32_t cap, uint64_t* d_rec_ids,
                                            float* d_rec_d, int32_t* d_rec_n, void* stream) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (cap < 1 || !d_rec_ids || !d_rec_d || !d_rec_n) return set_err(WV_ERR_INVALID, "invalid record buffers");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->qt_nq <= 0) return set_err(WV_ERR_INVALID, "quant_replay_record: no batch begun");
    hipStream_t s = (hipStream_t)stream;
    const int64_t nq = idx->qt_nq;
    const int R = idx->qt_R;
    HIPCHK(idx->ascI.ensure((size_t)nq * R * sizeof(uint64_t)));  // the state itself is not needed
    HIPCHK(idx->ascD.ensure((size_t)nq * R * sizeof(float)));
    HIPCHK(idx->ascN.ensure((size_t)nq * sizeof(int32_t)));
    int rc = quant_replay(idx, s, d_in_ids, d_in_d, d_in_len, 0, idx->ascI.as<uint64_t>(), idx->ascD.as<float>(),
                          idx->ascN.as<int32_t>(), d_rec_ids, d_rec_d, d_rec_n, cap);
    if (rc) return rc;
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

// from the whole worker heap (extracted ascending [nq][R], global ids): the
// result heap in pop order (flat_search.go) -> d_out_* [nq][k] without
// rescoring; with rescoring the candidates after the trim, ascending id-list
// order, as global ids d_cand_ids [nq][R] (unused slots ~0) + d_cand_n
extern "C" int wv_index_quant_finish(wv_index* idx, const uint64_t* d_asc_ids, const float* d_asc_d,
                                     const int32_t* d_asc_n, uint64_t* d_out_ids, float* d_out_d, int32_t* d_out_n,
                                     uint64_t* d_cand_ids, int32_t* d_cand_n, void* stream) {
    if (!idx || !d_asc_ids || !d_asc_d || !d_asc_n) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->qt_nq <= 0) return set_err(WV_ERR_INVALID, "quant_finish: no batch begun");
    if (idx->qt_rescore ? (!d_cand_ids || !d_cand_n) : (!d_out_ids || !d_out_d || !d_out_n))
        return set_err(WV_ERR_INVALID, "nil output buffer");
    hipStream_t s = (hipStream_t)stream;
    const int64_t nq = idx->qt_nq;
    const int R = idx->qt_R;
    if (idx->qt_form == 1) {  // searchByVectorQuantized: every worker-heap item is a candidate (ascending)
        HIPCHK(hipMemcpyAsync(d_cand_ids, d_asc_ids, (size_t)nq * R * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(d_cand_n, d_asc_n, (size_t)nq * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
        if (!stream) HIPCHK(hipStreamSynchronize(s));
        return WV_OK;
    }
    const size_t lds_f = (size_t)R * (sizeof(uint64_t) + sizeof(float)) + 16;
    if (lds_f > 64 * 1024)
        HIPCHK(hipFuncSetAttribute((const void*)k_pq_finish, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_f));
    k_pq_finish<<<(unsigned)nq, 64, lds_f, s>>>(d_asc_ids, d_asc_d, d_asc_n, idx->ident.as<int32_t>(), (int)nq, R,
                                                idx->qt_k, idx->qt_rescore, idx->id_base, d_out_ids, d_out_d, d_out_n,
                                                nullptr, d_cand_n, idx->qt_rescore ? idx->qt_trim : 0, d_cand_ids);
    HIPCHK(hipGetLastError());
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

// exact SingleDist of the candidates this shard holds (others left as they are)
extern "C" int wv_index_quant_rescore(wv_index* idx, const uint64_t* d_cand_ids, const int32_t* d_cand_n, float* d_E,
                                      void* stream) {
    if (!idx || !d_cand_ids || !d_cand_n || !d_E) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    if (idx->qt_nq <= 0) return set_err(WV_ERR_INVALID, "quant_rescore: no batch begun");
    hipStream_t s = (hipStream_t)stream;
    const int64_t nq = idx->qt_nq;
    const int R = idx->qt_R;
    const int64_t npairs = nq * R;
    const float* Qn = idx->qn.as<float>();
    const int32_t* qlist = idx->ident.as<int32_t>();
    const bool v5 = idx->variant == WV_VARIANT_AVX512;
#define WV_RS(M, V) k_rescore_ids<M, V><<<(unsigned)((npairs + 63) / 64), 64, 0, s>>>(idx->X, idx->dpad, Qn, idx->dims, d_cand_ids, d_cand_n, qlist, (int)nq, R, idx->id_base, idx->hiwater, d_E)
    switch (idx->metric) {
    case WV_METRIC_L2_SQUARED: if (v5) WV_RS(L2, AVX512); else WV_RS(L2, AVX256); break;
    case WV_METRIC_DOT: if (v5) WV_RS(DOT, AVX512); else WV_RS(DOT, AVX256); break;
    case WV_METRIC_COSINE_DOT: if (v5) WV_RS(COSINE, AVX512); else WV_RS(COSINE, AVX256); break;
    default: WV_RS(HAMMING, AVX256); break;
    }
#undef WV_RS
    HIPCHK(hipGetLastError());
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return WV_OK;
}

// the rescoring heap over the candidates: form 0 = h.rescore (hnsw/search.go:1067-1110),
// form 1 = searchByVectorQuantized's (flat/index.go:525-531, candidates ascending);
// d_E_all [world][nq][R], the entry of id from shard min(id / id_stride, world - 1)
extern "C" int wv_quant_rescore_final(int32_t device, int32_t form, int64_t nq, int32_t R, int32_t k, int32_t world,
                                      uint64_t id_stride, const uint64_t* d_cand_ids, const int32_t* d_cand_n,
                                      const float* d_E_all, uint64_t* d_out_ids, float* d_out_d, int32_t* d_out_n,
                                      void* stream) {
    HIPCHK(hipSetDevice(device));
    if (nq <= 0) return WV_OK;
    if (k <= 0 || R < k || world < 1) return set_err(WV_ERR_INVALID, "quant_rescore_final: invalid k / R / world");
    hipStream_t s = (hipStream_t)stream;
    std::vector<int32_t> id((size_t)nq);
    for (int64_t i = 0; i < nq; i++) id[i] = (int32_t)i;
    DBuf ql;
    HIPCHK(ql.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(hipMemcpyAsync(ql.p, id.data(), (size_t)nq * sizeof(int32_t), hipMemcpyHostToDevice, s));
    if (form == 1) {
        int rc = bq_final(s, nq, R, k, world, id_stride, ql.as<int32_t>(), d_cand_ids, d_cand_n, d_E_all, d_out_ids,
                          d_out_d, d_out_n, 1);
        if (rc) return rc;
    } else {
        const size_t lds_q = (size_t)(k + 1) * (sizeof(uint64_t) + sizeof(float)) + 16;
        if (lds_q > 64 * 1024)
            HIPCHK(hipFuncSetAttribute((const void*)k_pq_rescore_final, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds_q));
        k_pq_rescore_final<<<(unsigned)nq, 64, lds_q, s>>>(nullptr, d_E_all, d_cand_n, ql.as<int32_t>(), (int)nq, R, k,
                                                           0, d_out_ids, d_out_d, d_out_n, d_cand_ids, world, id_stride);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(s));  // ql is freed on return
    ql.release();
    return WV_OK;
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
int rq_init(wv_index* idx) {
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
        HIPCHK(hipMalloc(&idx->rq_meta, (size_t)idx->cap * RQ_META_B));
        HIPCHK(hipMemset(idx->rq_codes, 0, cb));
        HIPCHK(hipMemset(idx->rq_meta, 0, (size_t)idx->cap * RQ_META_B));
        if (idx->rq_bits == 1) {
            HIPCHK(hipMalloc(&idx->rq1_pm, (size_t)idx->cap * D));
            HIPCHK(hipMemset(idx->rq1_pm, 0, (size_t)idx->cap * D));
        }
    }
    return WV_OK;
}

// encode nq prepared query rows (idx->qn, normalised for cosine) into idx->rqq / rqm
int rq_encode_queries(wv_index* idx, hipStream_t s, int64_t nq) {
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
int rq_dist(wv_index* idx, hipStream_t s, const uint32_t* valid, int64_t q0, int F, int64_t ld, float* E,
                   float* bmin, const void* qcodes, const float4* qmeta) {
    const int64_t nslots = idx->hiwater;
    const float fl2 = idx->metric == WV_METRIC_L2_SQUARED ? 1.f : 0.f;
    const float fcos = idx->metric == WV_METRIC_COSINE_DOT ? 1.f : 0.f;
    if (!qcodes) qcodes = idx->rqq.p;
    if (!qmeta) qmeta = idx->rqm.as<float4>();
    dim3 grid((unsigned)((F + RQ_QPB - 1) / RQ_QPB), (unsigned)(ld / 256));
    if (idx->rq_bits == 8)
        k_rq8_dist<<<grid, 256, 0, s>>>(reinterpret_cast<const uint4*>(idx->rq_codes), idx->rq_meta, idx->rq_D, valid,
                                        nslots, reinterpret_cast<const uint4*>(qcodes), qmeta, q0, F, fl2, fcos, ld, E,
                                        bmin);
    else
        k_rq1_dist<<<grid, 256, 0, s>>>(reinterpret_cast<const uint64_t*>(idx->rq_codes), idx->cap, idx->rq_meta,
                                        idx->rq_D / 64, valid, nslots, reinterpret_cast<const uint64_t*>(qcodes), qmeta,
                                        q0, F, fl2, fcos, ld, E, bmin);
    HIPCHK(hipGetLastError());
    return WV_OK;
}

// rq-8 / rq-1 on the integer matrix cores (rq8_mfma.hip): the query
// fragments stay in VGPRs up to D = 1024; the candidate lists hold R + 2
// entries; rq-1 needs its +-1 plane
static bool rq8_route(const wv_index* idx, int R) {
    return (idx->rq_bits == 8 || (idx->rq_bits == 1 && idx->rq1_pm)) && idx->rq_mfma && idx->rq_D <= 1024 &&
           qs_R(R + 1) != 0 && idx->hiwater > 0;
}

template <int NC>
static void launch_rq8_keys(const RQ8Args& a, unsigned grid, hipStream_t s, int bits) {
    constexpr size_t lds = (size_t)rq8_nbuf(NC) * ((size_t)32 * 64 * NC + 656);  // the ring (k_rq8_keys)
    if (bits == 8) {
        if (lds > 64 * 1024)
            (void)hipFuncSetAttribute((const void*)k_rq8_keys<NC, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        k_rq8_keys<NC, 8><<<grid, 512, lds, s>>>(a);
    } else {
        if (lds > 64 * 1024)
            (void)hipFuncSetAttribute((const void*)k_rq8_keys<NC, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        k_rq8_keys<NC, 1><<<grid, 512, lds, s>>>(a);
    }
}

// exact rq-8 block minima -> candidate blocks -> exact distances of their
// rows: the ascending R-lists (ascI / ascD / ascN) of every query, oF[q] = 1
// where a tie or a NaN leaves the heap's order to the replay
static int rq8_candidates(wv_index* idx, hipStream_t s, int64_t nq, int R, const uint32_t* valid) {
    const int D = idx->rq_D, NC = D / 64;
    const int64_t nblk = (idx->hiwater + 31) / 32;
    const int RT = qs_R(R + 1);
    const int Lc = 64 * (RT - 1);
    const int64_t nq_pad = round_up(nq, 256);
    // query chunks: key rows of at most 4 GiB
    int64_t QC = std::max<int64_t>(256, ((4ll << 30) / (nblk * 4)) / 256 * 256);
    QC = std::min<int64_t>(QC, nq_pad);
    HIPCHK(idx->rq8Qp.ensure((size_t)nq_pad * D));
    HIPCHK(idx->rq8Qcs.ensure((size_t)nq_pad * sizeof(uint32_t)));
    HIPCHK(idx->rq8Qm.ensure((size_t)nq_pad * sizeof(float4)));
    HIPCHK(idx->qsKey.ensure((size_t)QC * nblk * sizeof(float)));
    HIPCHK(idx->qsCand.ensure((size_t)nq * Lc * sizeof(uint32_t)));
    HIPCHK(idx->qsNc.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(idx->oF.ensure((size_t)nq * sizeof(int32_t)));
    unsigned char* Qp = idx->rq8Qp.as<unsigned char>();
    uint32_t* Qcs = idx->rq8Qcs.as<uint32_t>();
    float4* Qm = idx->rq8Qm.as<float4>();
    HIPCHK(hipMemsetAsync(Qm, 0, (size_t)nq_pad * sizeof(float4), s));
    HIPCHK(hipMemcpyAsync(Qm, idx->rqm.p, (size_t)nq * sizeof(float4), hipMemcpyDeviceToDevice, s));
    const int bits = idx->rq_bits;
    if (bits == 8) {
        k_rq8_qprep<<<(unsigned)(nq_pad / 4), 256, 0, s>>>(idx->rqq.as<uint4>(), D, nq, nq_pad, Qp, Qcs);
    } else {
        const int64_t nt = nq_pad * (D / 16);
        k_rq1_qprep<<<(unsigned)((nt + 255) / 256), 256, 0, s>>>(idx->rqq.as<uint64_t>(), Qm, D, nq, nq_pad, Qp);
    }
    HIPCHK(hipGetLastError());
    const float fl2 = idx->metric == WV_METRIC_L2_SQUARED ? 1.f : 0.f;
    const float fcos = idx->metric == WV_METRIC_COSINE_DOT ? 1.f : 0.f;
    RQ8Args a{};
    a.codes = bits == 8 ? reinterpret_cast<const unsigned char*>(idx->rq_codes) : idx->rq1_pm;
    a.meta = idx->rq_meta;
    a.csum = rq_csum(idx);
    a.valid = valid;
    a.key = idx->qsKey.as<float>();
    a.ldk = nblk;
    a.nblk = nblk;
    a.fl2 = fl2;
    a.fcos = fcos;
    a.dbg_serial = idx->rq_serial;
    idx->rq_dbg_nq = std::min<int64_t>(QC, nq);
    idx->rq_dbg_nb = nblk;
    for (int64_t c0 = 0; c0 < nq; c0 += QC) {
        const int64_t cn = std::min<int64_t>(QC, nq - c0);
        const int64_t cpad = round_up(cn, 256);
        a.Qp = Qp + c0 * D;
        a.qmeta = Qm + c0;
        a.qcsum = Qcs + c0;
        a.nqg = (int)(cpad / 256);
        // spans: ~2048 workgroups (8 per CU), at least 16 blocks each
        int64_t nspans = std::max<int64_t>(1, std::min<int64_t>(nblk / 16, (2048 + a.nqg - 1) / a.nqg));
        const int64_t bps = (nblk + nspans - 1) / nspans;
        nspans = (nblk + bps - 1) / bps;
        a.blocks_per_span = (int)bps;
        a.nspans = (int)nspans;
        const unsigned grid = (unsigned)(a.nqg * nspans);
        const bool time_it = idx->timing && c0 == 0;
        if (time_it) HIPCHK(hipEventRecord(idx->ev0, s));
        switch (NC) {
        case 1: launch_rq8_keys<1>(a, grid, s, bits); break;
        case 2: launch_rq8_keys<2>(a, grid, s, bits); break;
        case 3: launch_rq8_keys<3>(a, grid, s, bits); break;
        case 4: launch_rq8_keys<4>(a, grid, s, bits); break;
        case 5: launch_rq8_keys<5>(a, grid, s, bits); break;
        case 6: launch_rq8_keys<6>(a, grid, s, bits); break;
        case 7: launch_rq8_keys<7>(a, grid, s, bits); break;
        case 8: launch_rq8_keys<8>(a, grid, s, bits); break;
        case 9: launch_rq8_keys<9>(a, grid, s, bits); break;
        case 10: launch_rq8_keys<10>(a, grid, s, bits); break;
        case 11: launch_rq8_keys<11>(a, grid, s, bits); break;
        case 12: launch_rq8_keys<12>(a, grid, s, bits); break;
        case 13: launch_rq8_keys<13>(a, grid, s, bits); break;
        case 14: launch_rq8_keys<14>(a, grid, s, bits); break;
        case 15: launch_rq8_keys<15>(a, grid, s, bits); break;
        default: launch_rq8_keys<16>(a, grid, s, bits); break;
        }
        HIPCHK(hipGetLastError());
        if (time_it) HIPCHK(hipEventRecord(idx->ev1, s));
        const unsigned gw = (unsigned)((cn + 3) / 4);
        uint32_t* cand = idx->qsCand.as<uint32_t>() + c0 * Lc;
        int32_t* ncand = idx->qsNc.as<int32_t>() + c0;
        int32_t* of = idx->oF.as<int32_t>() + c0;
        const size_t lq = (size_t)4 * (bits == 8 ? D : (5 * (D / 64) + 1) / 2 * 16);
        const void* qsrc = bits == 8 ? (const void*)a.Qp : idx->rqq.p;
#define WV_RQC(RTV, B)                                                                                                \
    k_rq8_cand<RTV, B><<<gw, 256, lq, s>>>(idx->rq_codes, idx->cap, idx->rq_meta, valid, idx->hiwater, qsrc, c0,       \
                                           a.qmeta, D, fl2, fcos, cand, Lc, ncand, (int)cn, R, idx->id_base,           \
                                           idx->ascI.as<uint64_t>() + c0 * R, idx->ascD.as<float>() + c0 * R,         \
                                           idx->ascN.as<int32_t>() + c0, of)
#define WV_RQ8(RTV)                                                                                                   \
    do {                                                                                                              \
        k_rq8_sel<RTV><<<gw, 256, 0, s>>>(a.key, nblk, nblk, (int)cn, R, cand, Lc, ncand, of);                        \
        if (bits == 8) WV_RQC(RTV, 8);                                                                                 \
        else WV_RQC(RTV, 1);                                                                                           \
    } while (0)
        if (RT == 2) WV_RQ8(2);
        else if (RT == 4) WV_RQ8(4);
        else if (RT == 8) WV_RQ8(8);
        else WV_RQ8(16);
#undef WV_RQ8
#undef WV_RQC
        HIPCHK(hipGetLastError());
    }
    idx->stats.mfma_launches++;
    idx->stats.last_route = WV_ROUTE_RQ8_INT8;
    return WV_OK;
}

// the R-heap replay of searchByVectorQuantized for nrep queries: every query
// (list == nullptr: asc rows by query index) or the listed ones (their codes
// compacted into groups of RQ_QPB first, asc rows by query): exact quantized
// distances + block minima (k_rq*_dist), the heap replayed in id order
// (k_replay_scan).  Query groups: multiples of RQ_QPB, two distance buffers
// of up to 16 GiB each (a quarter of the free HBM at most); group i's
// distances (stream s) overlap group i-1's replay (stream aux).
static int rq_replay(wv_index* idx, hipStream_t s, const uint32_t* valid, int R, const int32_t* list, int64_t nrep) {
    const void* qc = nullptr;
    const float4* qm = nullptr;
    if (list) {
        const int64_t nf32 = round_up(nrep, RQ_QPB);
        if (idx->rq_bits == 1) {
            const int ne = 5 * (idx->rq_D / 64);
            HIPCHK(idx->rq8Fq.ensure((size_t)nf32 * ne * sizeof(uint64_t)));
            HIPCHK(idx->rq8Fm.ensure((size_t)nf32 * sizeof(float4)));
            HIPCHK(hipMemsetAsync(idx->rq8Fq.p, 0, (size_t)nf32 * ne * sizeof(uint64_t), s));
            HIPCHK(hipMemsetAsync(idx->rq8Fm.p, 0, (size_t)nf32 * sizeof(float4), s));
            const int64_t nt = nrep * ne;
            k_rq1_gather_q<<<(unsigned)((nt + 255) / 256), 256, 0, s>>>(idx->rqq.as<uint64_t>(), idx->rqm.as<float4>(), ne,
                                                                         list, (int)nrep, idx->rq8Fq.as<uint64_t>(),
                                                                         idx->rq8Fm.as<float4>());
        } else {
            const int nch = idx->rq_D / 16;
            HIPCHK(idx->rq8Fq.ensure((size_t)nf32 * idx->rq_D));
            HIPCHK(idx->rq8Fm.ensure((size_t)nf32 * sizeof(float4)));
            HIPCHK(hipMemsetAsync(idx->rq8Fq.p, 0, (size_t)nf32 * idx->rq_D, s));
            HIPCHK(hipMemsetAsync(idx->rq8Fm.p, 0, (size_t)nf32 * sizeof(float4), s));
            const int64_t nt = nrep * nch;
            k_rq8_gather_q<<<(unsigned)((nt + 255) / 256), 256, 0, s>>>(idx->rqq.as<uint4>(), idx->rqm.as<float4>(), nch,
                                                                         list, (int)nrep, idx->rq8Fq.as<uint4>(),
                                                                         idx->rq8Fm.as<float4>());
        }
        HIPCHK(hipGetLastError());
        qc = idx->rq8Fq.p;
        qm = idx->rq8Fm.as<float4>();
    }
    const int32_t* qlist = list ? list : idx->ident.as<int32_t>();
    const int rep_by_query = list ? 1 : 0;
    idx->stats.replayed_queries += (uint64_t)nrep;
    const int64_t nslots = idx->hiwater;
    const int64_t ld = std::max<int64_t>(round_up(nslots, EBLK), EBLK);
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    const int64_t have = (int64_t)(Eb0_bytes(idx) + free_b / 4);
    const int64_t budget = std::max<int64_t>(std::min<int64_t>(16ll << 30, have), 1ll << 30);
    int64_t G = (budget / (ld * 4)) / RQ_QPB * RQ_QPB;
    G = std::max<int64_t>(RQ_QPB, std::min<int64_t>(G, round_up(nrep, RQ_QPB)));
    if (!list) idx->stats.last_group_queries = (uint64_t)std::min<int64_t>(G, nrep);
    int rc = ensure_aux(idx);
    if (rc) return rc;
    DBuf* Eb[2] = {&idx->rE, &idx->rE2};
    DBuf* Bb[2] = {&idx->rB, &idx->rB2};
    for (int b = 0; b < 2; b++) {
        HIPCHK(Eb[b]->ensure((size_t)G * ld * sizeof(float)));
        HIPCHK(Bb[b]->ensure((size_t)G * (ld / EBLK) * sizeof(float)));
    }
    int64_t gi = 0;
    for (int64_t g0 = 0; g0 < nrep; g0 += G, gi++) {
        const int F = (int)std::min<int64_t>(G, nrep - g0);
        const int b = (int)(gi & 1);
        if (gi >= 2) HIPCHK(hipStreamWaitEvent(s, idx->evr[b], 0));
        const bool time_it = idx->timing && g0 == 0 && !list;
        if (time_it) HIPCHK(hipEventRecord(idx->ev0, s));
        rc = rq_dist(idx, s, valid, g0, F, ld, Eb[b]->as<float>(), Bb[b]->as<float>(), qc, qm);
        if (rc) return rc;
        if (time_it) HIPCHK(hipEventRecord(idx->ev1, s));
        HIPCHK(hipEventRecord(idx->evd[b], s));
        HIPCHK(hipStreamWaitEvent(idx->aux, idx->evd[b], 0));
        // asc rows by list position (every query, in order) or by query
        const int64_t ao = rep_by_query ? 0 : g0;
        HIPCHK(launch_replay_scan(R, (unsigned)F, idx->aux, Eb[b]->as<float>(), Bb[b]->as<float>(), valid, nslots, ld,
                                  qlist + g0, F, R, idx->id_base, nullptr, nullptr, nullptr, 1, rep_by_query, R,
                                  idx->ascI.as<uint64_t>() + ao * R, idx->ascD.as<float>() + ao * R,
                                  idx->ascN.as<int32_t>() + ao, 0, 0, nullptr, nullptr, nullptr, 0));
        HIPCHK(hipEventRecord(idx->evr[b], idx->aux));
    }
    // join: the rescoring on s reads every group's heap
    for (int b = 0; b < 2 && b < gi; b++) HIPCHK(hipStreamWaitEvent(s, idx->evr[b], 0));
    return WV_OK;
}

// the listed queries' R-heaps replayed from the MFMA route's exact 32-row
// minima (k_rq8_replay), when the last rq8_candidates kept every query's keys
// (one query chunk); else the distance-matrix replay (rq_replay)
static int rq8_replay_list(wv_index* idx, hipStream_t s, const uint32_t* valid, int R, const int32_t* list,
                           int64_t n, int64_t nq) {
    if (idx->rq_dbg_nq != nq || idx->rq_serial == 8) return rq_replay(idx, s, valid, R, list, n);
    idx->stats.replayed_queries += (uint64_t)n;
    const int D = idx->rq_D;
    const int64_t nblk = idx->rq_dbg_nb;
    const float fl2 = idx->metric == WV_METRIC_L2_SQUARED ? 1.f : 0.f;
    const float fcos = idx->metric == WV_METRIC_COSINE_DOT ? 1.f : 0.f;
    const size_t lds = rq8_replay_lds(R, rq_query_lds_u4(idx->rq_bits, D));
    const bool b8 = idx->rq_bits == 8;
    const void* fn = b8 ? (const void*)k_rq8_replay<8> : (const void*)k_rq8_replay<1>;
    if (lds > 64 * 1024) HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const void* qsrc = b8 ? (const void*)idx->rq8Qp.p : idx->rqq.p;
#define WV_RQR(B)                                                                                                  \
    k_rq8_replay<B><<<(unsigned)n, 512, lds, s>>>(idx->qsKey.as<float>(), nblk, nblk, idx->rq_codes, idx->cap,      \
                                                 idx->rq_meta, valid, idx->hiwater, qsrc, 0, idx->rq8Qm.as<float4>(), \
                                                 D, fl2, fcos, list, (int)n, R, idx->id_base,                      \
                                                 idx->ascI.as<uint64_t>(), idx->ascD.as<float>(),                  \
                                                 idx->ascN.as<int32_t>())
    if (b8) WV_RQR(8);
    else WV_RQR(1);
#undef WV_RQR
    HIPCHK(hipGetLastError());
    return WV_OK;
}

// flat.searchByVectorQuantized (flat/index.go:460-532) for rq-8 / rq-1: the
// worker R-heap fed in id order (addResult == insertToHeap, :470-487),
// extracted ascending (reversed pop order), fp32 rescoring of those
// candidates (k_rescore_ids) and the k-heap fed in pop order (k_bq_final,
// asc = 1).  rq-8 with rq8_route: the R-lists come from rq8_candidates and only
// its flagged queries are replayed; otherwise every query: exact quantized
// distances + block minima (k_rq*_dist) and the heap replayed in id order
// (k_replay_scan).
int search_rq(wv_index* idx, hipStream_t s, const float* d_qraw, int64_t nq, int64_t qd, int k,
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
    HIPCHK(idx->ident.ensure((size_t)nq * sizeof(int32_t)));
    {
        std::vector<int32_t> id((size_t)nq);
        for (int64_t i = 0; i < nq; i++) id[i] = (int32_t)i;
        HIPCHK(hipMemcpyAsync(idx->ident.p, id.data(), (size_t)nq * sizeof(int32_t), hipMemcpyHostToDevice, s));
    }
    HIPCHK(idx->ascI.ensure((size_t)nq * R * sizeof(uint64_t)));
    HIPCHK(idx->ascD.ensure((size_t)nq * R * sizeof(float)));
    HIPCHK(idx->ascN.ensure((size_t)nq * sizeof(int32_t)));
    HIPCHK(idx->candE.ensure((size_t)nq * R * sizeof(float)));
    const bool mfma = rq8_route(idx, R);
    idx->bq_nq = nq;
    idx->bq_R = R;
    if (!mfma) {
        rc = rq_replay(idx, s, valid, R, nullptr, nq);
        if (rc) return rc;
        rc = bq_rescore(idx, s, idx->ascI.as<uint64_t>(), idx->ascN.as<int32_t>(), idx->candE.as<float>());
        if (rc) return rc;
    } else {
        rc = rq8_candidates(idx, s, nq, R, valid);
        if (rc) return rc;
        idx->stats.last_group_queries = (uint64_t)nq;
        // oF: 1 = replayed, 2 = decided by the rescored distances (k_rq_tiecheck:
        // 3 replayed, else 0).  Every row is rescored first (replayed rows hold
        // no candidates yet), then the replayed queries' rows once more.
        rc = bq_rescore(idx, s, idx->ascI.as<uint64_t>(), idx->ascN.as<int32_t>(), idx->candE.as<float>());
        if (rc) return rc;
        k_rq_tiecheck<<<(unsigned)((nq + 3) / 4), 256, 0, s>>>(idx->candE.as<float>(), idx->ascN.as<int32_t>(), (int)nq,
                                                               R, k, idx->oF.as<int32_t>());
        HIPCHK(idx->qsList.ensure((size_t)nq * sizeof(int32_t)));
        HIPCHK(idx->flCtr.ensure(2 * sizeof(uint32_t)));
        HIPCHK(hipMemsetAsync(idx->flCtr.p, 0, 2 * sizeof(uint32_t), s));
        int32_t* list = idx->qsList.as<int32_t>();
        k_flag_list<<<(unsigned)((nq + 255) / 256), 256, 0, s>>>(idx->oF.as<int32_t>(), (int)nq, list,
                                                                  idx->flCtr.as<uint32_t>(), 0);
        HIPCHK(hipGetLastError());
        uint32_t cnt[2] = {0, 0};
        HIPCHK(hipMemcpyAsync(cnt, idx->flCtr.p, sizeof(cnt), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (cnt[1] > 0) {
            rc = rq8_replay_list(idx, s, valid, R, list, cnt[1], nq);
            if (rc) return rc;
            const int64_t np = (int64_t)cnt[1] * R;
            const bool v5 = idx->variant == WV_VARIANT_AVX512;
#define WV_RSL(M, V)                                                                                                 \
    k_rescore_list<M, V><<<(unsigned)((np + 63) / 64), 64, 0, s>>>(idx->X, idx->dpad, idx->qn.as<float>(), idx->dims,  \
                                                                   idx->ascI.as<uint64_t>(), idx->ascN.as<int32_t>(), \
                                                                   list, (int)cnt[1], R, idx->id_base, idx->hiwater,  \
                                                                   idx->candE.as<float>())
            switch (idx->metric) {
            case WV_METRIC_L2_SQUARED: if (v5) WV_RSL(L2, AVX512); else WV_RSL(L2, AVX256); break;
            case WV_METRIC_DOT: if (v5) WV_RSL(DOT, AVX512); else WV_RSL(DOT, AVX256); break;
            default: if (v5) WV_RSL(COSINE, AVX512); else WV_RSL(COSINE, AVX256); break;
            }
#undef WV_RSL
            HIPCHK(hipGetLastError());
        }
    }
    const int32_t* qlist = idx->ident.as<int32_t>();
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
    if (idx->rq_bits == 1 && idx->rq_serial == 16 && idx->rq1_pm) {  // debug: the +-1 plane, de-tiled [n][D]
        const int64_t ntile = (n + 255) / 256;
        std::vector<uint8_t> tiled((size_t)ntile * 256 * D);
        if (n) HIPCHK(hipMemcpy(tiled.data(), idx->rq1_pm, tiled.size(), hipMemcpyDeviceToHost));
        const int nch = D / 16;
        for (int64_t s2 = 0; s2 < n; s2++)
            for (int ch = 0; ch < nch; ch++)
                memcpy((uint8_t*)out + (size_t)s2 * D + ch * 16,
                       &tiled[(size_t)rq_tile_u4(s2, ch, nch) * 16], 16);
        return WV_OK;
    }
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
                memcpy(c + 16 + ch * 16, &tiled[(size_t)rq_tile_u4(s, ch, nch) * 16], 16);
            for (int j = 0; j < D; j++) c[16 + j] ^= 0x80;  // stored offset by 128
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
