// qs_replay.hip -- the block-key bounded heap replays (k_rp_bounds / k_rp_exact
// / k_rp_heap pooled form, k_blk_replay_par, k_blk_replay), launched for the
// flagged queries of a block-key search and for the cross-shard replays (see
// rt_index.h for the unit split).
#include "rt_index.h"

// the pooled block-key replay (k_rp_*) serves this k and key row length
// (the only block-key form that can record insertions)
bool blk_pooled(const wv_index* idx, int k, int64_t nb) {
    const int64_t nch = (nb + RP_CH - 1) / RP_CH;
    return k < 448 && nch <= RP_MAXCH && ((idx->replay_par == 2 && k < 64) || idx->replay_par == 3);
}

int launch_blk_replay(wv_index* idx, hipStream_t s, const float* key, int64_t ldk, int64_t nb, const float* eps,
                             const float4* qinfo, const uint32_t* valid, const float* Qn, const int32_t* list,
                             const uint32_t* counters, int nlist, int64_t max_list, int k, int kout, uint64_t* oi,
                             float* od, int32_t* on, const uint64_t* in_i, const float* in_d, const int32_t* in_n,
                             int extract, int by_list, uint64_t* rec_i, float* rec_d, int32_t* rec_n, int rec_cap) {
    const int metric = idx->metric == WV_METRIC_L2_SQUARED ? L2 : idx->metric == WV_METRIC_DOT ? DOT : COSINE;
    const bool v5 = idx->variant == WV_VARIANT_AVX512;
    const int64_t nch = (nb + RP_CH - 1) / RP_CH;
    if (max_list <= 0) return WV_OK;
    // pooled form by default for k < 64 (few flagged queries, latency-bound);
    // many flagged queries with large k (integer data, C2) replay faster in the
    // one-wave kernel, which visits only blocks under the true heap top
    const int RS = k < 64 ? 2 : k < 192 ? 4 : k < 448 ? 8 : 0;
    // per-query allow bitmaps (cur_vq): the pooled and the 8-wave forms bound
    // the heap top by block upper bounds A + eps, which hold for a block with a
    // row of the keys' row set (the union) but not necessarily one of the
    // query's own; the one-wave replay prunes by its true heap top only
    const bool ub_ok = idx->cur_vq == 0 || idx->cur_pqk;  // per-query keys bound the query's own rows
    // a few listed queries of a small batch, counted on the device (most such
    // calls list no query): the one-launch 8-wave form instead of the pooled
    // form's three launches.  A host list (counters NULL: the cross-shard
    // replay's flagged queries, every one of which replays) takes the pooled
    // form: 9 flagged C3 queries on a 1.25M-row shard 2.8 -> 0.5 ms
    const bool few = counters && max_list <= idx->rp_few && !rec_i && k < 64 && nch <= RP_MAXCH && idx->replay_par;
    if (ub_ok && !few && blk_pooled(idx, k, nb)) {
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
#define WV_RPB(RSV, M) k_rp_bounds<RSV, M><<<(unsigned)g1, 64 * rp_bounds_nw(RSV), 0, s>>>(key, ldk, nb, eps, qinfo, list, counters, nlist, k, in_d, in_n, idx->qsScratch.as<float>(), idx->rpBlk.as<uint32_t>(), idx->rpLb.as<float>(), idx->rpQ.as<int32_t>(), idx->rpCtr.as<uint32_t>(), pool_cap, idx->rpOff.as<int32_t>(), idx->rpTot.as<int32_t>(), by_list)
#define WV_RPBS(M) do { if (RS == 2) WV_RPB(2, M); else if (RS == 4) WV_RPB(4, M); else WV_RPB(8, M); } while (0)
        switch (metric) {
        case L2: WV_RPBS(L2); break;
        case DOT: WV_RPBS(DOT); break;
        default: WV_RPBS(COSINE); break;
        }
#undef WV_RPBS
#undef WV_RPB
        HIPCHK(hipGetLastError());
#define WV_RPE(M, V) k_rp_exact<M, V><<<1024, 256, 0, s>>>(idx->X, idx->dpad, valid, idx->hiwater, Qn, idx->dims, list, idx->rpBlk.as<uint32_t>(), idx->rpLb.as<float>(), idx->rpQ.as<int32_t>(), idx->rpCtr.as<uint32_t>(), pool_cap, idx->rpE.as<float>(), idx->rpVm.as<uint32_t>(), idx->cur_vq)
        switch (metric) {
        case L2: if (v5) WV_RPE(L2, AVX512); else WV_RPE(L2, AVX256); break;
        case DOT: if (v5) WV_RPE(DOT, AVX512); else WV_RPE(DOT, AVX256); break;
        default: if (v5) WV_RPE(COSINE, AVX512); else WV_RPE(COSINE, AVX256); break;
        }
#undef WV_RPE
        HIPCHK(hipGetLastError());
        const size_t hlds = (size_t)k * (sizeof(uint64_t) + sizeof(float)) + 64 * sizeof(float) + RPW * 32 * sizeof(float) + 8 + (RPW / 2) * sizeof(uint64_t) + 16;
        const int64_t g3 = std::min<int64_t>(max_list, 2048);
#define WV_RPH(M, V)                                                                                            \
    do {                                                                                                        \
        if (hlds > 64 * 1024) HIPCHK(hipFuncSetAttribute((const void*)k_rp_heap<M, V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)hlds)); \
        k_rp_heap<M, V><<<(unsigned)g3, 64, hlds, s>>>(key, ldk, nb, eps, qinfo, idx->X, idx->dpad, valid, idx->hiwater, Qn, idx->dims, list, counters, nlist, k, kout, idx->id_base, oi, od, on, in_i, in_d, in_n, extract, by_list, idx->rpBlk.as<uint32_t>(), idx->rpLb.as<float>(), idx->rpE.as<float>(), idx->rpVm.as<uint32_t>(), idx->rpOff.as<int32_t>(), idx->rpTot.as<int32_t>(), rec_i, rec_d, rec_n, rec_cap, idx->cur_vq); \
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
    if (ub_ok && k < 64 && nch <= RP_MAXCH && idx->replay_par) {
        const int64_t grid = std::min<int64_t>(max_list, 256);
        HIPCHK(idx->qsScratch.ensure((size_t)grid * nch * 64 * sizeof(float)));
#define WV_RPP(M, V) k_blk_replay_par<M, V><<<(unsigned)grid, 512, 0, s>>>(key, ldk, nb, eps, qinfo, idx->X, idx->dpad, valid, idx->hiwater, Qn, idx->dims, list, counters, nlist, k, kout, idx->id_base, oi, od, on, in_i, in_d, in_n, extract, by_list, idx->qsScratch.as<float>(), idx->cur_vq)
        switch (metric) {
        case L2: if (v5) WV_RPP(L2, AVX512); else WV_RPP(L2, AVX256); break;
        case DOT: if (v5) WV_RPP(DOT, AVX512); else WV_RPP(DOT, AVX256); break;
        default: if (v5) WV_RPP(COSINE, AVX512); else WV_RPP(COSINE, AVX256); break;
        }
#undef WV_RPP
        HIPCHK(hipGetLastError());
        return WV_OK;
    }
    // row filter from the bf16 planes (block-key indexes): gacc_r bounds the
    // accumulation error of k_blk_replay's two-way per-lane sum of dpb products
    const uint16_t* Xb = idx->qs_planes ? idx->Xb : nullptr;
    const float gd = (float)gamma_n(idx->dpb + 8), gacc_r = (float)gamma_n(idx->dpb + 2);
    const size_t rlds = packed_replay_lds(k) + 16 * 64 * sizeof(float) + (size_t)idx->dpb * sizeof(float);
    if (rlds > 160 * 1024) return set_err(WV_ERR_UNSUPPORTED, "k %d too large for the replay heap", k);
#define WV_RP(M, V)                                                                                             \
    do {                                                                                                        \
        if (rlds > 64 * 1024) { HIPCHK(hipFuncSetAttribute((const void*)k_blk_replay<M, V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)rlds)); HIPCHK(hipFuncSetAttribute((const void*)k_blk_replay<M, V, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)rlds)); } \
        if (idx->replay_dbg) k_blk_replay<M, V, 1><<<(unsigned)max_list, 64, rlds, s>>>(key, ldk, nb, eps, qinfo, idx->X, idx->dpad, valid, idx->hiwater, Qn, idx->dims, list, counters, nlist, k, kout, idx->id_base, oi, od, on, in_i, in_d, in_n, extract, by_list, Xb, idx->dpb, idx->xnorm2, idx->qsmax, idx->d_maxn2, gd, gacc_r, idx->cur_vq); \
        else k_blk_replay<M, V><<<(unsigned)max_list, 64, rlds, s>>>(key, ldk, nb, eps, qinfo, idx->X, idx->dpad, valid, idx->hiwater, Qn, idx->dims, list, counters, nlist, k, kout, idx->id_base, oi, od, on, in_i, in_d, in_n, extract, by_list, Xb, idx->dpb, idx->xnorm2, idx->qsmax, idx->d_maxn2, gd, gacc_r, idx->cur_vq); \
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

