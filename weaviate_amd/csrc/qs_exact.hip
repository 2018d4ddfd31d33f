// qs_exact.hip -- the block-key path's exact pass: reference-order fp32
// distances of the candidate blocks' rows and the verified top-(k+1)
// (k_blk_exact), and the block-major distance pass that feeds it
// (k_exact_bm) (see rt_index.h for the unit split).
#include "rt_index.h"

// k_blk_exact<RV, METRIC, VARIANT> over the queries of one chunk (list ==
// nullptr) or the listed ones; eb/ldE: block-major distances, capv: the per
// query cap of the (k+1)-th exact distance (nullptr: uncapped)
void launch_blk_exact(wv_index* idx, hipStream_t s, int RV, int metric, bool v5, const float* Qn,
                      const uint32_t* valid, int cn, int k, int kout, uint64_t* o_ids, float* o_d, int32_t* o_n,
                      int32_t* flags, const int32_t* list, const uint32_t* cnt, const float* eb, int64_t ldE,
                      const float* capv, const float4* qinfo, const Q8Filter* q8f, const uint32_t* fmask) {
    // the capped pass filters rows by their bf16-plane bound (k_blk_exact);
    // gacc_r: plane_dot's two-way accumulation of dpb products
    const uint16_t* Xb = idx->qs_planes && idx->exact_filter ? idx->Xb : nullptr;
    const float gd = (float)gamma_n(idx->dpb + 8), gacc_r = (float)gamma_n(idx->dpb + 2);
    // int8 keys: the row bound from the int8 plane (q8f), else the bf16 plane
    Q8Filter f8{};
    if (q8f && idx->exact_filter && (Xb || idx->q8_only)) f8 = *q8f;
#define WV_EXR(RV, M, V)                                                                                             \
    do {                                                                                                             \
        if (eb) k_blk_exact<RV, M, V, true><<<(unsigned)cn, 256, 0, s>>>(idx->X, idx->dpad, valid, idx->hiwater, Qn, idx->dims, idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(), cn, k, kout, idx->id_base, o_ids, o_d, o_n, flags, list, cnt, eb, ldE, capv, qinfo, Xb, idx->dpb, idx->xnorm2, idx->qsmax, idx->d_maxn2, gd, gacc_r, f8, nullptr, idx->cur_vq, idx->cur_tq, idx->qsEps.as<float>()); \
        else k_blk_exact<RV, M, V, false><<<(unsigned)cn, 256, 0, s>>>(idx->X, idx->dpad, valid, idx->hiwater, Qn, idx->dims, idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(), cn, k, kout, idx->id_base, o_ids, o_d, o_n, flags, list, cnt, nullptr, 0, capv, qinfo, Xb, idx->dpb, idx->xnorm2, idx->qsmax, idx->d_maxn2, gd, gacc_r, f8, fmask, idx->cur_vq, idx->cur_tq, idx->qsEps.as<float>()); \
    } while (0)
#define WV_EXM(RV)                                                          \
    switch (metric) {                                                       \
    case L2: if (v5) WV_EXR(RV, L2, AVX512); else WV_EXR(RV, L2, AVX256); break;   \
    case DOT: if (v5) WV_EXR(RV, DOT, AVX512); else WV_EXR(RV, DOT, AVX256); break; \
    default: if (v5) WV_EXR(RV, COSINE, AVX512); else WV_EXR(RV, COSINE, AVX256); break; \
    }
    if (RV == 2) { WV_EXM(2); } else if (RV == 4) { WV_EXM(4); } else if (RV == 8) { WV_EXM(8); }
    else {  // k + 1 <= 960 / 1984 / 4032: never block-major (9-bit list positions)
#define WV_EXB(RB, M, V) k_blk_exact<RB, M, V, false><<<(unsigned)cn, 256, 0, s>>>(idx->X, idx->dpad, valid, idx->hiwater, Qn, idx->dims, idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(), cn, k, kout, idx->id_base, o_ids, o_d, o_n, flags, list, cnt, nullptr, 0, capv, qinfo, Xb, idx->dpb, idx->xnorm2, idx->qsmax, idx->d_maxn2, gd, gacc_r, f8, nullptr, idx->cur_vq, idx->cur_tq, idx->qsEps.as<float>())
#define WV_EXBM(RB)                                                                     \
        switch (metric) {                                                               \
        case L2: if (v5) WV_EXB(RB, L2, AVX512); else WV_EXB(RB, L2, AVX256); break;    \
        case DOT: if (v5) WV_EXB(RB, DOT, AVX512); else WV_EXB(RB, DOT, AVX256); break; \
        default: if (v5) WV_EXB(RB, COSINE, AVX512); else WV_EXB(RB, COSINE, AVX256); break; \
        }
        if (RV == 16) { WV_EXBM(16); } else if (RV == 32) { WV_EXBM(32); } else { WV_EXBM(64); }
#undef WV_EXBM
#undef WV_EXB
    }
#undef WV_EXM
#undef WV_EXR
}

// k_q8_filt_bm<METRIC>: the int8 row filter block-major (survivor masks of
// every listing, fmask [cn][L]); the capped exact pass reads them
void launch_q8_filt_bm(wv_index* idx, hipStream_t s, int metric, const Q8Filter& f, const float* xn2,
                       const uint32_t* valid, int64_t nb, int L, const float* capv, const float4* qinfo, float gd,
                       uint32_t* fmask) {
    const size_t lds = (size_t)(f.dpb8 >> 5) * 1024 + (size_t)8 * (f.dpb8 >> 5) * 32;
#define WV_FB(M) k_q8_filt_bm<M><<<(unsigned)nb, 256, lds, s>>>(f, xn2, valid, idx->hiwater, idx->bmOff.as<uint32_t>(), idx->bmPairs.as<uint32_t>(), L, capv, qinfo, idx->d_maxn2, gd, fmask)
    switch (metric) {
    case L2: WV_FB(L2); break;
    case DOT: WV_FB(DOT); break;
    default: WV_FB(COSINE); break;
    }
#undef WV_FB
}

// k_exact_bm<METRIC, VARIANT>: every listed (query, row) distance of each
// candidate block, one workgroup per block (the block staged in LDS once)
void launch_exact_bm(wv_index* idx, hipStream_t s, int metric, bool v5, const float* Qn, int64_t nb, size_t bm_lds,
                     int64_t ldE) {
#define WV_BM(M, V) k_exact_bm<M, V><<<(unsigned)nb, 256, bm_lds, s>>>(idx->X, idx->dpad, idx->hiwater, Qn, idx->dims, idx->bmOff.as<uint32_t>(), idx->bmPairs.as<uint32_t>(), ldE, idx->bmE.as<float>())
    switch (metric) {
    case L2: if (v5) WV_BM(L2, AVX512); else WV_BM(L2, AVX256); break;
    case DOT: if (v5) WV_BM(DOT, AVX512); else WV_BM(DOT, AVX256); break;
    default: if (v5) WV_BM(COSINE, AVX512); else WV_BM(COSINE, AVX256); break;
    }
#undef WV_BM
}
