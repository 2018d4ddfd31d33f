// qs_runtime.hip -- the block-key exact search (search_qs), its bounded heap
// replays, the sharded two-phase search and the cross-shard replay / merge
// entry points (see rt_index.h for the unit split).
#include "rt_index.h"

// candidate-list rows R (L = 64 (R - 1) blocks, a power-of-two bitonic width
// 64 R): k + 1 <= 960 stays on the block-key path
int qs_R(int k) { return k + 1 <= 64 ? 2 : k + 1 <= 192 ? 4 : k + 1 <= 448 ? 8 : k + 1 <= 960 ? 16 : 0; }
// the single-index search goes further: 1984- and 4032-block lists (k + 1 <= 4032)
int qs_R_flat(int k) {
    const int r = qs_R(k);
    return r ? r : k + 1 <= 1984 ? 32 : k + 1 <= 4032 ? 64 : 0;
}

// the candidate lists (cand [cn][L], ncand, unflagged queries) inverted per
// 32-row block: bmOff [nb + 1] offsets of bmPairs (query << 9 | list position).
// bmCnt is all-zero between batches (k_inv_scatter counts it down); a new,
// regrown (the allocator may hand back the same address) or never-completed
// buffer is zeroed once.
int invert_lists(wv_index* idx, hipStream_t s, const uint32_t* cand, const int32_t* ncand, const int32_t* flags,
                 int64_t cn, int L, int64_t nb) {
    HIPCHK(idx->bmCnt.ensure((size_t)nb * sizeof(uint32_t)));
    HIPCHK(idx->bmOff.ensure((size_t)(nb + 1) * sizeof(uint32_t)));
    HIPCHK(idx->bmPairs.ensure((size_t)cn * L * sizeof(uint32_t)));
    if (idx->bmCnt_zp != idx->bmCnt.p || idx->bmCnt_zb != idx->bmCnt.bytes)
        HIPCHK(hipMemsetAsync(idx->bmCnt.p, 0, idx->bmCnt.bytes, s));
    idx->bmCnt_zp = nullptr;
    const unsigned gw = (unsigned)((cn + 3) / 4);
    k_inv_count<<<gw, 256, 0, s>>>(cand, ncand, flags, (int)cn, L, idx->bmCnt.as<uint32_t>());
    const unsigned nparts = (unsigned)((nb + INV_CHUNK - 1) / INV_CHUNK);
    HIPCHK(idx->bmPart.ensure((size_t)nparts * sizeof(uint32_t)));
    k_inv_part<<<nparts, 1024, 0, s>>>(idx->bmCnt.as<uint32_t>(), nb, idx->bmPart.as<uint32_t>());
    k_inv_scan<<<nparts, 1024, 0, s>>>(idx->bmCnt.as<uint32_t>(), nb, idx->bmPart.as<uint32_t>(),
                                       idx->bmOff.as<uint32_t>());
    k_inv_scatter<<<gw, 256, 0, s>>>(cand, ncand, flags, (int)cn, L, idx->bmOff.as<uint32_t>(),
                                     idx->bmCnt.as<uint32_t>(), idx->bmPairs.as<uint32_t>());
    HIPCHK(hipGetLastError());
    idx->bmCnt_zp = idx->bmCnt.p;
    idx->bmCnt_zb = idx->bmCnt.bytes;
    return WV_OK;
}

// the int8 block-key pass (k_q8_blockkey, 512 <= dpb8 <= 1536) over a.nslots
// ring slots for a.nqg 256-query groups, spans chosen as search_qs does
// (XCD-aware groups, 4 GiB span planes, whole rounds of workgroups)
int launch_q8_keys(wv_index* idx, hipStream_t s, Q8Args a, int dpb8, bool l2) {
    const int NC8 = dpb8 / 64;
    const int RB = dpb8 <= 768 ? 2 : 1;
    int64_t nspans = 256 / std::gcd(256, a.nqg);
    while ((int64_t)a.nqg * nspans < 256) nspans *= 2;
    if (idx->spans_opt > 0) nspans = idx->spans_opt;
    const int64_t max_sps = ((1ll << 32) - 2 * 256ll * dpb8) / ((int64_t)RB * 32 * dpb8);
    nspans = std::max<int64_t>(nspans, (a.nslots + max_sps - 1) / max_sps);
    if (idx->spans_opt <= 0) {
        const int64_t unit = 256 / std::gcd(256, a.nqg);
        nspans = (nspans + unit - 1) / unit * unit;
    }
    nspans = std::max<int64_t>(1, std::min<int64_t>(nspans, a.nslots));
    const int64_t sps = (a.nslots + nspans - 1) / nspans;
    a.slots_per_span = (int)sps;
    a.nspans = (int)((a.nslots + sps - 1) / sps);
    const size_t lds = (size_t)3 * RB * 2 * NC8 * 1024 + 1024 + (l2 ? (size_t)8 * 4 * RB * 128 : 0);
    dim3 grid((unsigned)((int64_t)a.nqg * a.nspans));
#define WV_Q8K(NCV, RBV, L2V)                                                                                  \
    do {                                                                                                       \
        HIPCHK(hipFuncSetAttribute((const void*)k_q8_blockkey<NCV, RBV, L2V, false, false, 1>,                 \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                     \
        k_q8_blockkey<NCV, RBV, L2V, false, false, 1><<<grid, 512, lds, s>>>(a);                                \
    } while (0)
#define WV_Q8KN(L2V)                                   \
    switch (NC8) {                                     \
    case 8: WV_Q8K(8, 2, L2V); break;                  \
    case 10: WV_Q8K(10, 2, L2V); break;                \
    case 12: WV_Q8K(12, 2, L2V); break;                \
    case 16: WV_Q8K(16, 1, L2V); break;                \
    case 20: WV_Q8K(20, 1, L2V); break;                \
    case 24: WV_Q8K(24, 1, L2V); break;                \
    default: return set_err(WV_ERR_UNSUPPORTED, "int8 keys: plane width %d", dpb8); \
    }
    if (l2) { WV_Q8KN(true); } else { WV_Q8KN(false); }
#undef WV_Q8KN
#undef WV_Q8K
    HIPCHK(hipGetLastError());
    return WV_OK;
}

// phase 0: the whole search.  Sharded two-phase form (mode 1, one query chunk):
// phase 1 = block keys + local candidate selection, topA [nq][k+1] = this
// shard's k+1 smallest block-key A values (eps in idx->qsEps); phase 2 = the
// global threshold from every shard's topA / eps (gA [W][nq][k+1], gE [W][nq],
// k_blk_gthresh), exact distances, overflow pass.
// per-query masked keys serve this index's multi-allow batches (the paired
// int8 dot / cosine key kernel; see search_qs)
bool pqa_keys_route(const wv_index* idx) {
    const bool q8 = idx->q8_planes && (idx->q8_opt || idx->q8_only);
    return idx->pqa_keys && q8 && !idx->q8_only && idx->dpb8 <= 768 && idx->metric != WV_METRIC_L2_SQUARED &&
           !idx->q8_stag && idx->q8_shape != 32 && idx->sel_dbg <= 0;
}

int search_qs(wv_index* idx, hipStream_t s, int64_t nq, int k, int mode, const uint32_t* valid,
                     uint64_t* o_ids, float* o_d, int32_t* o_n, int32_t* o_flags, int phase,
                     float* topA, const float* gA, const float* gE, int W) {
    const int kout = mode == 1 ? k + 1 : k;
    const int NK = idx->dpb / 16;
    // int8 block keys (q8_kernels.hip): NC 64-column chunks per block, RB8 blocks per ring slot
    // (above 1536 dims the int8 planes are the only ones: k_q8_blockkey_cp, 128-query groups)
    const bool q8 = idx->q8_planes && (idx->q8_opt || idx->q8_only);
    const bool q8cp = q8 && idx->q8_only;
    const bool q8wide = q8cp && idx->dpb8 > Q8_MAX_DPB;  // NP = dpb8 / 1024 column parts, 64-query groups
    const int NC8 = idx->dpb8 / 64;
    const int RB8 = idx->dpb8 <= 768 ? 2 : 1;
    const int RB = q8 ? RB8 : qs_rb(NK);
    const bool pqa = idx->pqa_valid != nullptr;
    // per-query keys (option pqa_keys, int8 paired dot / cosine keys): the key
    // pass masks each query's rows with its own bitmap (k_q8_blockkey<..,
    // MASK>), so every key bounds the query's own rows and the plain select,
    // 2-eps proof and bounded replay apply; otherwise (pqs) the union's keys with
    // the per-query deeper thresholds below
    const bool pqk = pqa && pqa_keys_route(idx);
    const bool pqs = pqa && !pqk;
    int R = qs_R_flat(k);
    if (q8) {  // the int8 bound is wider: 448-block lists (option q8_R; C3: ~110 candidate blocks
               // per query, R = 4 sent a few percent to the overflow pass, profiles/r04_c3ab1_*)
        if (idx->q8_R > 0) R = std::max(R, idx->q8_R);
        else R = std::max(R, 8);
    }
    if (pqs) R = std::max(R, idx->pqa_R);  // per-query lists on the union's keys: deeper thresholds (k_blk_select mq)
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
    // 448: the overflow pass; 960: per-query lists' second pass
    HIPCHK(idx->qsCand.ensure((size_t)qc * std::max(L, idx->pqa_valid ? 960 : 448) * sizeof(uint32_t)));
    HIPCHK(idx->qsNc.ensure((size_t)qc * sizeof(int32_t)));
    HIPCHK(idx->qsEps.ensure((size_t)qc * sizeof(float)));
    if (q8) {
        HIPCHK(idx->q8Qb.ensure((size_t)qc * idx->dpb8));
        HIPCHK(idx->q8Scale.ensure((size_t)qc * sizeof(float)));
        HIPCHK(idx->q8Info.ensure((size_t)qc * sizeof(float4)));
    }
    HIPCHK(idx->qsCap.ensure((size_t)qc * sizeof(float)));
    HIPCHK(idx->qsList.ensure((size_t)2 * qc * sizeof(int32_t)));
    if (!o_flags || phase) HIPCHK(idx->qsFlags.ensure((size_t)qc * sizeof(int32_t)));
    if (phase && qc < nq) return set_err(WV_ERR_UNSUPPORTED, "two-phase shard search: batch exceeds one query chunk");
    // per-query allow bitmaps (wv_index_search_by_vector_batch_multi_allow):
    // `valid` is their union (the block keys are lower bounds over it, so over
    // each query's own rows too); the exact pass and the replays read query
    // q's bitmap, and k_blk_exact proves completeness against the select's T
    if (pqa && (phase != 0 || mode != 0)) return set_err(WV_ERR_UNSUPPORTED, "per-query allow lists: top-k mode only");
    struct PqaScope {
        wv_index* i;
        ~PqaScope() { i->cur_vq = 0; i->cur_tq = nullptr; i->cur_pqk = false; }
    } pqa_scope{idx};
    // the select's completeness bounds: per-query lists, and lists whose
    // threshold the select lowered (phase 0 only: the sharded phases keep the
    // 2-eps argument their global threshold relies on)
    HIPCHK(idx->qsT.ensure((size_t)qc * sizeof(float)));
    float* t_sel = (pqs || (phase == 0 && idx->sel_lower)) ? idx->qsT.as<float>() : nullptr;
    const size_t rlds = packed_replay_lds(k) + 16 * 64 * sizeof(float) + (size_t)idx->dpb * sizeof(float);
    if (mode == 0 && rlds > 160 * 1024) return set_err(WV_ERR_UNSUPPORTED, "k %d too large for the replay heap", k);
    // error-bound constants: reference-order fp32 (gamma_{dpb+8}) and the MFMA's
    // fp32 accumulation over NK chained 16-deep products (u' = 2^-22)
    const double u4 = 2.384185791015625e-07;
    const double hdep = NK + 16.0;
    const float gacc = (float)(hdep * u4 / (1.0 - hdep * u4));
    const float gd = (float)gamma_n(idx->dpb + 8);
    // int8 keys: S = fl(fl(sq sb) float(sum)), at most three roundings of |q^ . x^|
    const float gacc8 = 4.0001f * 5.9604645e-08f;
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
        // the exact pass's and the replays' row bitmap(s)
        const uint32_t* exv = pqa ? idx->pqa_valid + c0 * idx->pqa_vq : valid;
        idx->cur_vq = pqa ? idx->pqa_vq : 0;
        idx->cur_tq = t_sel;
        idx->cur_pqk = pqk;
        float4* qinfo = idx->qsInfo.as<float4>();
        if (phase != 2) {
            k_query_split<<<(unsigned)((cn_pad + 3) / 4), 256, 0, s>>>(Qn, idx->dpad, idx->dpb, cn, cn_pad,
                                                                       idx->qsQb.as<uint16_t>(), qinfo);
            if (q8)
                k_query_q8<<<(unsigned)((cn_pad + 3) / 4), 256, 0, s>>>(Qn, idx->dpad, idx->dims, idx->dpb8, cn, cn_pad,
                                                                        qinfo, idx->q8Qb.as<unsigned char>(),
                                                                        idx->q8Scale.as<float>(),
                                                                        idx->q8Info.as<float4>());
        }
        // the selection's bound: int8 keys use their own query split and maxima
        const float4* qinfo_sel = q8 ? idx->q8Info.as<float4>() : qinfo;
        const uint32_t* qmax_sel = q8 ? idx->qmax8 : idx->qsmax;
        const float gacc_sel = q8 ? gacc8 : gacc;
        Q8Filter q8f{idx->X8, idx->sb8, idx->dpb8, idx->q8Qb.as<unsigned char>(), idx->q8Scale.as<float>(),
                     idx->q8Info.as<float4>(), idx->qmax8, gacc8};
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
        const bool w4 = !q8 && idx->dpb > QS_W4_DPB;
        const int w4_nb = NK == 64 ? 4 : 3;
        a.nqg = (int)(cn_pad / (q8wide ? 64 : (w4 || q8cp) ? 128 : QS_QPB));
        int64_t nspans = 256 / std::gcd(256, a.nqg);
        while ((int64_t)a.nqg * nspans < 256) nspans *= 2;
        if (idx->spans_opt > 0) nspans = idx->spans_opt;
        {   // a span's plane bytes (+ one tile of slack) must stay below 4 GiB (32-bit buffer offsets)
            const int64_t row_b = q8 ? (int64_t)idx->dpb8 : (int64_t)idx->dpb * 2;
            const int64_t slot_b = (int64_t)RB * 32 * row_b;
            const int64_t max_sps = ((1ll << 32) - 2 * 256ll * row_b) / slot_b;
            nspans = std::max<int64_t>(nspans, (nslots + max_sps - 1) / max_sps);
        }
        if (idx->spans_opt <= 0) {  // whole rounds of one workgroup per CU (10M x 1024: 5 spans = 320 groups -> 8)
            const int64_t unit = 256 / std::gcd(256, a.nqg);
            nspans = (nspans + unit - 1) / unit * unit;
        }
        nspans = std::max<int64_t>(1, std::min<int64_t>(nspans, nslots));
        const int64_t sps = (nslots + nspans - 1) / nspans;
        a.slots_per_span = (int)sps;
        a.nspans = (int)((nslots + sps - 1) / sps);
        const bool l2 = metric == L2;
        const size_t lds = q8wide ? (size_t)3 * 32 * 1024 + 1024 + (l2 ? (size_t)4 * 512 : 0)
                         : q8cp ? (size_t)3 * NC8 * 1024 + 1024 + (l2 ? (size_t)8 * 4 * 128 : 0)
                         : q8 ? (size_t)3 * RB * 2 * NC8 * 1024 + 1024 + (l2 ? (size_t)8 * 4 * RB * 128 : 0) +
                                    (pqk ? (size_t)8 * 1024 : 0)
                         : w4 ? (size_t)w4_nb * (NK / 4) * 2048 + 256 + (l2 ? (size_t)4 * 4 * 128 : 0)
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
#define WV_Q8S(NCV, RBV, L2V, STV, PFV)                                                                        \
    do {                                                                                                       \
        HIPCHK(hipFuncSetAttribute((const void*)k_q8_blockkey<NCV, RBV, L2V, STV, false, PFV>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
        k_q8_blockkey<NCV, RBV, L2V, STV, false, PFV><<<grid, 512, lds, s>>>(q8a);                              \
    } while (0)
#define WV_Q8(NCV, RBV, L2V) do { if (idx->q8_pf == 2) WV_Q8S(NCV, RBV, L2V, false, 2); else WV_Q8S(NCV, RBV, L2V, false, 1); } while (0)
#ifdef WV_QS_DBG  // timing experiments (k_q8_blockkey DBG bits), not in the product build
#define WV_Q8D(DV)                                                                                             \
    do {                                                                                                       \
        HIPCHK(hipFuncSetAttribute((const void*)k_q8_blockkey<12, 2, false, false, false, 1, DV>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
        k_q8_blockkey<12, 2, false, false, false, 1, DV><<<grid, 512, lds, s>>>(q8a);                           \
    } while (0)
#endif
#define WV_Q8L(NCV, L2V)                                                                                       \
    do {                                                                                                       \
        HIPCHK(hipFuncSetAttribute((const void*)k_q8_blockkey<NCV, 2, L2V, false, false, 1, 0, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
        k_q8_blockkey<NCV, 2, L2V, false, false, 1, 0, true><<<grid, 512, lds, s>>>(q8a);                     \
    } while (0)
        // a partial last query group (batches that are not a multiple of 256):
        // the padding's waves skip their MFMAs (LIVE)
        const bool q8live = idx->q8_live && cn % QS_QPB != 0;
// per-query keys (pqk: never L2, stag or the 32-wide shape)
#define WV_Q8M(NCV, LIVEV)                                                                                     \
    do {                                                                                                       \
        HIPCHK(hipFuncSetAttribute((const void*)k_q8_blockkey<NCV, 2, false, false, false, 1, 0, LIVEV, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
        k_q8_blockkey<NCV, 2, false, false, false, 1, 0, LIVEV, true><<<grid, 512, lds, s>>>(q8a);           \
    } while (0)
#define WV_Q8T(NCV, L2V)                                                                                       \
    do {                                                                                                       \
        if constexpr (!L2V) {                                                                                  \
            if (pqk) { if (q8live) WV_Q8M(NCV, true); else WV_Q8M(NCV, false); break; }                       \
        }                                                                                                      \
        if (idx->q8_stag) WV_Q8S(NCV, 2, L2V, true, 1); else if (q8live) WV_Q8L(NCV, L2V); else WV_Q8(NCV, 2, L2V); \
    } while (0)
#define WV_Q8N(L2V)                                    \
    switch (NC8) {                                     \
    case 8: WV_Q8T(8, L2V); break;                     \
    case 10: WV_Q8T(10, L2V); break;                   \
    case 12: WV_Q8T(12, L2V); break;                   \
    case 16: WV_Q8(16, 1, L2V); break;                 \
    case 20: WV_Q8(20, 1, L2V); break;                 \
    default: WV_Q8(24, 1, L2V); break;                 \
    }
        idx->stats.last_route = q8 ? WV_ROUTE_QS_INT8 : w4 ? WV_ROUTE_QS_W4 : WV_ROUTE_QS_BF16;
        if (q8) {
            Q8Args q8a;
            q8a.X8 = idx->X8;
            q8a.sb = idx->sb8;
            q8a.xnorm2 = idx->xnorm2;
            q8a.valid = valid;
            q8a.Q8 = idx->q8Qb.as<unsigned char>();
            q8a.qscale = idx->q8Scale.as<float>();
            q8a.key = a.key;
            q8a.ldk = ldk;
            q8a.nslots = nslots;
            q8a.slots_per_span = a.slots_per_span;
            q8a.nspans = a.nspans;
            q8a.nqg = a.nqg;
            q8a.nq_live = cn;
            q8a.prio = idx->q8_prio;
            if (pqk) {  // query q of this chunk: its bitmap row (the exact pass's too)
                q8a.qmask = exv;
                q8a.qmask_ld = idx->pqa_vq;
                q8a.qmask_n = cn;
            }
#ifdef WV_QS_DBG
            if (idx->sel_dbg > 0 && !l2 && NC8 == 12) {
                switch (idx->sel_dbg) {
                case 1: WV_Q8D(1); break;
                case 2: WV_Q8D(2); break;
                case 3: WV_Q8D(3); break;
                case 4: WV_Q8D(4); break;
                case 5: WV_Q8D(5); break;
                case 6: WV_Q8D(6); break;
                case 8: WV_Q8D(8); break;
                case 9: WV_Q8D(9); break;
                default: WV_Q8D(7); break;
                }
            } else
#endif
            // small batches: the register-streaming kernel (one plane pass, no
            // 256-query padding of the MFMA work), the same keys
            const int qg = cn <= 16 ? 1 : 2;
            const bool gemv = idx->q8_gemv && !q8cp && !pqk && cn <= 32 && NC8 <= (qg == 1 ? 24 : 16) && nb < (1ll << 40);
            if (gemv) {
                idx->stats.last_route = WV_ROUTE_Q8_GEMV;
                const unsigned gg = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, (nb + 3) / 4));
#define WV_Q8G(NCV, QGV, L2V) k_q8_gemv<NCV, QGV, L2V><<<gg, 256, 0, s>>>(q8a, nb)
#define WV_Q8GQ(NCV, L2V) do { if (qg == 1) WV_Q8G(NCV, 1, L2V); else WV_Q8G(NCV, 2, L2V); } while (0)
#define WV_Q8GN(L2V)                                   \
    switch (NC8) {                                     \
    case 8: WV_Q8GQ(8, L2V); break;                    \
    case 10: WV_Q8GQ(10, L2V); break;                  \
    case 12: WV_Q8GQ(12, L2V); break;                  \
    case 16: WV_Q8GQ(16, L2V); break;                  \
    case 20: WV_Q8G(20, 1, L2V); break;                \
    default: WV_Q8G(24, 1, L2V); break;                \
    }
                if (l2) { WV_Q8GN(true); } else { WV_Q8GN(false); }
#undef WV_Q8GN
#undef WV_Q8GQ
#undef WV_Q8G
            } else if (idx->q8_shape == 32) {
#define WV_Q832(NCV, RBV, L2V)                                                                                \
    do {                                                                                                      \
        HIPCHK(hipFuncSetAttribute((const void*)k_q8_blockkey32<NCV, RBV, L2V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
        k_q8_blockkey32<NCV, RBV, L2V><<<grid, 512, lds, s>>>(q8a);                                            \
    } while (0)
#define WV_Q832N(L2V)                                  \
    switch (NC8) {                                     \
    case 8: WV_Q832(16, 2, L2V); break;                \
    case 10: WV_Q832(20, 2, L2V); break;               \
    case 12: WV_Q832(24, 2, L2V); break;               \
    case 16: WV_Q832(32, 1, L2V); break;               \
    case 20: WV_Q832(40, 1, L2V); break;               \
    default: WV_Q832(48, 1, L2V); break;               \
    }
                if (l2) { WV_Q832N(true); } else { WV_Q832N(false); }
#undef WV_Q832N
#undef WV_Q832
            } else if (q8cp) {
#define WV_Q8CP(NCSV, L2V)                                                                                     \
    do {                                                                                                       \
        HIPCHK(hipFuncSetAttribute((const void*)k_q8_blockkey_cp<NCSV, L2V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
        k_q8_blockkey_cp<NCSV, L2V><<<grid, 512, lds, s>>>(q8a);                                               \
    } while (0)
#define WV_Q8CPW(NPV, L2V)                                                                                     \
    do {                                                                                                       \
        HIPCHK(hipFuncSetAttribute((const void*)k_q8_blockkey_cp<16, L2V, NPV, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
        k_q8_blockkey_cp<16, L2V, NPV, 4><<<grid, 256, lds, s>>>(q8a);                                         \
    } while (0)
#define WV_Q8CPN(L2V)                                  \
    switch (NC8) {                                     \
    case 32: WV_Q8CP(16, L2V); break;                  \
    case 40: WV_Q8CP(20, L2V); break;                  \
    case 48: WV_Q8CP(24, L2V); break;                  \
    case 64: WV_Q8CPW(4, L2V); break;                  \
    case 80: WV_Q8CPW(5, L2V); break;                  \
    default: WV_Q8CPW(6, L2V); break;                  \
    }
                if (l2) { WV_Q8CPN(true); } else { WV_Q8CPN(false); }
#undef WV_Q8CPN
#undef WV_Q8CPW
#undef WV_Q8CP
            } else if (l2) { WV_Q8N(true); } else { WV_Q8N(false); }
        } else if (w4) {
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
#undef WV_Q8N
#undef WV_Q8T
#undef WV_Q8M
#undef WV_Q8L
#undef WV_Q8S
#undef WV_Q8
        HIPCHK(hipGetLastError());
        if (time_it) { HIPCHK(hipEventRecord(idx->ev1, s)); idx->timed = 1; }
        idx->stats.mfma_launches++;
#ifdef WV_QS_DBG  // timing experiments: the keys are wrong, skip the rest of the pipeline
        if (idx->sel_dbg > 0) {
            HIPCHK(hipMemsetAsync(o_n + c0, 0, (size_t)cn * sizeof(int32_t), s));
            continue;
        }
#endif
        }
        // ---- candidate blocks, exact rows, proof ----
        int32_t* flags = phase ? idx->qsFlags.as<int32_t>() : o_flags ? o_flags + c0 : idx->qsFlags.as<int32_t>();
        int32_t* olist = idx->qsList.as<int32_t>() + qc;  // second half: the overflow list
        // select / exact pass RV over all queries (list == nullptr) or over the listed ones
        // phase 0: the first select resets the flag-list cursors (qscount[1], [3])
        const bool ctr_reset = phase == 0;
        // sel_rc: a failed scratch allocation (checked after every sel call)
        int sel_rc = WV_OK;
        auto sel = [&](int RV, const int32_t* list, const uint32_t* cnt, float* tA) {
            const unsigned gw = (unsigned)((cn + 3) / 4);
            uint32_t* lc = (ctr_reset && !list) ? idx->qscount : nullptr;
            // the filtering select keeps a sorted list of 64 (RT - 1) >= k+1 entries
            // instead of the output capacity's: it pays where RT < RV (int8 keys'
            // 448-block lists at k < 64: C3 select 2.81 -> 2.14 ms, 1.25M-row
            // shard 1.42 -> 0.59 ms); at RT == RV the sorted-list form is faster
            // (C2: 0.61 vs 0.92 ms)
            const int RT = qs_R_flat(k);
            // small batches: the split selection (P waves per query)
            if (!list && !pqs && cn <= idx->sel_split_max && RT <= RV && RT <= 8) {
                const int P = (int)std::max<int64_t>(1, std::min<int64_t>(256, (nb + 2047) / 2048));
                const int LV = 64 * (RV - 1);
                const size_t pb = (size_t)cn * P * (k + 1) * sizeof(float);
                if (idx->qsScratch.ensure(pb + (size_t)cn * sizeof(float)) != hipSuccess) {
                    sel_rc = set_err(WV_ERR_HIP, "split selection: %zu bytes of scratch", pb + (size_t)cn * sizeof(float));
                    return;
                }
                float* part = idx->qsScratch.as<float>();
                float* Tq = part + (size_t)cn * P * (k + 1);
                dim3 gp((unsigned)P, (unsigned)cn);
#define WV_SPLIT(RTV)                                                                                             \
    do {                                                                                                          \
        k_sel_part<RTV><<<gp, 64, 0, s>>>(a.key, ldk, nb, k, P, part);                                            \
        k_sel_mid<RTV><<<(unsigned)cn, 64, 0, s>>>(part, P, (int)cn, k, metric, qinfo_sel, qmax_sel, idx->d_maxn2, \
                                                   gd, gacc_sel, idx->qsNc.as<int32_t>(), flags,                  \
                                                   idx->qsEps.as<float>(), Tq, tA, idx->qsCap.as<float>(), lc);    \
    } while (0)
                if (RT == 2) WV_SPLIT(2); else if (RT == 4) WV_SPLIT(4); else WV_SPLIT(8);
#undef WV_SPLIT
                k_sel_collect<<<gp, 64, 0, s>>>(a.key, ldk, nb, P, metric, qinfo_sel, Tq, idx->qsCand.as<uint32_t>(), LV,
                                                idx->qsNc.as<int32_t>(), flags);
                k_sel_clamp<<<(unsigned)((cn + 255) / 256), 256, 0, s>>>((int)cn, LV, idx->qsNc.as<int32_t>());
                if (t_sel)  // no lowered threshold (+inf): the 2-eps argument holds
                    k_fill_u32<<<(unsigned)((cn + 255) / 256), 256, 0, s>>>(reinterpret_cast<uint32_t*>(t_sel), cn,
                                                                            0x7f800000u);
                return;
            }
            if (idx->sel_filter && RT < RV && !pqs) {
#define WV_SELF(RV, RTV) k_blk_select_f<RV, RTV><<<gw, 256, 0, s>>>(a.key, ldk, nb, (int)cn, k, metric, qinfo_sel, qmax_sel, idx->d_maxn2, gd, gacc_sel, idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(), flags, idx->qsEps.as<float>(), list, cnt, tA, idx->qsCap.as<float>(), lc, t_sel)
                if (RV == 4) WV_SELF(4, 2);
                else if (RT == 2) WV_SELF(8, 2);
                else WV_SELF(8, 4);
#undef WV_SELF
                return;
            }
#define WV_SELR(RV) k_blk_select<RV><<<gw, 256, 0, s>>>(a.key, ldk, nb, (int)cn, k, metric, qinfo_sel, qmax_sel, idx->d_maxn2, gd, gacc_sel, idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(), flags, idx->qsEps.as<float>(), list, cnt, tA, idx->qsCap.as<float>(), lc, t_sel, pqs ? exv : nullptr, pqs ? idx->pqa_vq : 0, pqs ? idx->pqa_m + c0 : nullptr)
            if (RV == 2) WV_SELR(2); else if (RV == 4) WV_SELR(4); else if (RV == 8) WV_SELR(8); else if (RV == 16) WV_SELR(16);
            else if (RV == 32) WV_SELR(32); else WV_SELR(64);
#undef WV_SELR
        };
        // per query an upper bound of the (k+1)-th smallest exact distance: the
        // select's (phase 0), lowered to the global one by k_blk_gthresh (phase 2)
        const float* capv = idx->exact_cap ? idx->qsCap.as<float>() : nullptr;
        auto exa = [&](int RV, const int32_t* list, const uint32_t* cnt, const float* eb = nullptr, int64_t ldE = 0,
                       const uint32_t* fmask = nullptr) {
            launch_blk_exact(idx, s, RV, metric, v5, Qn, exv, (int)cn, k, kout, o_ids + c0 * kout, o_d + c0 * kout,
                             o_n + c0, flags, list, cnt, eb, ldE, capv, qinfo, q8 && idx->q8_filter ? &q8f : nullptr,
                             fmask);
        };
        if (phase != 2) sel(R, nullptr, nullptr, phase == 1 ? topA : nullptr);
        if (sel_rc) return sel_rc;
        HIPCHK(hipGetLastError());
        if (phase == 1) continue;
        if (phase == 2)  // the global threshold cuts this shard's candidate lists
            k_blk_gthresh<<<(unsigned)((cn + 3) / 4), 256, 0, s>>>(gA, gE, W, (int)cn, k, metric, qinfo, a.key, ldk,
                                                                  idx->qsCand.as<uint32_t>(), L, idx->qsNc.as<int32_t>(),
                                                                  idx->qsEps.as<float>(), flags,
                                                                  idx->exact_cap ? idx->qsCap.as<float>() : nullptr);
        const size_t bm_lds = (size_t)32 * (idx->dpad + 4) * sizeof(float);
        // (bmE holds cn*L*32 floats: above a 4 GiB budget, or past the 2^23
        // queries k_inv_scatter's packed (q << 9 | j) can name, the
        // candidate-major k_blk_exact computes the distances itself)
        const bool bm_rows = idx->exact_bm && bm_lds <= 64 * 1024 && nb < (1ll << 31) && cn < (1ll << 23) && L <= 512 &&
                             (int64_t)cn * L * 32 * 4 <= (4ll << 30);
        // wider rows with int8 keys: the int8 row filter runs block-major
        // (k_q8_filt_bm reads each listed block's codes once), the exact
        // distances stay per query
        // (small batches keep the per-query filter: the inversion and the
        // block-major launch cost more than the few listed blocks save there)
        const bool bm_filt = !bm_rows && q8 && idx->q8_bm && idx->q8_filter && idx->exact_filter && capv &&
                             idx->dpb8 <= 1536 && nb < (1ll << 31) && cn >= idx->q8_bm_min && cn < (1ll << 23) &&
                             L <= 512;
        if (bm_rows || bm_filt) {
            // block-major exact distances: invert the candidate lists per block
            const int64_t ldE = (int64_t)L * 32;
            HIPCHK(idx->bmCnt.ensure((size_t)nb * sizeof(uint32_t)));
            HIPCHK(idx->bmOff.ensure((size_t)(nb + 1) * sizeof(uint32_t)));
            HIPCHK(idx->bmPairs.ensure((size_t)cn * L * sizeof(uint32_t)));
            if (bm_rows) HIPCHK(idx->bmE.ensure((size_t)cn * ldE * sizeof(float)));
            else HIPCHK(idx->fMask.ensure((size_t)cn * L * sizeof(uint32_t)));
            {
                int rc = invert_lists(idx, s, idx->qsCand.as<uint32_t>(), idx->qsNc.as<int32_t>(), flags, cn, L, nb);
                if (rc) return rc;
            }
            if (bm_rows) {
                launch_exact_bm(idx, s, metric, v5, Qn, nb, bm_lds, ldE);
                HIPCHK(hipGetLastError());
                exa(R, nullptr, nullptr, idx->bmE.as<float>(), ldE);
            } else {
                launch_q8_filt_bm(idx, s, metric, q8f, idx->xnorm2, valid, nb, L, capv, qinfo, (float)gamma_n(idx->dpb + 8),
                                  idx->fMask.as<uint32_t>());
                HIPCHK(hipGetLastError());
                exa(R, nullptr, nullptr, nullptr, 0, idx->fMask.as<uint32_t>());
            }
        } else {
            exa(R, nullptr, nullptr);
        }
        HIPCHK(hipGetLastError());
        if (R < 8) {  // candidate lists that overflowed (flag 2): again with the 448-block lists
            if (!ctr_reset) HIPCHK(hipMemsetAsync(idx->qscount + 3, 0, sizeof(uint32_t), s));
            k_flag_list<<<(unsigned)((cn + 255) / 256), 256, 0, s>>>(flags, (int)cn, olist, idx->qscount + 2, 2);
            sel(8, olist, idx->qscount + 2, nullptr);
            if (sel_rc) return sel_rc;
            exa(8, olist, idx->qscount + 2);
            HIPCHK(hipGetLastError());
        }
        if (pqs && R < 16) {
            // per-query lists whose proof failed (flag 1): once more with
            // 960-block lists at the deepest threshold before the replay (the
            // one-wave replay walks most blocks when the key bound is wide)
            HIPCHK(idx->pqaM2.ensure((size_t)(c0 + cn) * sizeof(int32_t)));
            k_fill_u32<<<(unsigned)((cn + 255) / 256), 256, 0, s>>>(idx->pqaM2.as<uint32_t>() + c0, cn, 960u);
            k_flag_list<<<(unsigned)((cn + 255) / 256), 256, 0, s>>>(flags, (int)cn, olist, idx->qscount + 2, 1);
            const int32_t* keep = idx->pqa_m;
            idx->pqa_m = idx->pqaM2.as<int32_t>();  // the select reads pqa_m + c0
            sel(16, olist, idx->qscount + 2, nullptr);
            if (sel_rc) return sel_rc;
            idx->pqa_m = keep;
            exa(16, olist, idx->qscount + 2);
            HIPCHK(hipGetLastError());
        }
        if (idx->qs_force_flag) HIPCHK(hipMemsetAsync(flags, 1, (size_t)cn * sizeof(int32_t), s));
        if (phase == 2 && o_flags)
            HIPCHK(hipMemcpyAsync(o_flags + c0, flags, (size_t)cn * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
        if (mode == 1) continue;
        if (pqs && o_flags) continue;  // per-query lists on the union's keys: the caller searches the unresolved queries alone
        // ---- flagged queries: the exact heap replay, bounded by the block keys ----
        if (!ctr_reset) HIPCHK(hipMemsetAsync(idx->qscount + 1, 0, sizeof(uint32_t), s));
        k_flag_list<<<(unsigned)((cn + 255) / 256), 256, 0, s>>>(flags, (int)cn, idx->qsList.as<int32_t>(), idx->qscount, 0);
        {
            int rc = launch_blk_replay(idx, s, a.key, ldk, nb, idx->qsEps.as<float>(), qinfo, exv, Qn,
                                       idx->qsList.as<int32_t>(), idx->qscount, 0, cn, k, kout, o_ids + c0 * kout,
                                       o_d + c0 * kout, o_n + c0, nullptr, nullptr, nullptr, 1, 0);
            if (rc) return rc;
        }
        // per-query keys: the flagged queries are resolved here, none is left for the caller
        if (pqk && o_flags) HIPCHK(hipMemsetAsync(o_flags + c0, 0, (size_t)cn * sizeof(int32_t), s));
    }
    if (idx->timing) {
        HIPCHK(hipEventRecord(idx->evt1, s));
        idx->timed_total = 1;
    }
    if (qc >= nq && valid == idx->present) idx->qs_keys_nq = nq;
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
    const bool qs = idx->compression == WV_COMPRESSION_NONE && (idx->qs_planes || idx->q8_only) && !idx->has_nonfinite &&
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
    const size_t rlds = packed_replay_lds(k) + 16 * 64 * sizeof(float) + (size_t)idx->dpb * sizeof(float);
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

