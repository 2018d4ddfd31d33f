// vector_index.hip -- the rest of the db.VectorIndex surface the shard calls on
// a flat index (adapters/repos/db/vector_index.go:25-54): Iterate,
// QueryVectorDistancer, Preload, UpdateUserConfig (+ ValidateUserConfigUpdate)
// and CompressionStats.  Included by runtime.hip (same translation unit: uses
// its index struct, prepare_queries, the RQ encoders and add_rows_locked).
#pragma once

namespace wv {
namespace {  // internal linkage: each runtime unit compiles the kernels it launches

// QueryVectorDistancer.DistanceFunc over listed slots (flat/index.go:1160-1240,
// default branch: SingleDist(normalised query, stored row)).  Lane per slot;
// slot < 0 = not present (left to the host).
template <int METRIC, int VARIANT>
__global__ __launch_bounds__(64) void k_query_slots_dist(const float* __restrict__ X, int64_t dpad,
                                                         const float* __restrict__ q, int d,
                                                         const int64_t* __restrict__ slots, int64_t n,
                                                         float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t s = slots[i];
    out[i] = s < 0 ? 0.f : exact_dist<METRIC, VARIANT>(q, X + s * dpad, d);
}

// cached BQ branch (:1205-1214): BinaryQuantizer.DistanceBetweenCompressedVectors
// = HammingBitwise(code, query code).  Codes word-major (bq_kernels.hip).
__global__ __launch_bounds__(64) void k_bq_query_slots(const uint64_t* __restrict__ codes, int64_t ccap, int words,
                                                       const uint64_t* __restrict__ qcode,
                                                       const int64_t* __restrict__ slots, int64_t n,
                                                       float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t s = slots[i];
    if (s < 0) { out[i] = 0.f; return; }
    uint32_t c = 0;
    for (int w = 0; w < words; w++) c += (uint32_t)__popcll(codes[(int64_t)w * ccap + s] ^ qcode[w]);
    out[i] = (float)c;
}

}  // namespace
}  // namespace wv

static const char* metric_name(int m) {
    switch (m) {
    case WV_METRIC_L2_SQUARED: return "l2-squared";
    case WV_METRIC_DOT: return "dot";
    case WV_METRIC_COSINE_DOT: return "cosine";
    default: return "hamming";
    }
}

// flat.Iterate (flat/index.go:1057-1079): ids in ascending key order (the
// bucket cursor over big-endian id keys) until fn returns 0.  The id list is
// snapshotted under the lock, fn runs without it (fn may call back in).
extern "C" int wv_index_iterate(wv_index* idx, int (*fn)(uint64_t id, void* user), void* user) {
    if (!idx || !fn) return set_err(WV_ERR_INVALID, "nil argument");
    std::vector<uint64_t> ids;
    {
        std::lock_guard<std::mutex> g(idx->mu);
        ids.reserve((size_t)idx->npresent);
        for (int64_t s = 0; s < idx->hiwater; s++)
            if (idx->h_present[s]) ids.push_back(idx->id_base + (uint64_t)s);
    }
    for (uint64_t id : ids)
        if (!fn(id, user)) break;
    return WV_OK;
}

// flat.QueryVectorDistancer(query).DistanceFunc(id) for n ids
// (flat/index.go:1160-1240).  Uncompressed, PQ, or BQ/RQ without the cache:
// SingleDist(normalised query, stored row); a missing id reads an empty value
// from the bucket, so SingleDist fails with "<qd> vs 0: vector lengths don't
// match".  BQ / RQ-8 / RQ-1 with option "cache" = 1 (BQ.Cache / RQ.Cache):
// the quantized scan distance (createDistanceCalcQuantized, :534-566) of the
// cached code; an id beyond the cache fails with "node %d is larger than the
// cache size %d".  out_rc: per-id status (NULL: the first failing id's error is
// returned, out[] written up to it).
extern "C" int wv_index_query_distances(wv_index* idx, const float* query, int64_t qd, const uint64_t* ids,
                                        int64_t n, float* out, int32_t* out_rc) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (n < 0 || (n > 0 && (!ids || !out)) || qd < 0 || (qd > 0 && !query)) return set_err(WV_ERR_INVALID, "bad arguments");
    if (n == 0) return WV_OK;
    std::lock_guard<std::mutex> g(idx->mu);
    HIPCHK(hipSetDevice(idx->device));
    const bool quant = idx->cache_opt && ((idx->compression == WV_COMPRESSION_BQ) || (idx->rq_bits && idx->rq_ready));
    std::vector<int64_t> slots((size_t)n, -1);
    std::vector<int32_t> rcs((size_t)n, WV_OK);
    std::vector<std::string> msgs((size_t)n);
    char buf[256];
    for (int64_t i = 0; i < n; i++) {
        const uint64_t id = ids[i];
        const bool in_range = id >= idx->id_base && (int64_t)(id - idx->id_base) < idx->hiwater;
        const int64_t s = in_range ? (int64_t)(id - idx->id_base) : -1;
        const bool present = s >= 0 && idx->h_present[s];
        if (quant) {
            if (id < idx->id_base || id - idx->id_base > (uint64_t)idx->hiwater) {  // int32(nodeID) > cache.Len()
                snprintf(buf, sizeof buf, "node %llu is larger than the cache size %lld", (unsigned long long)id,
                         (long long)idx->hiwater);
                rcs[i] = WV_ERR_INVALID;
                msgs[i] = buf;
            } else if (!present) {  // the cache miss reads an empty code
                snprintf(buf, sizeof buf, "0 vs %d: vector lengths don't match",
                         idx->compression == WV_COMPRESSION_BQ ? idx->words : idx->rq_D);
                rcs[i] = WV_ERR_VECTOR_LENGTH;
                msgs[i] = buf;
            } else {
                slots[i] = s;
            }
        } else if (!present || qd != idx->dims) {
            snprintf(buf, sizeof buf, "%lld vs %d: vector lengths don't match", (long long)qd, present ? idx->dims : 0);
            rcs[i] = WV_ERR_VECTOR_LENGTH;
            msgs[i] = buf;
        } else {
            slots[i] = s;
        }
    }
    int64_t nvalid = 0;
    for (int64_t i = 0; i < n; i++) nvalid += slots[i] >= 0;
    std::vector<float> h((size_t)n, 0.f);
    if (nvalid > 0) {
        if (qd != idx->dims && quant)  // the quantizer encodes a query of the index's length only
            return set_err(WV_ERR_VECTOR_LENGTH, "%lld vs %d: vector lengths don't match", (long long)qd, idx->dims);
        hipStream_t s = idx->stream;
        HIPCHK(idx->qraw.ensure((size_t)qd * sizeof(float)));
        HIPCHK(hipMemcpyAsync(idx->qraw.p, query, (size_t)qd * sizeof(float), hipMemcpyHostToDevice, s));
        int rc = prepare_queries(idx, s, idx->qraw.as<float>(), 1, QB);
        if (rc) return rc;
        const float* Qn = idx->qn.as<float>();
        DBuf dS, dO;
        HIPCHK(dS.ensure((size_t)n * sizeof(int64_t)));
        HIPCHK(dO.ensure((size_t)n * sizeof(float)));
        HIPCHK(hipMemcpyAsync(dS.p, slots.data(), (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice, s));
        const unsigned grid = (unsigned)((n + 63) / 64);
        if (quant && idx->compression == WV_COMPRESSION_BQ) {
            DBuf qc;
            HIPCHK(qc.ensure((size_t)idx->words * sizeof(uint64_t)));
            k_bq_encode_rows<<<(unsigned)((idx->words + 255) / 256), 256, 0, s>>>(Qn, idx->dpad, 1, idx->dims, nullptr,
                                                                                  qc.as<uint64_t>(), 1);
            k_bq_query_slots<<<grid, 64, 0, s>>>(idx->codes, idx->cap, idx->words, qc.as<uint64_t>(),
                                                 dS.as<int64_t>(), n, dO.as<float>());
            HIPCHK(hipGetLastError());
            HIPCHK(hipMemcpyAsync(h.data(), dO.p, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            qc.release();
        } else if (quant) {  // RQ-8 / RQ-1: the scan distances of the quantized search, gathered
            rc = rq_encode_queries(idx, s, 1);
            if (rc) return rc;
            const int64_t ld = std::max<int64_t>(round_up(idx->hiwater, EBLK), EBLK);
            const int64_t nq32 = round_up(1, RQ_QPB);
            DBuf E, B;
            HIPCHK(E.ensure((size_t)nq32 * ld * sizeof(float)));
            HIPCHK(B.ensure((size_t)nq32 * (ld / EBLK) * sizeof(float)));
            rc = rq_dist(idx, s, idx->present, 0, 1, ld, E.as<float>(), B.as<float>());
            if (rc) return rc;
            std::vector<float> row((size_t)idx->hiwater);
            HIPCHK(hipMemcpyAsync(row.data(), E.p, (size_t)idx->hiwater * sizeof(float), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            for (int64_t i = 0; i < n; i++)
                if (slots[i] >= 0) h[i] = row[slots[i]];
            E.release();
            B.release();
        } else {
            const bool v5 = idx->variant == WV_VARIANT_AVX512;
#define WV_QD(M, V) k_query_slots_dist<M, V><<<grid, 64, 0, s>>>(idx->X, idx->dpad, Qn, idx->dims, dS.as<int64_t>(), n, dO.as<float>())
            switch (idx->metric) {
            case WV_METRIC_L2_SQUARED: if (v5) WV_QD(L2, AVX512); else WV_QD(L2, AVX256); break;
            case WV_METRIC_DOT: if (v5) WV_QD(DOT, AVX512); else WV_QD(DOT, AVX256); break;
            case WV_METRIC_COSINE_DOT: if (v5) WV_QD(COSINE, AVX512); else WV_QD(COSINE, AVX256); break;
            default: WV_QD(HAMMING, AVX256); break;
            }
#undef WV_QD
            HIPCHK(hipGetLastError());
            HIPCHK(hipMemcpyAsync(h.data(), dO.p, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        dS.release();
        dO.release();
    }
    for (int64_t i = 0; i < n; i++) {
        if (rcs[i] != WV_OK && !out_rc) return set_err(rcs[i], "%s", msgs[i].c_str());
        out[i] = rcs[i] == WV_OK ? h[i] : 0.f;
        if (out_rc) out_rc[i] = rcs[i];
    }
    return WV_OK;
}

// flat.Preload (flat/index.go:844-865): for a compressed index the stored row's
// code goes to the compressed bucket (and the cache).  Here codes and rows live
// together in HBM, so Preload of a compressed index stores the row (its code
// is derived on the device, as Add does) without counting it as indexed; an
// uncompressed index ignores it, as the reference does.
extern "C" int wv_index_preload(wv_index* idx, uint64_t id, const float* vec, int64_t d) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (d > 0 && !vec) return set_err(WV_ERR_INVALID, "nil vector");
    std::lock_guard<std::mutex> g(idx->mu);
    const bool compressed = idx->compression == WV_COMPRESSION_BQ || (idx->rq_bits && idx->rq_ready);
    if (!compressed) return WV_OK;
    HIPCHK(hipSetDevice(idx->device));
    const uint64_t count = idx->count;
    int rc = add_rows_locked(idx, &id, vec, 1, d);
    idx->count = count;
    return rc;
}

// flat.UpdateUserConfig (flat/index.go:763-776): the only mutable field the
// flat index applies is the compression rescore limit (extractCompressionRescore,
// :170-180: BQ.RescoreLimit / RQ.RescoreLimit, else 0).
extern "C" int wv_index_update_user_config(wv_index* idx, const wv_config* updated) {
    if (!idx || !updated) return set_err(WV_ERR_INVALID, "nil argument");
    std::lock_guard<std::mutex> g(idx->mu);
    note_mutation(idx);
    const bool bq_rq = updated->compression == WV_COMPRESSION_BQ || updated->compression == WV_COMPRESSION_RQ8 ||
                       updated->compression == WV_COMPRESSION_RQ1;
    // (PQ / SQ here are the hnsw flatSearch restatement: limit / SQ.RescoreLimit follow the same field)
    idx->rescore_limit = bq_rq || updated->compression == WV_COMPRESSION_PQ || updated->compression == WV_COMPRESSION_SQ
                             ? updated->rescore_limit : 0;
    return WV_OK;
}

// flat.ValidateUserConfigUpdate (flat/index.go:1106-1154): distance, pq, bq,
// rq and rq.bits are immutable (checked in that order).
extern "C" int wv_validate_user_config_update(const wv_config* initial, const wv_config* updated) {
    if (!initial || !updated) return set_err(WV_ERR_INVALID, "nil argument");
    auto b = [](bool v) { return v ? "true" : "false"; };
    if (initial->metric != updated->metric)
        return set_err(WV_ERR_INVALID, "distance is immutable: attempted change from \"%s\" to \"%s\"",
                       metric_name(initial->metric), metric_name(updated->metric));
    const int ci = initial->compression, cu = updated->compression;
    const bool rqi = ci == WV_COMPRESSION_RQ8 || ci == WV_COMPRESSION_RQ1, rqu = cu == WV_COMPRESSION_RQ8 || cu == WV_COMPRESSION_RQ1;
    if ((ci == WV_COMPRESSION_PQ) != (cu == WV_COMPRESSION_PQ))
        return set_err(WV_ERR_INVALID, "pq is immutable: attempted change from \"%s\" to \"%s\"", b(ci == WV_COMPRESSION_PQ),
                       b(cu == WV_COMPRESSION_PQ));
    if ((ci == WV_COMPRESSION_BQ) != (cu == WV_COMPRESSION_BQ))
        return set_err(WV_ERR_INVALID, "bq is immutable: attempted change from \"%s\" to \"%s\"", b(ci == WV_COMPRESSION_BQ),
                       b(cu == WV_COMPRESSION_BQ));
    if (rqi != rqu) return set_err(WV_ERR_INVALID, "rq is immutable: attempted change from \"%s\" to \"%s\"", b(rqi), b(rqu));
    if (rqi && ci != cu)
        return set_err(WV_ERR_INVALID, "rq.bits is immutable: attempted change from \"%d\" to \"%d\"",
                       ci == WV_COMPRESSION_RQ8 ? 8 : 1, cu == WV_COMPRESSION_RQ8 ? 8 : 1);
    return WV_OK;
}

// flat.CompressionStats (flat/index.go:1246-1249): UncompressedStats{} --
// CompressionType "none", CompressionRatio 1.0 (compressionhelpers/compression.go:1015-1024).
extern "C" int wv_index_compression_stats(wv_index* idx, char* type_out, int64_t type_cap, double* ratio) {
    if (!idx) return set_err(WV_ERR_INVALID, "nil index");
    if (type_out && type_cap > 0) snprintf(type_out, (size_t)type_cap, "%s", "none");
    if (ratio) *ratio = 1.0;
    return WV_OK;
}
