// pq_kernels.hip -- gfx950 kernels of the product quantizer
// (compressionhelpers/product_quantization.go, kmeans_encoder.go,
// kmeans/kmeans.go) and of the PQ brute-force search (hnsw/flat_search.go).
//
// Training runs all m segment k-means problems at once (grid.y = segment):
//   k_km_gather_centers   centers[s][c] = segment s of training row subset[s][c]
//   k_km_assign_brute     nearestBruteForce (kmeans.go:373-383)      thread/(row,seg)
//   k_km_neighbors        updateCenterNeighbors (:398-417): sqrt distances to
//                         the other centers, bitonic-sorted per center
//   k_km_assign_prune     nearestWithPruning (:354-371)               thread/(row,seg)
//   k_km_update_centers   updateCenters (:302-332): one workgroup per segment,
//                         thread = cluster, float64 sums in data order
// Search (per query batch):
//   k_pq_lut              LUT[q][s][c] = Provider.Step(q_seg, centroid) (sequential)
//   k_pq_adc              sum of LUT entries in segment order, Wrap, per row;
//                         LUT chunks staged in LDS; exact distances + 256-row
//                         block minima for the heap replay (k_replay_scan)
//   k_pq_finish           flatSearch's merge of the worker heap into the result
//                         heap (pop order), optional rescoring, extraction
// Codes live segment-word-major: codes[(s / 4) * ccap + slot] holds segments
// 4(s/4) .. 4(s/4)+3 of row `slot` as bytes (coalesced dword per lane).
#pragma once

namespace wv {

constexpr int KM_T = 256;  // threads per k-means workgroup; k <= 256 (NewProductQuantizer)

__device__ __forceinline__ float l2_seg(const float* a, const float* b, int ds, int variant) {
    return variant == AVX512 ? exact_raw<L2, AVX512, false>(a, b, ds) : exact_raw<L2, AVX256, false>(a, b, ds);
}

// centers[s][c][:] = T[subset[s * k + c]][s * ds : (s + 1) * ds]
__global__ void k_km_gather_centers(const float* __restrict__ T, int64_t ldt, const int64_t* __restrict__ subset,
                                    int m, int k, int ds, float* __restrict__ centers) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)m * k * ds) return;
    const int j = (int)(i % ds);
    const int64_t sc = i / ds;
    const int s = (int)(sc / k);
    centers[i] = T[subset[sc] * ldt + (int64_t)s * ds + j];
}

// nearestBruteForce: minDist = MaxFloat32, strict <, lowest index wins
__global__ __launch_bounds__(256) void k_km_assign_brute(const float* __restrict__ T, int64_t ldt, int64_t n, int k,
                                                         int ds, const float* __restrict__ centers, int variant,
                                                         const int32_t* __restrict__ active,
                                                         uint32_t* __restrict__ assign) {
    extern __shared__ float csm[];
    const int s = blockIdx.y;
    if (active && !active[s]) return;
    const float* cs = centers + (int64_t)s * k * ds;
    for (int i = threadIdx.x; i < k * ds; i += blockDim.x) csm[i] = cs[i];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* x = T + i * ldt + (int64_t)s * ds;
    float mn = 3.40282346638528859811704183484516925440e+38f;
    uint32_t idx = 0;
    for (int c = 0; c < k; c++) {
        const float d = l2_seg(x, csm + c * ds, ds, variant);
        if (d < mn) { mn = d; idx = (uint32_t)c; }
    }
    assign[(int64_t)s * n + i] = idx;
}

// updateCenterNeighbors: block (c, s); thread j < k computes the euclidean
// distance float32(sqrt(float64(l2))) to center j; the k-1 others are sorted by
// (distance, index) (the reference's pdqsort leaves exact ties unspecified).
__global__ __launch_bounds__(KM_T) void k_km_neighbors(const float* __restrict__ centers, int k, int ds, int variant,
                                                       const int32_t* __restrict__ active,
                                                       uint32_t* __restrict__ nb_idx, float* __restrict__ nb_dist) {
    __shared__ float key[KM_T];
    __shared__ uint32_t val[KM_T];
    const int c = blockIdx.x, s = blockIdx.y, t = threadIdx.x;
    if (active && !active[s]) return;
    const float* cs = centers + (int64_t)s * k * ds;
    float dk = __builtin_inff();
    uint32_t vi = 0xFFFFFFFFu;
    if (t < k && t != c) {
        const int c1 = t < c ? t : c, c2 = t < c ? c : t;  // dist(centers[c1], centers[c2]), c1 < c2
        const float d = l2_seg(cs + c1 * ds, cs + c2 * ds, ds, variant);
        dk = (float)sqrt((double)d);
        vi = (uint32_t)t;
    }
    key[t] = dk;
    val[t] = vi;
    __syncthreads();
    for (int kk = 2; kk <= KM_T; kk <<= 1) {
        for (int j = kk >> 1; j > 0; j >>= 1) {
            const int p = t ^ j;
            if (p > t) {
                const bool up = (t & kk) == 0;
                const bool less_pt = key[p] < key[t] || (key[p] == key[t] && val[p] < val[t]);
                const bool less_tp = key[t] < key[p] || (key[t] == key[p] && val[t] < val[p]);
                if (up ? less_pt : less_tp) {
                    float tk = key[t]; key[t] = key[p]; key[p] = tk;
                    uint32_t tv = val[t]; val[t] = val[p]; val[p] = tv;
                }
            }
            __syncthreads();
        }
    }
    if (t < k - 1) {
        const int64_t o = ((int64_t)s * k + c) * (k - 1) + t;
        nb_idx[o] = val[t];
        nb_dist[o] = key[t];
    }
}

// nearestWithPruning from the previous center; counts changes per segment
__global__ __launch_bounds__(256) void k_km_assign_prune(const float* __restrict__ T, int64_t ldt, int64_t n, int k,
                                                         int ds, const float* __restrict__ centers, int variant,
                                                         const uint32_t* __restrict__ nb_idx,
                                                         const float* __restrict__ nb_dist,
                                                         const int32_t* __restrict__ active,
                                                         uint32_t* __restrict__ assign,
                                                         unsigned long long* __restrict__ changes) {
    extern __shared__ float csm[];
    __shared__ unsigned int wchg;
    const int s = blockIdx.y;
    if (!active[s]) return;
    const float* cs = centers + (int64_t)s * k * ds;
    for (int i = threadIdx.x; i < k * ds; i += blockDim.x) csm[i] = cs[i];
    if (threadIdx.x == 0) wchg = 0;
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const float* x = T + i * ldt + (int64_t)s * ds;
        const uint32_t prev = assign[(int64_t)s * n + i];
        float mn = l2_seg(csm + prev * ds, x, ds, variant);
        const float cd = (float)sqrt((double)mn);
        uint32_t idx = prev;
        const int64_t nb0 = ((int64_t)s * k + prev) * (k - 1);
        for (int j = 0; j < k - 1; j++) {
            if (nb_dist[nb0 + j] >= 2.f * cd) break;
            const uint32_t c = nb_idx[nb0 + j];
            const float d = l2_seg(x, csm + c * ds, ds, variant);
            if (d < mn) { mn = d; idx = c; }
        }
        if (idx != prev) {
            assign[(int64_t)s * n + i] = idx;
            atomicAdd(&wchg, 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && wchg) atomicAdd(&changes[s], (unsigned long long)wchg);
}

// updateCenters: workgroup per segment, thread = cluster.  Rows are walked in
// index order in chunks staged through LDS; each thread adds the members of
// its own cluster in that order into float64 sums (LDS), then divides.
// Empty clusters keep their center (kmeans.go:318-326).
__global__ __launch_bounds__(KM_T) void k_km_update_centers(const float* __restrict__ T, int64_t ldt, int64_t n,
                                                            int k, int ds, const uint32_t* __restrict__ assign,
                                                            const int32_t* __restrict__ active,
                                                            float* __restrict__ centers) {
    extern __shared__ __attribute__((aligned(16))) unsigned char usm[];
    double* acc = reinterpret_cast<double*>(usm);                     // [k][ds]
    uint32_t* ca = reinterpret_cast<uint32_t*>(acc + (size_t)k * ds);   // [KM_T] chunk assignments
    float* cx = reinterpret_cast<float*>(ca + KM_T);                    // [KM_T][ds] chunk values
    const int s = blockIdx.x, t = threadIdx.x;
    if (active && !active[s]) return;
    for (int i = t; i < k * ds; i += KM_T) acc[i] = 0.0;
    uint32_t size = 0;
    for (int64_t c0 = 0; c0 < n; c0 += KM_T) {
        __syncthreads();
        const int64_t i = c0 + t;
        ca[t] = i < n ? assign[(int64_t)s * n + i] : 0xFFFFFFFFu;
        for (int e = t; e < KM_T * ds; e += KM_T) {
            const int64_t r = c0 + e / ds;
            cx[e] = r < n ? T[r * ldt + (int64_t)s * ds + e % ds] : 0.f;
        }
        __syncthreads();
        if (t < k) {
            const int lim = (int)(n - c0 < KM_T ? n - c0 : KM_T);
            for (int r = 0; r < lim; r++) {
                if (ca[r] != (uint32_t)t) continue;
                size++;
                for (int j = 0; j < ds; j++) acc[t * ds + j] += (double)cx[r * ds + j];
            }
        }
    }
    if (t < k && size > 0)
        for (int j = 0; j < ds; j++)
            centers[((int64_t)s * k + t) * ds + j] = (float)(acc[t * ds + j] / (double)size);
}

// KMeansEncoder.Encode over all segments: thread per (row, segment); centers of
// the segment in LDS; L2 SingleDist(segment, centroid), strict <.
// rows[slot * ld ...] -> codes[(s/4) * ccap + slot] byte (s % 4).
__global__ __launch_bounds__(256) void k_pq_encode(const float* __restrict__ rows, int64_t ld, int64_t n,
                                                   const uint32_t* __restrict__ slots, int k, int ds,
                                                   const float* __restrict__ centers, int variant,
                                                   uint32_t* __restrict__ codes, int64_t ccap) {
    extern __shared__ float csm[];
    const int s = blockIdx.y;
    const float* cs = centers + (int64_t)s * k * ds;
    for (int i = threadIdx.x; i < k * ds; i += blockDim.x) csm[i] = cs[i];
    __syncthreads();
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int64_t slot = slots ? (int64_t)slots[r] : r;
    const float* x = rows + slot * ld + (int64_t)s * ds;
    float mn = 3.40282346638528859811704183484516925440e+38f;
    uint32_t idx = 0;
    for (int c = 0; c < k; c++) {
        const float d = l2_seg(x, csm + c * ds, ds, variant);
        if (d < mn) { mn = d; idx = (uint32_t)c; }
    }
    unsigned char* b = reinterpret_cast<unsigned char*>(codes + (int64_t)(s >> 2) * ccap + slot);
    b[s & 3] = (unsigned char)idx;
}

// DistanceLookUpTable entry (product_quantization.go:85-104 computes them
// lazily; every entry has the same value): Step(query_seg, centroid),
// sequential and unfused (distancer/l2.go:63-72, dot_product.go:87-94).
__global__ void k_pq_lut(const float* __restrict__ Q, int64_t ldq, int64_t nq, int m, int k, int ds, int metric,
                         const float* __restrict__ centers, float* __restrict__ lut) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq * m * k) return;
    const int c = (int)(i % k);
    const int64_t qs = i / k;
    const int s = (int)(qs % m);
    const int64_t q = qs / m;
    const float* a = Q + q * ldq + (int64_t)s * ds;
    const float* b = centers + ((int64_t)s * k + c) * ds;
    float sum = 0.f;
    for (int j = 0; j < ds; j++) {
        if (metric == L2) { const float diff = a[j] - b[j]; const float sq = diff * diff; sum = sum + sq; }
        else { const float p = a[j] * b[j]; sum = sum + p; }
    }
    lut[i] = sum;
}

__device__ __forceinline__ float pq_wrap(int metric, float x) {
    if (metric == L2) return x;
    if (metric == DOT) return -x;
    const float w = 1.f - x;
    return w < 0.f ? 0.f : w;
}

// ADC over a row tile for listed query f = blockIdx.y: rows tile0 + 256 r + t,
// r < PQ_RPT.  LUT chunks of PQ_CH segments staged through LDS in segment
// order (the running sums stay in registers, so the fp32 addition order is
// the reference's).  Writes E[f][row] (+inf for invalid rows) and the 256-row
// block minima used by k_replay_scan.
constexpr int PQ_RPT = 16;
constexpr int PQ_CH = 32;
__global__ __launch_bounds__(256) void k_pq_adc(const uint32_t* __restrict__ codes, int64_t ccap, int m, int k,
                                                const uint32_t* __restrict__ valid, int64_t nslots,
                                                const float* __restrict__ lut, const int32_t* __restrict__ qlist,
                                                int metric, int64_t ld, float* __restrict__ E,
                                                float* __restrict__ bmin) {
    extern __shared__ float lsm[];  // [PQ_CH][k]
    __shared__ float red[4][PQ_RPT];
    const int t = threadIdx.x;
    const int f = blockIdx.y;
    const int64_t tile0 = (int64_t)blockIdx.x * 256 * PQ_RPT;
    const float* L = lut + (int64_t)qlist[f] * m * k;
    float sum[PQ_RPT];
#pragma unroll
    for (int r = 0; r < PQ_RPT; r++) sum[r] = 0.f;
    for (int s0 = 0; s0 < m; s0 += PQ_CH) {
        const int ns = m - s0 < PQ_CH ? m - s0 : PQ_CH;
        __syncthreads();
        for (int i = t; i < ns * k; i += 256) lsm[i] = L[(int64_t)s0 * k + i];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < PQ_RPT; r++) {
            const int64_t row = tile0 + 256 * r + t;
            if (row >= nslots) continue;
            float acc = sum[r];
            for (int sw = 0; sw < ns; sw += 4) {  // s0 is a multiple of 4
                const uint32_t w = codes[(int64_t)((s0 + sw) >> 2) * ccap + row];
                const int lim = ns - sw < 4 ? ns - sw : 4;
                for (int b = 0; b < lim; b++) acc = acc + lsm[(sw + b) * k + ((w >> (8 * b)) & 0xFFu)];
            }
            sum[r] = acc;
        }
    }
    const int lane = t & 63, wv = t >> 6;
#pragma unroll
    for (int r = 0; r < PQ_RPT; r++) {
        const int64_t row = tile0 + 256 * r + t;
        const bool ok = row < nslots && ((valid[row >> 5] >> (row & 31)) & 1u);
        const float e = ok ? pq_wrap(metric, sum[r]) : __builtin_inff();
        if (row < ld) E[(int64_t)f * ld + row] = e;
        float mm = e;
        for (int o = 32; o > 0; o >>= 1) mm = fminf(mm, __shfl_xor(mm, o));
        if (lane == 0) red[wv][r] = mm;
    }
    __syncthreads();
    if (t < PQ_RPT) {
        const int64_t blk = tile0 / 256 + t;
        if (blk < ld / 256)
            bmin[(int64_t)f * (ld / 256) + blk] = fminf(fminf(red[0][t], red[1][t]), fminf(red[2][t], red[3][t]));
    }
}

// flatSearch tail (hnsw/flat_search.go:96-141 with one worker): the worker
// heap's ascending extraction asc[li][0..n) is popped max-first
// (= reverse order) into the result heap via addResult (:214-224).
// rescore == 0: extract (fill from the back) -> out rows q = qlist[li].
// rescore == 1: pop all into ascending ids (search.go:1058-1064) -> cand slots
//               [li][R] for k_rescore; cand_n[li].
// Dynamic LDS: [R] u64 | [R] f32.
__global__ __launch_bounds__(64) void k_pq_finish(const uint64_t* __restrict__ asc_ids,
                                                  const float* __restrict__ asc_d, const int32_t* __restrict__ asc_n,
                                                  const int32_t* __restrict__ qlist, int nlist, int R, int k,
                                                  int rescore, uint64_t id_base, uint64_t* __restrict__ out_ids,
                                                  float* __restrict__ out_d, int32_t* __restrict__ out_n,
                                                  uint32_t* __restrict__ cand_slot, int32_t* __restrict__ cand_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char psm[];
    uint64_t* hid = reinterpret_cast<uint64_t*>(psm);
    float* hd = reinterpret_cast<float*>(hid + R);
    const int li = blockIdx.x;
    if (li >= nlist || threadIdx.x != 0) return;
    ReplayHeap hp{hid, hd, 0};
    const int n = asc_n[li];
    for (int i = n - 1; i >= 0; i--) {
        const uint64_t id = asc_ids[(int64_t)li * R + i];
        const float d = asc_d[(int64_t)li * R + i];
        if (hp.len < R) rh_insert(hp, id, d);
        else if (hp.dist[0] > d) { uint64_t a; float b; rh_pop(hp, &a, &b); rh_insert(hp, id, d); }
    }
    const int q = qlist[li];
    const int m = hp.len;
    if (!rescore) {
        for (int i = m - 1; i >= 0; i--) {
            uint64_t a; float b;
            rh_pop(hp, &a, &b);
            if (i < k) { out_ids[(int64_t)q * k + i] = a; out_d[(int64_t)q * k + i] = b; }
        }
        out_n[q] = m < k ? m : k;
        return;
    }
    for (int i = m - 1; i >= 0; i--) {
        uint64_t a; float b;
        rh_pop(hp, &a, &b);
        cand_slot[(int64_t)li * R + i] = (uint32_t)(a - id_base);
    }
    for (int i = m; i < R; i++) cand_slot[(int64_t)li * R + i] = NO_ID;
    cand_n[li] = m;
}

// h.rescore with one worker (hnsw/search.go:1067-1110): in ascending-id-list
// order, Insert then Pop while Len > k; then extraction.  LDS [k+1] u64 | f32.
__global__ __launch_bounds__(64) void k_pq_rescore_final(const uint32_t* __restrict__ cand_slot,
                                                         const float* __restrict__ candE,
                                                         const int32_t* __restrict__ cand_n,
                                                         const int32_t* __restrict__ qlist, int nlist, int R, int k,
                                                         uint64_t id_base, uint64_t* __restrict__ out_ids,
                                                         float* __restrict__ out_d, int32_t* __restrict__ out_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char qsm[];
    uint64_t* hid = reinterpret_cast<uint64_t*>(qsm);
    float* hd = reinterpret_cast<float*>(hid + (k + 1));
    const int li = blockIdx.x;
    if (li >= nlist || threadIdx.x != 0) return;
    ReplayHeap hp{hid, hd, 0};
    const int n = cand_n[li];
    for (int i = 0; i < n; i++) {
        rh_insert(hp, id_base + cand_slot[(int64_t)li * R + i], candE[(int64_t)li * R + i]);
        if (hp.len > k) { uint64_t a; float b; rh_pop(hp, &a, &b); }
    }
    const int q = qlist[li];
    const int m = hp.len;
    for (int i = m - 1; i >= 0; i--) {
        uint64_t a; float b;
        rh_pop(hp, &a, &b);
        out_ids[(int64_t)q * k + i] = a;
        out_d[(int64_t)q * k + i] = b;
    }
    out_n[q] = m;
}

}  // namespace wv
