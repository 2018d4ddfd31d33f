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
// Codes live in 256-row tiles of 16-segment groups: the 16 code bytes of
// segments [16g, 16g+16) of row r are the uint4 at ((r/256) * G16 + g) * 256 +
// r%256 (G16 = ceil(m/16)), so 64 lanes on consecutive rows read 1 KiB
// contiguous per group (pq_code_word gives the u32 holding segment s).
#pragma once

namespace wv {
namespace {  // internal linkage: each runtime unit compiles the kernels it launches

constexpr int KM_T = 256;  // threads per k-means workgroup; k <= 256 (NewProductQuantizer)

// u32 index of the word holding segment s of row r (byte s % 4)
__host__ __device__ __forceinline__ int64_t pq_code_word(int64_t r, int s, int g16) {
    return ((((r >> 8) * g16 + (s >> 4)) << 8) + (r & 255)) * 4 + ((s >> 2) & 3);
}

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
// rows[slot * ld ...] -> codes[slot * mwp + s/4] byte (s % 4).
// DS > 0: the row's segment is held in registers (compile-time length; the
// AVX-512 kernel differs from AVX2 only for n >= 128, so ds <= 32 needs no
// variant); DS == 0: generic length.
template <int DS>
__global__ __launch_bounds__(256) void k_pq_encode(const float* __restrict__ rows, int64_t ld, int64_t n,
                                                   const uint32_t* __restrict__ slots, int k, int ds,
                                                   const float* __restrict__ centers, int variant,
                                                   uint32_t* __restrict__ codes, int g16) {
    extern __shared__ __attribute__((aligned(16))) float csm[];
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
    if (DS > 0) {
        float xr[DS > 0 ? DS : 1];
#pragma unroll
        for (int j = 0; j < DS; j++) xr[j] = x[j];
        for (int c = 0; c < k; c++) {
            const float d = exact_raw<L2, AVX256, false>(xr, csm + c * DS, DS);
            if (d < mn) { mn = d; idx = (uint32_t)c; }
        }
    } else {
        for (int c = 0; c < k; c++) {
            const float d = l2_seg(x, csm + c * ds, ds, variant);
            if (d < mn) { mn = d; idx = (uint32_t)c; }
        }
    }
    unsigned char* b = reinterpret_cast<unsigned char*>(codes + pq_code_word(slot, s, g16));
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

// ADC over a row tile blockIdx.y for listed query f = blockIdx.x (queries
// fastest: the blocks of one tile run together and share its codes in L2): rows tile0 + 256 r + t,
// r < PQ_RPT.  LUT chunks of PQ_CH segments staged through LDS in segment
// order (the running sums stay in registers, so the fp32 addition order is
// the reference's).  Writes E[f][row] (+inf for invalid rows) and the 256-row
// block minima used by k_replay_scan.
constexpr int PQ_RPT = 8;
constexpr int PQ_CH = 32;
template <int KC>  // KC = ks when 256 (LDS offsets become immediates), 0 = runtime k
__global__ __launch_bounds__(256, 2) void k_pq_adc(const uint32_t* __restrict__ codes, int g16, int m, int kk,
                                                   const uint32_t* __restrict__ valid, int64_t nslots,
                                                   const float* __restrict__ lut, const int32_t* __restrict__ qlist,
                                                   int metric, int64_t ld, float* __restrict__ E,
                                                   float* __restrict__ bmin) {
    extern __shared__ float lsm[];  // [PQ_CH][k]
    __shared__ float red[4][PQ_RPT];
    const int k = KC > 0 ? KC : kk;
    const int t = threadIdx.x;
    const int f = blockIdx.x;
    const int64_t tile0 = (int64_t)blockIdx.y * 256 * PQ_RPT;
    // this block's PQ_RPT 256-row code tiles: uint4 (tile r, group g, lane t) at (r * g16 + g) * 256 + t
    const uint4* cbase = reinterpret_cast<const uint4*>(codes) + (int64_t)blockIdx.y * PQ_RPT * g16 * 256;
    const int64_t rem64 = nslots - tile0;
    const int rem = rem64 < 256 * PQ_RPT ? (int)rem64 : 256 * PQ_RPT;  // rows of this tile that exist
    const float* L = lut + (int64_t)qlist[f] * m * k;
    float sum[PQ_RPT];
#pragma unroll
    for (int r = 0; r < PQ_RPT; r++) sum[r] = 0.f;
    for (int s0 = 0; s0 < m; s0 += PQ_CH) {
        const int ns = m - s0 < PQ_CH ? m - s0 : PQ_CH;
        __syncthreads();
        for (int i = t; i < ns * k; i += 256) lsm[i] = L[(int64_t)s0 * k + i];
        __syncthreads();
#pragma unroll 1
        for (int c16 = 0; c16 < ns; c16 += 16) {
            const float* lc = lsm + c16 * k;
            const int g = (s0 + c16) >> 4;
            const int nv = ns - c16 < 16 ? ns - c16 : 16;
            if (nv == 16) {
#pragma unroll
                for (int rb = 0; rb < PQ_RPT; rb += 4) {
                    uint4 cw[4];
#pragma unroll
                    for (int rr = 0; rr < 4; rr++) {
                        const int r = rb + rr;
                        cw[rr] = 256 * r + t < rem ? cbase[(uint32_t)((r * g16 + g) * 256 + t)] : make_uint4(0u, 0u, 0u, 0u);
                    }
#pragma unroll
                    for (int rr = 0; rr < 4; rr++) {
                        float acc = sum[rb + rr];
                        const uint32_t wv4[4] = {cw[rr].x, cw[rr].y, cw[rr].z, cw[rr].w};
#pragma unroll
                        for (int w = 0; w < 4; w++)
#pragma unroll
                            for (int b = 0; b < 4; b++) acc = acc + lc[(4 * w + b) * k + ((wv4[w] >> (8 * b)) & 0xFFu)];
                        sum[rb + rr] = acc;
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < PQ_RPT; r++) {
                    const uint4 c4 = 256 * r + t < rem ? cbase[(uint32_t)((r * g16 + g) * 256 + t)] : make_uint4(0u, 0u, 0u, 0u);
                    const uint32_t wv4[4] = {c4.x, c4.y, c4.z, c4.w};
                    float acc = sum[r];
#pragma unroll 1
                    for (int j = 0; j < nv; j++) acc = acc + lc[j * k + ((wv4[j >> 2] >> (8 * (j & 3))) & 0xFFu)];
                    sum[r] = acc;
                }
            }
        }
    }
    const int lane = t & 63, wv = t >> 6;
    const int64_t lrem = ld - tile0;
    float* Ef = E + (int64_t)f * ld + tile0;
#pragma unroll
    for (int r = 0; r < PQ_RPT; r++) {
        const int lr = 256 * r + t;
        const int64_t row = tile0 + lr;
        const bool ok = lr < rem && ((valid[row >> 5] >> (row & 31)) & 1u);
        const float e = ok ? pq_wrap(metric, sum[r]) : __builtin_inff();
        if (lr < lrem) Ef[lr] = e;
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

// k_pq_adc for two listed queries per workgroup (f = 2 blockIdx.x, +1): the
// LUT chunk is staged interleaved [segment][code][2 queries], so one
// ds_read_b64 fetches both queries' entries of a code.  A random-code lookup
// is bank-conflict bound (ds_read_b32 and ds_read_b64 are both serviced as
// 2 x 32 lanes with bank = code mod 32): the b64 read pays that
// once per two lookups, and the tile's codes are read once for both queries.
// Per query the fp32 sums keep segment order (bit-identical to k_pq_adc).
// nf = listed queries of this launch; an odd last workgroup runs one query.
// RPT 256-row code tiles per workgroup: PQ_RPT = 8 (16 and 32 spill to scratch
// and ran 4x / 12x slower on C5).
template <int KC, int RPT>
__global__ __launch_bounds__(256, 2) void k_pq_adc2(const uint32_t* __restrict__ codes, int g16, int m, int kk,
                                                    const uint32_t* __restrict__ valid, int64_t nslots,
                                                    const float* __restrict__ lut, const int32_t* __restrict__ qlist,
                                                    int nf, int metric, int64_t ld, float* __restrict__ E,
                                                    float* __restrict__ bmin) {
    extern __shared__ float2 lsm2[];  // [PQ_CH][k] x 2 queries
    __shared__ float red[2][4][RPT];
    const int k = KC > 0 ? KC : kk;
    const int t = threadIdx.x;
    const int f0 = 2 * blockIdx.x;
    const bool two = f0 + 1 < nf;
    const int64_t tile0 = (int64_t)blockIdx.y * 256 * RPT;
    const uint4* cbase = reinterpret_cast<const uint4*>(codes) + (int64_t)blockIdx.y * RPT * g16 * 256;
    const int64_t rem64 = nslots - tile0;
    const int rem = rem64 < 256 * RPT ? (int)rem64 : 256 * RPT;
    const float* L0 = lut + (int64_t)qlist[f0] * m * k;
    const float* L1 = two ? lut + (int64_t)qlist[f0 + 1] * m * k : L0;
    float sa[RPT], sb[RPT];
#pragma unroll
    for (int r = 0; r < RPT; r++) sa[r] = sb[r] = 0.f;
    for (int s0 = 0; s0 < m; s0 += PQ_CH) {
        const int ns = m - s0 < PQ_CH ? m - s0 : PQ_CH;
        __syncthreads();
        for (int i = t; i < ns * k; i += 256) lsm2[i] = make_float2(L0[(int64_t)s0 * k + i], L1[(int64_t)s0 * k + i]);
        __syncthreads();
#pragma unroll 1
        for (int c16 = 0; c16 < ns; c16 += 16) {
            const float2* lc = lsm2 + c16 * k;
            const int g = (s0 + c16) >> 4;
            const int nv = ns - c16 < 16 ? ns - c16 : 16;
            if (nv == 16) {
#pragma unroll
                for (int rb = 0; rb < RPT; rb += 4) {
                    uint4 cw[4];
#pragma unroll
                    for (int rr = 0; rr < 4; rr++) {
                        const int r = rb + rr;
                        cw[rr] = 256 * r + t < rem ? cbase[(uint32_t)((r * g16 + g) * 256 + t)] : make_uint4(0u, 0u, 0u, 0u);
                    }
#pragma unroll
                    for (int rr = 0; rr < 4; rr++) {
                        float a0 = sa[rb + rr], a1 = sb[rb + rr];
                        const uint32_t wv4[4] = {cw[rr].x, cw[rr].y, cw[rr].z, cw[rr].w};
#pragma unroll
                        for (int w = 0; w < 4; w++)
#pragma unroll
                            for (int b = 0; b < 4; b++) {
                                const float2 v = lc[(4 * w + b) * k + ((wv4[w] >> (8 * b)) & 0xFFu)];
                                a0 = a0 + v.x;
                                a1 = a1 + v.y;
                            }
                        sa[rb + rr] = a0;
                        sb[rb + rr] = a1;
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < RPT; r++) {
                    const uint4 c4 = 256 * r + t < rem ? cbase[(uint32_t)((r * g16 + g) * 256 + t)] : make_uint4(0u, 0u, 0u, 0u);
                    const uint32_t wv4[4] = {c4.x, c4.y, c4.z, c4.w};
                    float a0 = sa[r], a1 = sb[r];
#pragma unroll 1
                    for (int j = 0; j < nv; j++) {
                        const float2 v = lc[j * k + ((wv4[j >> 2] >> (8 * (j & 3))) & 0xFFu)];
                        a0 = a0 + v.x;
                        a1 = a1 + v.y;
                    }
                    sa[r] = a0;
                    sb[r] = a1;
                }
            }
        }
    }
    const int lane = t & 63, wv = t >> 6;
    const int64_t lrem = ld - tile0;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        float* Ef = E + (int64_t)(f0 + j) * ld + tile0;
#pragma unroll
        for (int r = 0; r < RPT; r++) {
            const int lr = 256 * r + t;
            const int64_t row = tile0 + lr;
            const bool ok = lr < rem && ((valid[row >> 5] >> (row & 31)) & 1u);
            const float e = ok ? pq_wrap(metric, j ? sb[r] : sa[r]) : __builtin_inff();
            if (E && (j == 0 || two) && lr < lrem) Ef[lr] = e;  // E == nullptr: block minima only
            float mm = e;
            for (int o = 32; o > 0; o >>= 1) mm = fminf(mm, __shfl_xor(mm, o));
            if (lane == 0) red[j][wv][r] = mm;
        }
    }
    __syncthreads();
    if (t < 2 * RPT) {
        const int j = t / RPT, r = t % RPT;
        const int64_t blk = tile0 / 256 + r;
        if ((j == 0 || two) && blk < ld / 256)
            bmin[(int64_t)(f0 + j) * (ld / 256) + blk] =
                fminf(fminf(red[j][0][r], red[j][1][r]), fminf(red[j][2][r], red[j][3][r]));
    }
}

// The minima-only PQ search (no B x N distance matrix): k_pq_adc2 wrote the
// 256-row block minima of every query, k_blk_select listed the blocks whose
// minimum is within (a rounding-size eps of) M = the (R+1)-th smallest block
// minimum -- every block that can hold one of the R+1 smallest ADC distances.
// Per query (one workgroup, thread = row of a candidate block): the ADC
// distance in segment order (bit-identical to k_pq_adc2), the rows with a
// value <= M collected and bitonic-sorted by (value, slot) in LDS.  Strictly
// increasing R+1 smallest values (or all of them when fewer) ARE the worker
// heap's content in its ascending extraction (flat_search.go:96-110: the heap
// keeps the R smallest; distinct values leave no order to the heap layout):
// written as asc[q] for k_pq_finish.  Ties, NaN, more than PQC_MAXB candidate
// blocks or PQC_CAP rows: flag_out[q] = 1 (the exact heap replay decides).
constexpr int PQC_MAXB = 64;
constexpr int PQC_CAP = 1024;
template <int KC>
__global__ __launch_bounds__(256) void k_pq_cand(const uint32_t* __restrict__ codes, int g16, int m, int kk,
                                                 const uint32_t* __restrict__ valid, int64_t nslots,
                                                 const float* __restrict__ lut, const float* __restrict__ bmin,
                                                 int64_t ldb, const uint32_t* __restrict__ cand, int L,
                                                 const int32_t* __restrict__ ncand, const int32_t* __restrict__ sel_flags,
                                                 int R, int metric, uint64_t id_base, uint64_t* __restrict__ asc_ids,
                                                 float* __restrict__ asc_d, int32_t* __restrict__ asc_n,
                                                 int32_t* __restrict__ flag_out) {
    __shared__ float sv[PQC_CAP];
    __shared__ uint32_t ss[PQC_CAP];
    __shared__ int s_cnt, s_bad;
    __shared__ float s_M;
    const int k = KC > 0 ? KC : kk;
    const int q = blockIdx.x;
    const int t = threadIdx.x;
    const int nc = ncand[q];
    if (sel_flags[q] != 0 || nc > PQC_MAXB || R + 1 > 64) {
        if (t == 0) flag_out[q] = 1;
        return;
    }
    if (t < 64) {  // M = the (R+1)-th smallest minimum of the candidate blocks (+inf when fewer)
        float key[1] = {t < nc ? bmin[(int64_t)q * ldb + cand[(int64_t)q * L + t]] : __builtin_inff()};
        uint32_t id[1] = {(uint32_t)t};
        bitonic_sort<1>(key, id, t);
        const float M = __shfl(key[0], R);
        if (t == 0) { s_M = R < nc ? M : __builtin_inff(); s_cnt = 0; s_bad = 0; }
    }
    __syncthreads();
    const float M = s_M;
    const float* Lq = lut + (int64_t)q * m * k;
    const uint4* c4 = reinterpret_cast<const uint4*>(codes);
    for (int j = 0; j < nc; j++) {
        const int64_t b = cand[(int64_t)q * L + j];
        const int64_t row = b * 256 + t;
        if (row >= nslots || !((valid[row >> 5] >> (row & 31)) & 1u)) continue;
        float sum = 0.f;
        for (int g = 0; g < g16; g++) {
            const uint4 cw = c4[(b * g16 + g) * 256 + t];
            const uint32_t w4[4] = {cw.x, cw.y, cw.z, cw.w};
            const int nv = m - 16 * g < 16 ? m - 16 * g : 16;
            for (int jj = 0; jj < nv; jj++) {
                const int sgm = 16 * g + jj;
                sum = sum + Lq[(int64_t)sgm * k + ((w4[jj >> 2] >> (8 * (jj & 3))) & 0xFFu)];
            }
        }
        const float e = pq_wrap(metric, sum);
        if (e != e) s_bad = 1;
        if (e <= M) {
            const int pos = atomicAdd(&s_cnt, 1);
            if (pos < PQC_CAP) { sv[pos] = e; ss[pos] = (uint32_t)row; }
        }
    }
    __syncthreads();
    const int n = s_cnt;
    if (n > PQC_CAP || s_bad) {
        if (t == 0) flag_out[q] = 1;
        return;
    }
    int p2 = 1;
    while (p2 < n) p2 <<= 1;
    for (int i = n + t; i < p2; i += 256) { sv[i] = __builtin_inff(); ss[i] = NO_ID; }
    __syncthreads();
    for (int k2 = 2; k2 <= p2; k2 <<= 1)
        for (int jj = k2 >> 1; jj > 0; jj >>= 1) {
            for (int i = t; i < p2; i += 256) {
                const int ixj = i ^ jj;
                if (ixj > i) {
                    const float a = sv[i], c = sv[ixj];
                    const uint32_t ia = ss[i], ic = ss[ixj];
                    const bool gt = a > c || (a == c && ia > ic);
                    if ((i & k2) == 0 ? gt : !gt) { sv[i] = c; sv[ixj] = a; ss[i] = ic; ss[ixj] = ia; }
                }
            }
            __syncthreads();
        }
    const int mm = n < R + 1 ? n : R + 1;
    if (t == 0) {
        bool strict = true;
        for (int i = 1; i < mm; i++) strict &= sv[i - 1] < sv[i];
        flag_out[q] = strict ? 0 : 1;
        asc_n[q] = n < R ? n : R;
    }
    if (t < R && t < n) {
        asc_ids[(int64_t)q * R + t] = id_base + ss[t];
        asc_d[(int64_t)q * R + t] = sv[t];
    }
}

// flatSearch tail (hnsw/flat_search.go:96-141 with one worker): the worker
// heap's ascending extraction asc[li][0..n) is popped max-first
// (= reverse order) into the result heap via addResult (:214-224).
// rescore == 0: extract (fill from the back) -> out rows q = qlist[li].
// rescore == 1: (trim > 0: Pop while Len > trim) pop all into ascending ids
//               (search.go:1048-1064) -> cand slots
//               [li][R] for k_rescore; cand_n[li].
// Dynamic LDS: [R] u64 | [R] f32.
__global__ __launch_bounds__(64) void k_pq_finish(const uint64_t* __restrict__ asc_ids,
                                                  const float* __restrict__ asc_d, const int32_t* __restrict__ asc_n,
                                                  const int32_t* __restrict__ qlist, int nlist, int R, int k,
                                                  int rescore, uint64_t id_base, uint64_t* __restrict__ out_ids,
                                                  float* __restrict__ out_d, int32_t* __restrict__ out_n,
                                                  uint32_t* __restrict__ cand_slot, int32_t* __restrict__ cand_n,
                                                  int trim, uint64_t* __restrict__ cand_ids = nullptr) {
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
    // SQ / RQ (search.go:1048-1057): Pop while Len > RescoreLimit (>= k)
    if (trim > 0)
        while (hp.len > trim) { uint64_t a; float b; rh_pop(hp, &a, &b); }
    const int mt = hp.len;
    for (int i = mt - 1; i >= 0; i--) {
        uint64_t a; float b;
        rh_pop(hp, &a, &b);
        if (cand_ids) cand_ids[(int64_t)li * R + i] = a;  // sharded: global ids (any shard)
        else cand_slot[(int64_t)li * R + i] = (uint32_t)(a - id_base);
    }
    for (int i = mt; i < R; i++) {
        if (cand_ids) cand_ids[(int64_t)li * R + i] = ~0ull;
        else cand_slot[(int64_t)li * R + i] = NO_ID;
    }
    cand_n[li] = mt;
}

// h.rescore with one worker (hnsw/search.go:1067-1110): in ascending-id-list
// order, Insert then Pop while Len > k; then extraction.  LDS [k+1] u64 | f32.
__global__ __launch_bounds__(64) void k_pq_rescore_final(const uint32_t* __restrict__ cand_slot,
                                                         const float* __restrict__ candE,
                                                         const int32_t* __restrict__ cand_n,
                                                         const int32_t* __restrict__ qlist, int nlist, int R, int k,
                                                         uint64_t id_base, uint64_t* __restrict__ out_ids,
                                                         float* __restrict__ out_d, int32_t* __restrict__ out_n,
                                                         const uint64_t* __restrict__ cand_ids = nullptr,
                                                         int world = 1, uint64_t id_stride = 0) {
    extern __shared__ __attribute__((aligned(16))) unsigned char qsm[];
    uint64_t* hid = reinterpret_cast<uint64_t*>(qsm);
    float* hd = reinterpret_cast<float*>(hid + (k + 1));
    const int li = blockIdx.x;
    if (li >= nlist || threadIdx.x != 0) return;
    ReplayHeap hp{hid, hd, 0};
    const int n = cand_n[li];
    for (int i = 0; i < n; i++) {
        // sharded (cand_ids): candE is [world][nlist][R], each shard's exact distances of
        // the ids it holds; the entry of id comes from shard min(id / id_stride, world - 1)
        uint64_t id;
        float e;
        if (cand_ids) {
            id = cand_ids[(int64_t)li * R + i];
            uint64_t w = id_stride ? id / id_stride : 0;
            w = w < (uint64_t)world ? w : (uint64_t)world - 1;
            e = candE[((int64_t)w * nlist + li) * R + i];
        } else {
            id = id_base + cand_slot[(int64_t)li * R + i];
            e = candE[(int64_t)li * R + i];
        }
        rh_insert(hp, id, e);
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


// ---------------------------------------------------------------------------
// k_pq_adc3: the ADC block minima with the queries on the lanes.  A random
// code per lane (k_pq_adc2: rows on the lanes) makes every LUT read a bank
// conflict lottery; here the 32 lanes of a ds_read_b64 group read ONE row's
// code for 64 queries (2 per lane): 256 contiguous bytes, conflict-free, and
// one v_pk_add_f32 adds both.  Workgroup: 8 waves x 128 rows = 1024 rows, 64
// queries (query group blockIdx.y); lane (p = lane & 31, h = lane >> 5) keeps
// the sums of queries 2p, 2p+1 for rows 128 w + 2 i + h, i < 64 (128 VGPRs).
// Per segment s (in order: each fp32 sum is the reference's segment-order
// sum, bit-identical to k_pq_adc / k_pq_adc2):
//   LUT slot s & 1 <- lutg[G][s] (64 KiB: [code][64 queries]) by LDS-DMA,
//   issued one segment ahead (two 64 KiB slots);
//   codes of the segment's 1024 rows from LDS ([16 segments][1024 rows] bytes,
//   restaged every 16 segments from the 256-row code tiles), eight rows per
//   broadcast ds_read_b64; the LUT address = v_perm(code byte, lane base).
// LDS reads are inline asm with counted lgkmcnt waits (the DMA would make the
// compiler drain vmcnt before every LDS read it sees).  Writes the 256-row
// block minima only (bmin[q][blk], +inf for invalid rows; K = 256).
// ---------------------------------------------------------------------------
typedef float pq_f2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* pq_lds_t;

// lutg[G][s][c][j] = lut[min(64 G + j, nq - 1)][s][c]
__global__ void k_pq_lut_group(const float* __restrict__ lut, int nq, int m, int K, int64_t total,
                               float* __restrict__ lutg) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int j = (int)(i & 63);
    const int64_t r = i >> 6;
    const int c = (int)(r % K);
    const int64_t gs = r / K;
    const int sg = (int)(gs % m);
    const int64_t G = gs / m;
    int64_t q = G * 64 + j;
    q = q < nq ? q : nq - 1;
    lutg[i] = lut[(q * m + sg) * K + c];
}

constexpr int PQ3_ROWS = 1024;
constexpr int PQ3_SLOT = 65536;                          // one segment's LUT: 256 codes x 64 queries x 4 B
constexpr int PQ3_LDS = 2 * PQ3_SLOT + 16 * PQ3_ROWS;    // two LUT slots + the codes of 16 segments

__device__ __forceinline__ uint2 pq3_ld8(unsigned a) {
    uint2 v;
    asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
template <int N>
__device__ __forceinline__ void pq3_wait_lgkm() {
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

// DBG (timing experiments only, wrong results): 1 = no LUT DMA in the loop, 2 = no per-segment wait + barrier
template <int DBG>
__global__ __launch_bounds__(512, 1) void k_pq_adc3(const uint32_t* __restrict__ codes, int g16, int m,
                                                    const uint32_t* __restrict__ valid, int64_t nslots,
                                                    const float* __restrict__ lutg, int nq, int metric,
                                                    int64_t nblk_ld, float* __restrict__ bmin) {
    __shared__ __attribute__((aligned(16))) unsigned char sm[PQ3_LDS];  // the kernel's only LDS: address 0
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int p = lane & 31, h = lane >> 5;
    const int64_t row0 = (int64_t)blockIdx.x * PQ3_ROWS;
    const int G = blockIdx.y;
    const unsigned smb = (unsigned)(size_t)((pq_lds_t)sm);
    const unsigned cod = smb + 2 * PQ3_SLOT;
    // the LUT address of code c in slot b: byte 0 = 8 p, byte 1 = c, byte 2 = b (slots at 0 / 64 KiB)
    const uint32_t selA = 0x0c020000u | ((4u + (uint32_t)h) << 8);       // code byte h   (row pairs 4j, 4j+2)
    const uint32_t selB = 0x0c020000u | ((4u + 2u + (uint32_t)h) << 8);  // code byte 2+h (row pairs 4j+1, 4j+3)
    const uint32_t lb0 = smb + 8u * (uint32_t)p;
    const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(lutg + (int64_t)G * m * 256 * 64), (short)0, -1, 0x00020000);
    auto dma = [&](int sg) {  // LUT segment sg -> slot sg & 1: 8 KiB per wave
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const unsigned off = (unsigned)(i * 8192 + w * 1024);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(lrs, (pq_lds_t)(size_t)(smb + (unsigned)((sg & 1) * PQ3_SLOT) + off),
                                                     16, (uint32_t)(16 * lane), (uint32_t)sg * PQ3_SLOT + off, 0, 0);
        }
    };
    // this thread's two rows (2 tid, 2 tid + 1) of the chunk: code uint4s of a 16-segment group
    auto load_codes = [&](int g, uint4& c0, uint4& c1) {
        const uint4* cb = reinterpret_cast<const uint4*>(codes);
        const int64_t r = row0 + 2 * tid;
        c0 = r < nslots ? cb[((r >> 8) * g16 + g) * 256 + (r & 255)] : make_uint4(0u, 0u, 0u, 0u);
        c1 = r + 1 < nslots ? cb[(((r + 1) >> 8) * g16 + g) * 256 + ((r + 1) & 255)] : make_uint4(0u, 0u, 0u, 0u);
    };
    // [16][1024] bytes: segment k's byte of rows 2 tid, 2 tid + 1 as one u16
    auto store_codes = [&](const uint4& c0, const uint4& c1) {
        const uint32_t a[4] = {c0.x, c0.y, c0.z, c0.w}, b[4] = {c1.x, c1.y, c1.z, c1.w};
#pragma unroll
        for (int k = 0; k < 16; k++) {
            // low byte: row 2 tid's code k, high byte: row 2 tid + 1's
            const uint32_t v = __builtin_amdgcn_perm(b[k >> 2], a[k >> 2], 0x0c0c0000u | (uint32_t)(k & 3) | ((uint32_t)(4 + (k & 3)) << 8));
            *(__attribute__((address_space(3))) uint16_t*)(size_t)(cod + (unsigned)(k * PQ3_ROWS + 2 * tid)) = (uint16_t)v;
        }
    };
    pq_f2 sum[64];
#pragma unroll
    for (int i = 0; i < 64; i++) sum[i] = pq_f2{0.f, 0.f};
    uint4 nc0, nc1;
    load_codes(0, nc0, nc1);
    dma(0);
    for (int s = 0; s < m; s++) {
        if ((s & 15) == 0) {
            // the group's codes: every wave is past the previous group's reads
            __syncthreads();
            store_codes(nc0, nc1);
            if (s + 16 < m) load_codes((s >> 4) + 1, nc0, nc1);
        }
        if (DBG != 2) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();  // slot s & 1 landed for every wave; slot (s + 1) & 1 is free
        }
        if (s + 1 < m && DBG != 1) dma(s + 1);
        // 16 broadcast reads: the codes of this wave's 128 rows
        const unsigned crow = cod + (unsigned)((s & 15) * PQ3_ROWS + w * 128);
        uint2 cw[16];
#pragma unroll
        for (int j = 0; j < 16; j++) cw[j] = pq3_ld8(crow + 8 * j);
        pq3_wait_lgkm<0>();
        const uint32_t lb = lb0 + (uint32_t)((s & 1) * PQ3_SLOT);
        // 64 row pairs in batches of 8: batch t + 1's reads in flight while t's are added
        uint2 v[2][8];
        auto issue = [&](int t, uint2 (&dst)[8]) {
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int i = 8 * t + u;          // row pair: code dword (i >> 1) & 1 of cw[i >> 2]
                const uint2 c = cw[i >> 2];
                const uint32_t word = ((i >> 1) & 1) ? c.y : c.x;
                dst[u] = pq3_ld8(__builtin_amdgcn_perm(word, lb, (i & 1) ? selB : selA));
            }
        };
        issue(0, v[0]);
#pragma unroll
        for (int t = 0; t < 8; t++) {
            if (t + 1 < 8) issue(t + 1, v[(t + 1) & 1]);
#pragma unroll
            for (int u = 0; u < 8; u++) {
                if (t + 1 < 8) {
                    switch (u) {
                    case 0: asm volatile("s_waitcnt lgkmcnt(15)" : "+v"(v[t & 1][0])); break;
                    case 1: asm volatile("s_waitcnt lgkmcnt(14)" : "+v"(v[t & 1][1])); break;
                    case 2: asm volatile("s_waitcnt lgkmcnt(13)" : "+v"(v[t & 1][2])); break;
                    case 3: asm volatile("s_waitcnt lgkmcnt(12)" : "+v"(v[t & 1][3])); break;
                    case 4: asm volatile("s_waitcnt lgkmcnt(11)" : "+v"(v[t & 1][4])); break;
                    case 5: asm volatile("s_waitcnt lgkmcnt(10)" : "+v"(v[t & 1][5])); break;
                    case 6: asm volatile("s_waitcnt lgkmcnt(9)" : "+v"(v[t & 1][6])); break;
                    default: asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(v[t & 1][7])); break;
                    }
                } else {
                    switch (u) {
                    case 0: asm volatile("s_waitcnt lgkmcnt(7)" : "+v"(v[t & 1][0])); break;
                    case 1: asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(v[t & 1][1])); break;
                    case 2: asm volatile("s_waitcnt lgkmcnt(5)" : "+v"(v[t & 1][2])); break;
                    case 3: asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(v[t & 1][3])); break;
                    case 4: asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(v[t & 1][4])); break;
                    case 5: asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(v[t & 1][5])); break;
                    case 6: asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(v[t & 1][6])); break;
                    default: asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[t & 1][7])); break;
                    }
                }
                const uint2 x = v[t & 1][u];
                sum[8 * t + u] += pq_f2{__uint_as_float(x.x), __uint_as_float(x.y)};
            }
        }
    }
    // per query: minimum over this wave's 128 rows (invalid rows +inf), then the
    // two waves of a 256-row block through LDS (after every LUT read is done)
    const int64_t rw = row0 + (int64_t)w * 128;
    uint32_t vw[4];
#pragma unroll
    for (int k = 0; k < 4; k++) vw[k] = rw + 32 * k < nslots ? valid[(rw >> 5) + k] : 0u;
    float m0 = __builtin_inff(), m1 = __builtin_inff();
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const int r = 2 * i + h;  // row within the wave's 128
        const bool ok = rw + r < nslots && ((vw[r >> 5] >> (r & 31)) & 1u);
        if (ok) {
            m0 = fminf(m0, pq_wrap(metric, sum[i].x));
            m1 = fminf(m1, pq_wrap(metric, sum[i].y));
        }
    }
    m0 = fminf(m0, __shfl_xor(m0, 32));
    m1 = fminf(m1, __shfl_xor(m1, 32));
    __syncthreads();
    float* red = reinterpret_cast<float*>(sm);  // [8 waves][64 queries]
    if (h == 0) {
        red[w * 64 + 2 * p] = m0;
        red[w * 64 + 2 * p + 1] = m1;
    }
    __syncthreads();
    if (tid < 256) {  // block b = tid >> 6 (waves 2b, 2b + 1), query j = tid & 63
        const int b = tid >> 6, j = tid & 63;
        const int64_t q = (int64_t)G * 64 + j;
        const int64_t blk = row0 / 256 + b;
        if (q < nq && blk < nblk_ld) bmin[q * nblk_ld + blk] = fminf(red[(2 * b) * 64 + j], red[(2 * b + 1) * 64 + j]);
    }
}

// ---------------------------------------------------------------------------
// k_pq_adc4: k_pq_adc3 with 16-byte LUT reads.  Same workgroup (8 waves x 128
// rows, 64 queries), same LDS image (two [code][64 queries] LUT slots + the
// [16][1024] code bytes) and the same LUT DMA; lane (qd = lane & 15, r = lane
// >> 4) keeps the sums of queries 4 qd .. 4 qd + 3 for the rows 128 w + 4 i + r,
// i < 32 (128 VGPRs).  One ds_read_b128 reads four rows' LUT entries for all
// 64 queries: its 16-lane groups ({0-3,12-15,20-27}, ...) hold 16 distinct
// query quads, so their banks (4 qd .. 4 qd + 3) never collide whatever the
// codes.  Per 256 lookups: one b128 read (4 LDS cycles), one v_perm (the
// address: byte 0 = 16 qd, byte 1 = row r's code, byte 2 = slot) and two
// v_pk_add_f32 — k_pq_adc3 spends two b64 reads, two v_perm and two pk_adds.
// Each sum is the same segment-order fp32 sum: results are bit-identical.
// ---------------------------------------------------------------------------
typedef float pq_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ pq_f4 pq4_ld16(unsigned a) {
    pq_f4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
    return v;
}

// DBG (timing experiment only, wrong results): 1 = no LUT DMA in the loop
template <int DBG>
__global__ __launch_bounds__(512, 1) void k_pq_adc4(const uint32_t* __restrict__ codes, int g16, int m,
                                                    const uint32_t* __restrict__ valid, int64_t nslots,
                                                    const float* __restrict__ lutg, int nq, int metric,
                                                    int64_t nblk_ld, float* __restrict__ bmin) {
    __shared__ __attribute__((aligned(16))) unsigned char sm[PQ3_LDS];  // the kernel's only LDS: address 0
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int qd = lane & 15, r = lane >> 4;
    const int64_t row0 = (int64_t)blockIdx.x * PQ3_ROWS;
    const int G = blockIdx.y;
    const unsigned smb = (unsigned)(size_t)((pq_lds_t)sm);
    const unsigned cod = smb + 2 * PQ3_SLOT;
    // byte 0 = 16 qd (lb), byte 1 = code byte r of the word, byte 2 = slot (lb), byte 3 = 0
    const uint32_t sel = 0x0c020000u | ((4u + (uint32_t)r) << 8);
    const uint32_t lb0 = smb + 16u * (uint32_t)qd;
    const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(lutg + (int64_t)G * m * 256 * 64), (short)0, -1, 0x00020000);
    auto dma = [&](int sg) {  // LUT segment sg -> slot sg & 1: 8 KiB per wave
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const unsigned off = (unsigned)(i * 8192 + w * 1024);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(lrs, (pq_lds_t)(size_t)(smb + (unsigned)((sg & 1) * PQ3_SLOT) + off),
                                                     16, (uint32_t)(16 * lane), (uint32_t)sg * PQ3_SLOT + off, 0, 0);
        }
    };
    auto load_codes = [&](int g, uint4& c0, uint4& c1) {
        const uint4* cb = reinterpret_cast<const uint4*>(codes);
        const int64_t rr = row0 + 2 * tid;
        c0 = rr < nslots ? cb[((rr >> 8) * g16 + g) * 256 + (rr & 255)] : make_uint4(0u, 0u, 0u, 0u);
        c1 = rr + 1 < nslots ? cb[(((rr + 1) >> 8) * g16 + g) * 256 + ((rr + 1) & 255)] : make_uint4(0u, 0u, 0u, 0u);
    };
    auto store_codes = [&](const uint4& c0, const uint4& c1) {
        const uint32_t a[4] = {c0.x, c0.y, c0.z, c0.w}, b[4] = {c1.x, c1.y, c1.z, c1.w};
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t v = __builtin_amdgcn_perm(b[k >> 2], a[k >> 2], 0x0c0c0000u | (uint32_t)(k & 3) | ((uint32_t)(4 + (k & 3)) << 8));
            *(__attribute__((address_space(3))) uint16_t*)(size_t)(cod + (unsigned)(k * PQ3_ROWS + 2 * tid)) = (uint16_t)v;
        }
    };
    pq_f2 sa[32], sb[32];  // queries (4 qd, 4 qd + 1) and (4 qd + 2, 4 qd + 3) of row 4 i + r
#pragma unroll
    for (int i = 0; i < 32; i++) {
        sa[i] = pq_f2{0.f, 0.f};
        sb[i] = pq_f2{0.f, 0.f};
    }
    uint4 nc0, nc1;
    load_codes(0, nc0, nc1);
    dma(0);
    for (int s = 0; s < m; s++) {
        if ((s & 15) == 0) {
            __syncthreads();
            store_codes(nc0, nc1);
            if (s + 16 < m) load_codes((s >> 4) + 1, nc0, nc1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // slot s & 1 landed for every wave; slot (s + 1) & 1 is free
        if (s + 1 < m && DBG != 1) dma(s + 1);
        const unsigned crow = cod + (unsigned)((s & 15) * PQ3_ROWS + w * 128);
        uint2 cw[16];
#pragma unroll
        for (int j = 0; j < 16; j++) cw[j] = pq3_ld8(crow + 8 * j);
        pq3_wait_lgkm<0>();
        const uint32_t lb = lb0 + (uint32_t)((s & 1) * PQ3_SLOT);
        // 32 row quads in batches of 4: batch t + 1's reads in flight while t's are added
        pq_f4 v[2][4];
        auto issue = [&](int t, pq_f4 (&dst)[4]) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = 4 * t + u;  // rows 4 i .. 4 i + 3: dword i & 1 of cw[i >> 1]
                const uint2 c = cw[i >> 1];
                dst[u] = pq4_ld16(__builtin_amdgcn_perm((i & 1) ? c.y : c.x, lb, sel));
            }
        };
        issue(0, v[0]);
#pragma unroll
        for (int t = 0; t < 8; t++) {
            if (t + 1 < 8) issue(t + 1, v[(t + 1) & 1]);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (t + 1 < 8) {
                    switch (u) {
                    case 0: asm volatile("s_waitcnt lgkmcnt(7)" : "+v"(v[t & 1][0])); break;
                    case 1: asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(v[t & 1][1])); break;
                    case 2: asm volatile("s_waitcnt lgkmcnt(5)" : "+v"(v[t & 1][2])); break;
                    default: asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(v[t & 1][3])); break;
                    }
                } else {
                    switch (u) {
                    case 0: asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(v[t & 1][0])); break;
                    case 1: asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(v[t & 1][1])); break;
                    case 2: asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(v[t & 1][2])); break;
                    default: asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[t & 1][3])); break;
                    }
                }
                const pq_f4 x = v[t & 1][u];
                sa[4 * t + u] += pq_f2{x.x, x.y};
                sb[4 * t + u] += pq_f2{x.z, x.w};
            }
        }
    }
    // per query: minimum over this wave's 128 rows (invalid rows +inf), across the
    // four row lanes r, then the two waves of a 256-row block through LDS
    const int64_t rw = row0 + (int64_t)w * 128;
    uint32_t vw[4];
#pragma unroll
    for (int k = 0; k < 4; k++) vw[k] = rw + 32 * k < nslots ? valid[(rw >> 5) + k] : 0u;
    float mq[4] = {__builtin_inff(), __builtin_inff(), __builtin_inff(), __builtin_inff()};
#pragma unroll
    for (int i = 0; i < 32; i++) {
        const int rr = 4 * i + r;  // row within the wave's 128
        const bool ok = rw + rr < nslots && ((vw[rr >> 5] >> (rr & 31)) & 1u);
        if (ok) {
            mq[0] = fminf(mq[0], pq_wrap(metric, sa[i].x));
            mq[1] = fminf(mq[1], pq_wrap(metric, sa[i].y));
            mq[2] = fminf(mq[2], pq_wrap(metric, sb[i].x));
            mq[3] = fminf(mq[3], pq_wrap(metric, sb[i].y));
        }
    }
#pragma unroll
    for (int c = 0; c < 4; c++) {
        mq[c] = fminf(mq[c], __shfl_xor(mq[c], 16));
        mq[c] = fminf(mq[c], __shfl_xor(mq[c], 32));
    }
    __syncthreads();
    float* red = reinterpret_cast<float*>(sm);  // [8 waves][64 queries]
    if (r == 0) {
#pragma unroll
        for (int c = 0; c < 4; c++) red[w * 64 + 4 * qd + c] = mq[c];
    }
    __syncthreads();
    if (tid < 256) {  // block b = tid >> 6 (waves 2b, 2b + 1), query j = tid & 63
        const int b = tid >> 6, j = tid & 63;
        const int64_t q = (int64_t)G * 64 + j;
        const int64_t blk = row0 / 256 + b;
        if (q < nq && blk < nblk_ld) bmin[q * nblk_ld + blk] = fminf(red[(2 * b) * 64 + j], red[(2 * b + 1) * 64 + j]);
    }
}

// ---------------------------------------------------------------------------
// PQ block keys on the integer matrix cores.  For l2-squared
// the ADC sum is ||q - x~||^2 up to fp32 rounding (LUT entries and their sum
// are sums of non-negative terms: relative error <= gamma_{m + ds + 3}), x~ =
// the row's decoded centroids.  The distance is translation invariant, so the
// reconstruction is stored centred, x_c = fl(x~ - mu) with mu the per-dimension
// mean of the codebook, as an int8 plane (k_block_q8: per-32-row-block
// scales, residual maxima); the queries are centred the same way.  Centred
// vectors are 2x shorter on U[0,1) data, which is what makes the int8 key's
// Cauchy-Schwarz bound (|q^| R + |q - q^| H ..., qs_eps) narrow enough to cut
// 10M rows to ~100 candidate blocks per query.
// ---------------------------------------------------------------------------

// rows [row0, row0 + n) decoded and centred into out[(r - row0) * dpad + c]
// (fp32, zero padded), n2[r] = sum of squares (fp32), maxima[4] = max n2
// (float bits); one wave per row
__global__ __launch_bounds__(256) void k_pq_decode_center(const uint32_t* __restrict__ codes, int g16, int m, int ds,
                                                          int K, const float* __restrict__ centers,
                                                          const float* __restrict__ mu, int64_t row0, int64_t n,
                                                          int dims, int dpad, float* __restrict__ out,
                                                          float* __restrict__ n2, uint32_t* __restrict__ maxima) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const int64_t r = row0 + i;
    const unsigned char* cb = reinterpret_cast<const unsigned char*>(codes);
    float ss = 0.f;
    for (int c = lane; c < dpad; c += 64) {
        float v = 0.f;
        if (c < dims) {
            const int sg = c / ds, e = c - sg * ds;
            const int code = cb[pq_code_word(r, sg, g16) * 4 + (sg & 3)];
            v = centers[((int64_t)sg * K + code) * ds + e] - mu[c];
        }
        out[i * dpad + c] = v;
        ss = fmaf(v, v, ss);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    if (lane == 0) {
        n2[r] = ss;
        atomicMax(&maxima[4], __float_as_uint(ss));
    }
}

// centred queries: Qc[q] = fl(Qn[q] - mu) (zero padding rows q >= nq and
// columns c >= dims), qinfo[q] = (|q_c|^2, 0, 0, non-finite); wave per query
__global__ __launch_bounds__(256) void k_pq_center_queries(const float* __restrict__ Qn, int dpad, int dims,
                                                           const float* __restrict__ mu, int64_t nq, int64_t nq_pad,
                                                           float* __restrict__ Qc, float4* __restrict__ qinfo) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq_pad) return;
    float ss = 0.f;
    bool bad = false;
    for (int c = lane; c < dpad; c += 64) {
        const float v = (q < nq && c < dims) ? Qn[q * dpad + c] - mu[c] : 0.f;
        Qc[q * dpad + c] = v;
        ss = fmaf(v, v, ss);
        bad |= !__builtin_isfinite(v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    bad = __any(bad);
    if (lane == 0) qinfo[q] = make_float4(ss, 0.f, 0.f, (bad || !(ss < 1e30f)) ? 1.f : 0.f);
}

// the exact ADC distance (the reference's segment-order fp32 sum) of every
// valid row of query q's candidate 32-row blocks (k_blk_select(_f) lists:
// cand[q][L], ncand[q]), the rows below cap[q] kept and sorted by (distance,
// slot).  The R + 1 smallest distances are among them (the select's proof
// with eps >= |A - ADC|); strictly increasing -> they are the worker heap's
// content and its ascending extraction; else, or a list overflow (sel_flags),
// more than PQC_CAP rows below the cap or a NaN, flag_out[q] = 1 (the full
// replay resolves q).  Workgroup per query, 8 blocks x 32 rows per pass;
// fmask (k_q8_filt_bm survivor masks [q][L]) skips rows whose int8 bound
// already reaches the cap; qlist / qcount: the listed queries only.
template <int KC>
__global__ __launch_bounds__(256) void k_pq_cand8(const uint32_t* __restrict__ codes, int g16, int m, int kk,
                                                  const uint32_t* __restrict__ valid, int64_t nslots,
                                                  const float* __restrict__ lut, const uint32_t* __restrict__ cand,
                                                  int L, const int32_t* __restrict__ ncand,
                                                  const int32_t* __restrict__ sel_flags, const float* __restrict__ cap,
                                                  int R, int metric, uint64_t id_base, uint64_t* __restrict__ asc_ids,
                                                  float* __restrict__ asc_d, int32_t* __restrict__ asc_n,
                                                  int32_t* __restrict__ flag_out, const uint32_t* __restrict__ fmask,
                                                  const int32_t* __restrict__ qlist, const uint32_t* __restrict__ qcount) {
    __shared__ float sv[PQC_CAP];
    __shared__ uint32_t ss[PQC_CAP];
    __shared__ int s_cnt, s_bad;
    const int k = KC > 0 ? KC : kk;
    int q = blockIdx.x;
    if (qlist) {  // a second pass over the listed queries (qcount[1] of them)
        if ((uint32_t)q >= qcount[1]) return;
        q = qlist[q];
    }
    const int t = threadIdx.x;
    if (sel_flags[q] != 0) {
        if (t == 0) flag_out[q] = 1;
        return;
    }
    if (t == 0) { s_cnt = 0; s_bad = 0; }
    __syncthreads();
    const int nc = ncand[q];
    const float capq = cap[q];
    const float* Lq = lut + (int64_t)q * m * k;
    const unsigned char* cb = reinterpret_cast<const unsigned char*>(codes);
    for (int j0 = 0; j0 < nc; j0 += 8) {
        const int j = j0 + (t >> 5);
        if (j >= nc) break;
        const int64_t row = (int64_t)cand[(int64_t)q * L + j] * 32 + (t & 31);
        if (row >= nslots || !((valid[row >> 5] >> (row & 31)) & 1u)) continue;
        // the block-major int8 row bound (k_q8_filt_bm): a row whose A_row - eps
        // reaches the cap has an ADC >= cap, which the list never keeps
        if (fmask && !((fmask[(int64_t)q * L + j] >> (t & 31)) & 1u)) continue;
        float sum = 0.f;
        for (int g = 0; g < g16; g++) {
            const uint4 cw = *reinterpret_cast<const uint4*>(cb + ((((row >> 8) * g16 + g) << 8) + (row & 255)) * 16);
            const uint32_t w4[4] = {cw.x, cw.y, cw.z, cw.w};
            const int nv = m - 16 * g < 16 ? m - 16 * g : 16;
            float lv[16];
#pragma unroll
            for (int jj = 0; jj < 16; jj++)
                lv[jj] = jj < nv ? Lq[(int64_t)(16 * g + jj) * k + ((w4[jj >> 2] >> (8 * (jj & 3))) & 0xFFu)] : 0.f;
            for (int jj = 0; jj < nv; jj++) sum = sum + lv[jj];
        }
        const float e = pq_wrap(metric, sum);
        if (e != e) s_bad = 1;
        if (e < capq) {
            const int pos = atomicAdd(&s_cnt, 1);
            if (pos < PQC_CAP) { sv[pos] = e; ss[pos] = (uint32_t)row; }
        }
    }
    __syncthreads();
    const int n = s_cnt;
    if (n > PQC_CAP || s_bad) {
        if (t == 0) flag_out[q] = 1;
        return;
    }
    int p2 = 1;
    while (p2 < n) p2 <<= 1;
    for (int i = n + t; i < p2; i += 256) { sv[i] = __builtin_inff(); ss[i] = NO_ID; }
    __syncthreads();
    for (int k2 = 2; k2 <= p2; k2 <<= 1)
        for (int jj = k2 >> 1; jj > 0; jj >>= 1) {
            for (int i = t; i < p2; i += 256) {
                const int ixj = i ^ jj;
                if (ixj > i) {
                    const float a = sv[i], c = sv[ixj];
                    const uint32_t ia = ss[i], ic = ss[ixj];
                    const bool gt = a > c || (a == c && ia > ic);
                    if ((i & k2) == 0 ? gt : !gt) { sv[i] = c; sv[ixj] = a; ss[i] = ic; ss[ixj] = ia; }
                }
            }
            __syncthreads();
        }
    const int mm = n < R + 1 ? n : R + 1;
    if (t == 0) {
        bool strict = true;
        for (int i = 1; i < mm; i++) strict &= sv[i - 1] < sv[i];
        flag_out[q] = strict ? 0 : 1;
        asc_n[q] = n < R ? n : R;
    }
    for (int i = t; i < R && i < n; i += 256) {
        asc_ids[(int64_t)q * R + i] = id_base + ss[i];
        asc_d[(int64_t)q * R + i] = sv[i];
    }
}

}  // namespace
}  // namespace wv
