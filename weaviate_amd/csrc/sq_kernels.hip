// sq_kernels.hip -- the HNSW compressor distancers of hnsw.flatSearch
// (hnsw/flat_search.go:28-141) that the flat index does not have: scalar
// quantization (compressionhelpers/scalar_quantization.go) and the BQ
// compressor's HammingBitwise as a materialised distance row.
//
//   k_sq_encode   ScalarQuantizer.Encode (:124-137): per element codeFor
//                 (:114-122) in float32, then the 8-byte tail (big-endian sum
//                 and sum of squares of the codes) kept as a uint2 per row.
//   k_sq_dist     DistanceBetweenCompressedVectors (:45-57): the exact
//                 uint32 byte dot product (v_dot4_u32_u8, == dotByteImpl);
//                 l2SquaredByteImpl = sum2_x + sum2_y - 2 dot (exact integers);
//                 then the reference's float32 expression, unfused.
//   k_bq_dist     BinaryQuantizer.DistanceBetweenCompressedVectors =
//                 distancer.HammingBitwise (binary_quantization.go:53-55).
// Both distance kernels write E[f][slot] and 256-row block minima like
// k_rq8_dist (rq_emit), consumed by k_replay_scan (the worker heap).
//
// Layouts: SQ data codes as rq-8 (256-row tiles of 16-byte chunks, Dq =
// round_up(d, 16) zero padded: zero bytes add nothing to the dot product and
// the sums cover the d real codes); query codes group-tiled (RQ_QPB queries).
#pragma once

namespace wv {
namespace {  // internal linkage: each runtime unit compiles the kernels it launches

constexpr float SQ_CODES = 255.0f;  // codes (scalar_quantization.go:24)

// codeFor (scalar_quantization.go:114-122): float32 (x - b) * codes / a, then
// math.Floor in float64 and the byte conversion (NaN -> 0, as cvttsd2si's
// integer indefinite truncated to a byte)
__device__ __forceinline__ uint32_t sq_code_for(float x, float a, float b) {
    if (x < b) return 0u;
    if (x - b > a) return 255u;
    float t = x - b;
    t = t * SQ_CODES;
    t = t / a;
    if (!(t == t)) return 0u;
    const double f = floor((double)t);
    return (uint32_t)(int64_t)f & 255u;
}

// rows[slot * ld] (slot = slots[r] or r) -> codes (data: 256-row tiles, query:
// RQ_QPB-row group tiles) and meta {sum, sum2}.  One wave per row.
template <int QUERY>
__global__ __launch_bounds__(256) void k_sq_encode(const float* __restrict__ rows, int64_t ld, int64_t n, int d,
                                                   const uint32_t* __restrict__ slots, int Dq, float a, float b,
                                                   uint4* __restrict__ codes, uint2* __restrict__ meta) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n) return;
    const int64_t slot = slots ? (int64_t)slots[r] : r;
    const float* x = rows + (QUERY ? r : slot) * ld;
    const int nch = Dq >> 4;
    uint32_t sum = 0, sum2 = 0;
    for (int c = lane; c < nch; c += 64) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint32_t word = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int e = c * 16 + j * 4 + i;
                const uint32_t cd = e < d ? sq_code_for(x[e], a, b) : 0u;
                sum += cd;
                sum2 += cd * cd;
                word |= cd << (8 * i);
            }
            w[j] = word;
        }
        const int64_t idx = QUERY ? ((slot / RQ_QPB) * nch + c) * RQ_QPB + slot % RQ_QPB
                                  : ((slot >> 8) * nch + c) * 256 + (slot & 255);
        codes[idx] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    sum = wave_sum_u32(sum);
    sum2 = wave_sum_u32(sum2);
    if (lane == 0) meta[slot] = make_uint2(sum, sum2);
}

// SQ distances of query group [q0 + RQ_QPB*blockIdx.x, +RQ_QPB) against the
// 256 rows of tile blockIdx.y (grid and outputs as k_rq8_dist).
// metric: L2 / DOT / COSINE (the Provider type of the index)
__global__ __launch_bounds__(256) void k_sq_dist(const uint4* __restrict__ codes, const uint2* __restrict__ meta, int Dq,
                                                 const uint32_t* __restrict__ valid, int64_t nslots,
                                                 const uint4* __restrict__ qcodes, const uint2* __restrict__ qmeta,
                                                 int64_t q0, int F, int metric, float a2, float ab, float ib2, int64_t ld,
                                                 float* __restrict__ E, float* __restrict__ bmin) {
    __shared__ float red[4][RQ_QPB];
    const int tid = threadIdx.x;
    const int64_t tile = blockIdx.y;
    const int64_t g = (q0 / RQ_QPB) + blockIdx.x;
    const int64_t f0 = (int64_t)blockIdx.x * RQ_QPB;
    const int64_t slot = tile * 256 + tid;
    const int nch = Dq >> 4;
    uint32_t acc[RQ_QPB];
#pragma unroll
    for (int q = 0; q < RQ_QPB; q++) acc[q] = 0;
    const uint4* xr = codes + tile * nch * 256 + tid;
    const uint4* qg = qcodes + g * nch * RQ_QPB;
    for (int c = 0; c < nch; c++) {
        const uint4 x = xr[(int64_t)c * 256];
        const uint4* qc = qg + c * RQ_QPB;
#pragma unroll
        for (int q = 0; q < RQ_QPB; q++) {
            const uint4 y = qc[q];
            uint32_t t = acc[q];
            t = __builtin_amdgcn_udot4(x.x, y.x, t, false);
            t = __builtin_amdgcn_udot4(x.y, y.y, t, false);
            t = __builtin_amdgcn_udot4(x.z, y.z, t, false);
            t = __builtin_amdgcn_udot4(x.w, y.w, t, false);
            acc[q] = t;
        }
    }
    const bool ok = slot < nslots && ((valid[slot >> 5] >> (slot & 31)) & 1u);
    const uint2 xm = ok ? meta[slot] : make_uint2(0u, 0u);
    float dist[RQ_QPB];
#pragma unroll
    for (int q = 0; q < RQ_QPB; q++) {
        const uint2 ym = qmeta[g * RQ_QPB + q];
        if (metric == L2) {
            const uint32_t l2 = xm.y + ym.y - 2u * acc[q];  // sum (x - y)^2, exact
            dist[q] = a2 * (float)l2;
        } else {
            float t = a2 * (float)acc[q];
            const float u = ab * (float)(xm.x + ym.x);  // norm(x) + norm(y): uint32 sum of the codes
            t = t + u;
            t = t + ib2;
            dist[q] = metric == DOT ? -t : 1.0f - t;
        }
    }
    rq_emit<RQ_QPB>(dist, ok, slot, f0, F, ld, tile, E, bmin, red);
}

// BQ compressor distances: popcount(x ^ y) over the words as float32.  Data
// codes word-major [W][cap]; query codes word-major [W][nq] (wave-uniform).
__global__ __launch_bounds__(256) void k_bq_dist(const uint64_t* __restrict__ codes, int64_t cap, int W,
                                                 const uint32_t* __restrict__ valid, int64_t nslots,
                                                 const uint64_t* __restrict__ qcodes, int64_t nq, int64_t q0, int F,
                                                 int64_t ld, float* __restrict__ E, float* __restrict__ bmin) {
    __shared__ float red[4][RQ_QPB];
    const int tid = threadIdx.x;
    const int64_t tile = blockIdx.y;
    const int64_t f0 = (int64_t)blockIdx.x * RQ_QPB;
    const int64_t qb = q0 + f0;
    const int64_t slot = tile * 256 + tid;
    uint32_t acc[RQ_QPB];
#pragma unroll
    for (int q = 0; q < RQ_QPB; q++) acc[q] = 0;
    const bool inr = slot < cap;
    for (int w = 0; w < W; w++) {
        const uint64_t x = inr ? codes[(int64_t)w * cap + slot] : 0ull;
#pragma unroll
        for (int q = 0; q < RQ_QPB; q++) {
            const uint64_t y = qb + q < nq ? qcodes[(int64_t)w * nq + qb + q] : 0ull;
            acc[q] += (uint32_t)__popcll(x ^ y);
        }
    }
    const bool ok = slot < nslots && ((valid[slot >> 5] >> (slot & 31)) & 1u);
    float dist[RQ_QPB];
#pragma unroll
    for (int q = 0; q < RQ_QPB; q++) dist[q] = (float)acc[q];
    rq_emit<RQ_QPB>(dist, ok, slot, f0, F, ld, tile, E, bmin, red);
}

}  // namespace
}  // namespace wv
