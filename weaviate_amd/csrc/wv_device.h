// wv_device.h -- device-side building blocks shared by the gfx950 kernels.
//
//  * exact_dist<METRIC,VARIANT>(): one lane computes Provider.SingleDist(q, x)
//    with the exact accumulation structure of the reference's AVX2 / AVX-512
//    kernels (distancer/c/{l2,dot}_avx{256,512}_amd64.c), so fp32 results are
//    bit-identical to the reference host path.  The whole library is compiled
//    with -ffp-contract=off; the only fused ops are the explicit fmaf()s.
//  * wave-wide bitonic sort / merge over (float key, uint32 id) pairs.
//  * the counter-based synthetic-data generator.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wv {
namespace {  // internal linkage: each runtime unit compiles the kernels it launches

enum Metric : int { L2 = 0, DOT = 1, COSINE = 2, HAMMING = 3 };
enum Variant : int { AVX256 = 1, AVX512 = 2 };

constexpr uint32_t NO_ID = 0xFFFFFFFFu;

// ---------------------------------------------------------------------------
// exact-order distance (lane-per-pair)
// ---------------------------------------------------------------------------

template <int METRIC>
__device__ __forceinline__ float elem_step(float acc, float a, float b) {
    if (METRIC == L2) {
        float d = a - b;
        return fmaf(d, d, acc);
    } else {
        return fmaf(a, b, acc);
    }
}

// scalar paths: l2 = (a-b)^2 mul then add (asm/l2_avx256_amd64.s vmulss/vaddss);
// dot = fma (asm/dot_avx256_amd64.s vfmadd231ss).
template <int METRIC>
__device__ __forceinline__ float scalar_step(float sum, float a, float b) {
    if (METRIC == L2) {
        float d = a - b;
        float sq = d * d;
        return sum + sq;
    } else {
        return fmaf(a, b, sum);
    }
}

// c/l2_avx256_amd64.c:97-104 reduction: ((v0+v1)+(v2+v3)) + ((v4+v5)+(v6+v7)),
// v_l = (acc3_l + acc2_l) + (acc1_l + acc0_l).
__device__ __forceinline__ float reduce_ymm4(const float (&acc)[4][8]) {
    float v[8];
#pragma unroll
    for (int l = 0; l < 8; l++) {
        float a01 = acc[1][l] + acc[0][l];
        float a23 = acc[3][l] + acc[2][l];
        v[l] = a23 + a01;
    }
    float lo = (v[0] + v[1]) + (v[2] + v[3]);
    float hi = (v[4] + v[5]) + (v[6] + v[7]);
    return lo + hi;
}

template <bool ALIGNED = true>
__device__ __forceinline__ float4 ld4(const float* p) {
    if (ALIGNED) return *reinterpret_cast<const float4*>(p);
    return make_float4(p[0], p[1], p[2], p[3]);
}

// Raw kernel value (l2 sum or dot sum) with the reference accumulation order.
// ALIGNED: q and x are 16-byte aligned (rows padded to multiples of 32 floats);
// otherwise (PQ segments at arbitrary offsets) the same order with scalar loads.
template <int METRIC, int VARIANT, bool ALIGNED = true>
__device__ float exact_raw(const float* __restrict__ q, const float* __restrict__ x, int n) {
    float sum = 0.f;
    if (n < 8) {
        for (int i = 0; i < n; i++) sum = scalar_step<METRIC>(sum, q[i], x[i]);
        return sum;
    }
    float acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
        for (int l = 0; l < 8; l++) acc[j][l] = 0.f;
    int e = 0;
    if (VARIANT == AVX512 && n >= 128) {
        // c/l2_avx512_amd64.c:43-112
        float acc5[8][16];
#pragma unroll
        for (int r = 0; r < 8; r++)
#pragma unroll
            for (int j = 0; j < 16; j++) acc5[r][j] = 0.f;
        do {
#pragma unroll
            for (int r = 0; r < 8; r++) {
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    float4 a = ld4<ALIGNED>(q + e + 16 * r + 4 * c);
                    float4 b = ld4<ALIGNED>(x + e + 16 * r + 4 * c);
                    acc5[r][4 * c + 0] = elem_step<METRIC>(acc5[r][4 * c + 0], a.x, b.x);
                    acc5[r][4 * c + 1] = elem_step<METRIC>(acc5[r][4 * c + 1], a.y, b.y);
                    acc5[r][4 * c + 2] = elem_step<METRIC>(acc5[r][4 * c + 2], a.z, b.z);
                    acc5[r][4 * c + 3] = elem_step<METRIC>(acc5[r][4 * c + 3], a.w, b.w);
                }
            }
            e += 128;
        } while (n - e >= 128);
#pragma unroll
        for (int j = 0; j < 16; j++) {
            float a0 = acc5[1][j] + acc5[0][j];
            float a2 = acc5[3][j] + acc5[2][j];
            float a4 = acc5[5][j] + acc5[4][j];
            float a6 = acc5[7][j] + acc5[6][j];
            a0 = a2 + a0;
            a4 = a6 + a4;
            acc5[0][j] = a4 + a0;
        }
#pragma unroll
        for (int l = 0; l < 8; l++) acc[0][l] = acc5[0][l] + acc[0][l];
#pragma unroll
        for (int l = 0; l < 8; l++) acc[0][l] = acc5[0][8 + l] + acc[0][l];
        if (e == n) return sum + reduce_ymm4(acc);
    }
    while (n - e >= 32) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
#pragma unroll
            for (int c = 0; c < 2; c++) {
                float4 a = ld4<ALIGNED>(q + e + 8 * j + 4 * c);
                float4 b = ld4<ALIGNED>(x + e + 8 * j + 4 * c);
                acc[j][4 * c + 0] = elem_step<METRIC>(acc[j][4 * c + 0], a.x, b.x);
                acc[j][4 * c + 1] = elem_step<METRIC>(acc[j][4 * c + 1], a.y, b.y);
                acc[j][4 * c + 2] = elem_step<METRIC>(acc[j][4 * c + 2], a.z, b.z);
                acc[j][4 * c + 3] = elem_step<METRIC>(acc[j][4 * c + 3], a.w, b.w);
            }
        }
        e += 32;
    }
    while (n - e >= 8) {
#pragma unroll
        for (int l = 0; l < 8; l++) acc[0][l] = elem_step<METRIC>(acc[0][l], q[e + l], x[e + l]);
        e += 8;
    }
    for (; e < n; e++) sum = scalar_step<METRIC>(sum, q[e], x[e]);
    return sum + reduce_ymm4(acc);
}

// Float-element hamming (c/hamming_avx256_amd64.c): SIMD lanes use ordered
// not-equal (NaN == equal), scalar elements (n<8, or the last n%8) use !=.
__device__ __forceinline__ float exact_hamming_f32(const float* q, const float* x, int n) {
    int cnt = 0;
    int simd = n < 8 ? 0 : n - (n % 8);
    for (int i = 0; i < simd; i++) {
        float a = q[i], b = x[i];
        cnt += (a == a && b == b && a != b) ? 1 : 0;
    }
    for (int i = simd; i < n; i++) cnt += (q[i] != x[i]) ? 1 : 0;
    return (float)cnt;
}

// Provider.SingleDist with Wrap: distancer/l2.go:46, dot_product.go:68,
// cosine_dist.go:42-55 (1 - dot, clamped at 0), hamming.go:80.
template <int METRIC, int VARIANT>
__device__ __forceinline__ float exact_dist(const float* q, const float* x, int n) {
    if (METRIC == HAMMING) return exact_hamming_f32(q, x, n);
    float r = exact_raw<METRIC == L2 ? L2 : DOT, VARIANT>(q, x, n);
    if (METRIC == L2) return r;
    if (METRIC == DOT) return -r;
    float p = 1.f - r;
    return p < 0.f ? 0.f : p;
}

// ---------------------------------------------------------------------------
// exact-order distance, 8 lanes per row (coalesced rows)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float lane_xor1(float v) {  // DPP quad_perm [1,0,3,2]
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float lane_xor2(float v) {  // DPP quad_perm [2,3,0,1]
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
}
__device__ __forceinline__ float lane_xor4(float v) {  // ds_swizzle bitmask mode, xor_mask 4
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (4 << 10) | 0x1F));
}

// True when exact_dist8 computes exact_dist<METRIC, VARIANT> for n elements:
// the AVX2 order, and the AVX-512 order below 128 elements where both coincide.
template <int METRIC, int VARIANT>
__device__ __forceinline__ bool exact8_ok(int n) {
    return METRIC != HAMMING && (VARIANT == AVX256 || n < 128);
}

// exact_dist8<METRIC, G>: exact_dist<METRIC, AVX256> of G rows per 8-lane
// group at once.  Lane sub = lane & 7 owns float4 slot sub of every
// 32-element chunk, i.e. acc[sub >> 1][4 (sub & 1) .. +3] of exact_raw, so a
// load instruction reads whole 128-byte lines of 8 rows (the lane-per-row form
// reads 16 bytes of 64 rows).  reduce_ymm4's tree pairs the slots by xor 2
// (acc1 + acc0, acc3 + acc2), xor 4 (a23 + a01) and xor 1 (lo + hi); IEEE
// addition is commutative, so both partners hold the identical sum.  The
// 8-element tail feeds acc[0] (slots 0 and 1) and the scalar tail `sum` in
// every lane, as in exact_raw.  All 64 lanes must be active, each group with
// the same q and n; every lane returns its group's distances.
template <int METRIC, int G>
__device__ __forceinline__ void exact_dist8(const float* __restrict__ q, const float* const (&x)[G], int n,
                                            int sub, float (&out)[G]) {
    constexpr int M = METRIC == L2 ? L2 : DOT;
    float4 acc[G];
    float sum[G];
#pragma unroll
    for (int g = 0; g < G; g++) { acc[g] = make_float4(0.f, 0.f, 0.f, 0.f); sum[g] = 0.f; }
    int e = 0;
    if (n >= 8) {
        // one row per group: four chunks' loads in flight (16 VGPRs)
#pragma unroll(G == 1 ? 4 : 1)
        for (; n - e >= 32; e += 32) {
            const float4 a = ld4(q + e + 4 * sub);
            float4 b[G];
#pragma unroll
            for (int g = 0; g < G; g++) b[g] = ld4(x[g] + e + 4 * sub);
#pragma unroll
            for (int g = 0; g < G; g++) {
                acc[g].x = elem_step<M>(acc[g].x, a.x, b[g].x);
                acc[g].y = elem_step<M>(acc[g].y, a.y, b[g].y);
                acc[g].z = elem_step<M>(acc[g].z, a.z, b[g].z);
                acc[g].w = elem_step<M>(acc[g].w, a.w, b[g].w);
            }
        }
        for (; n - e >= 8; e += 8) {
            if (sub < 2) {
                const float4 a = ld4(q + e + 4 * sub);
#pragma unroll
                for (int g = 0; g < G; g++) {
                    const float4 b = ld4(x[g] + e + 4 * sub);
                    acc[g].x = elem_step<M>(acc[g].x, a.x, b.x);
                    acc[g].y = elem_step<M>(acc[g].y, a.y, b.y);
                    acc[g].z = elem_step<M>(acc[g].z, a.z, b.z);
                    acc[g].w = elem_step<M>(acc[g].w, a.w, b.w);
                }
            }
        }
    }
    for (; e < n; e++) {
        const float a = q[e];
#pragma unroll
        for (int g = 0; g < G; g++) sum[g] = scalar_step<M>(sum[g], a, x[g][e]);
    }
#pragma unroll
    for (int g = 0; g < G; g++) {
        float r = sum[g];
        if (n >= 8) {
            float4 p = acc[g];
            p.x = p.x + lane_xor2(p.x); p.y = p.y + lane_xor2(p.y);
            p.z = p.z + lane_xor2(p.z); p.w = p.w + lane_xor2(p.w);
            p.x = p.x + lane_xor4(p.x); p.y = p.y + lane_xor4(p.y);
            p.z = p.z + lane_xor4(p.z); p.w = p.w + lane_xor4(p.w);
            float h = (p.x + p.y) + (p.z + p.w);
            h = h + lane_xor1(h);
            r = r + h;
        }
        if (METRIC == DOT) r = -r;
        if (METRIC == COSINE) { r = 1.f - r; r = r < 0.f ? 0.f : r; }
        out[g] = r;
    }
}

// 64 rows per wave with exact_dist8: xp[g] is the row of lane 8g + (lane >> 3);
// returns the distance of row `lane` (the lane-per-row layout of the callers).
template <int METRIC>
__device__ __forceinline__ float exact8_rows64(const float* __restrict__ q, const float* const (&xp)[8], int n, int lane) {
    float dv[8];
    exact_dist8<METRIC, 8>(q, xp, n, lane & 7, dv);
    float r = 0.f;
#pragma unroll
    for (int g = 0; g < 8; g++) {
        const float t = __shfl(dv[g], (lane & 7) * 8);
        r = (lane >> 3) == g ? t : r;
    }
    return r;
}

// ---------------------------------------------------------------------------
// wave-wide bitonic sort over NS = 64*R (key,id) pairs; element e = r*64+lane.
// Order: key ascending, then id ascending (placeholders: +inf, NO_ID).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool kv_less(float ka, uint32_t ia, float kb, uint32_t ib) {
    return ka < kb || (ka == kb && ia < ib);
}

template <int R>
__device__ __forceinline__ void cmpx_step(float (&key)[R], uint32_t (&id)[R], int k, int j, int lane) {
    if (j >= 64) {
        const int m = j >> 6;
#pragma unroll
        for (int r = 0; r < R; r++) {
            int p = r ^ m;
            if (p > r) {
                int e = r * 64 + lane;
                bool up = (e & k) == 0;
                bool sw = up ? kv_less(key[p], id[p], key[r], id[r]) : kv_less(key[r], id[r], key[p], id[p]);
                if (sw) {
                    float tk = key[r]; key[r] = key[p]; key[p] = tk;
                    uint32_t ti = id[r]; id[r] = id[p]; id[p] = ti;
                }
            }
        }
    } else {
#pragma unroll
        for (int r = 0; r < R; r++) {
            int e = r * 64 + lane;
            float ok = __shfl_xor(key[r], j);
            uint32_t oi = (uint32_t)__shfl_xor((int)id[r], j);
            bool up = (e & k) == 0;
            bool lower = (lane & j) == 0;
            bool other_less = kv_less(ok, oi, key[r], id[r]);
            // lower element keeps the min when ascending, the max when descending
            bool take = (lower == up) ? other_less : !other_less && !(ok == key[r] && oi == id[r]);
            if (take) { key[r] = ok; id[r] = oi; }
        }
    }
}

template <int R>
__device__ __forceinline__ void bitonic_sort(float (&key)[R], uint32_t (&id)[R], int lane) {
    constexpr int NS = 64 * R;
#pragma unroll
    for (int k = 2; k <= NS; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) cmpx_step<R>(key, id, k, j, lane);
}

// Rows 0..R-2 already sorted, row R-1 arbitrary: sort row R-1 alone, reverse
// it (the R rows then form one bitonic sequence) and run only the final merge
// stage of the 64R network -- the same sorted list as bitonic_sort<R>.
template <int R>
__device__ __forceinline__ void bitonic_merge_last(float (&key)[R], uint32_t (&id)[R], int lane) {
    float pk[1] = {key[R - 1]};
    uint32_t pi[1] = {id[R - 1]};
    bitonic_sort<1>(pk, pi, lane);
    key[R - 1] = __shfl(pk[0], 63 - lane);
    id[R - 1] = (uint32_t)__shfl((int)pi[0], 63 - lane);
#pragma unroll
    for (int j = 32 * R; j > 0; j >>= 1) cmpx_step<R>(key, id, 64 * R, j, lane);
}

// ---------------------------------------------------------------------------
// synthetic data generator (identical to oracle/oracle.c or_gen_value)
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ float gen_value(int kind, uint64_t seed, uint64_t row, uint64_t col) {
    uint64_t h = mix64(seed * 0x9E3779B97F4A7C15ULL + (row << 16) + col + 0x632BE59BD9B4E019ULL);
    if (kind == 1) return (float)(h >> 57);
    if (kind == 2) return (float)(h >> 40) * 5.9604644775390625e-08f;
    return (float)(h >> 40) * 1.1920928955078125e-07f - 1.0f;
}

}  // namespace
}  // namespace wv
