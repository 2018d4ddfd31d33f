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
