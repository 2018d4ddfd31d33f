// rq_kernels.hip -- flat's rotational-quantization modes on gfx950
// (flat/quantizer.go:85-99: "rq-8" = compressionhelpers.RotationalQuantizer
// with 8 bits, "rq-1" = BinaryRotationalQuantizer).
//
//   k_rq_encode<BITS,VARIANT,QUERY>  FastRotation.Rotate (fast_rotation.go:101-122)
//                      in LDS (one 256-thread block per vector: signed swap
//                      permutation, then blocked Walsh-Hadamard butterflies with
//                      the reference's stride order), then
//                      BITS=8: RotationalQuantizer.encode (rotational_quantization.go:182-213)
//                      BITS=1 data: BinaryRotationalQuantizer.Encode (binary_rotational_quantization.go:158-187)
//                      BITS=1 query: encodeQuery (:254-314, 5 bit planes)
//   k_rq8_dist         DistanceBetweenCompressedVectors(candidate, query)
//                      (rotational_quantization.go:294-306): v_dot4_u32_u8 over
//                      the code bytes (exact uint32 == dotByteImpl), then the
//                      reference's float32 expression, unfused.
//   k_rq1_dist         BinaryRQDistancer.Distance (:364-385): 5 xor/popcount
//                      planes per 64-bit word, exact integer estimator.
// Both distance kernels write the exact quantized distance E[f][slot] and the
// 256-row block minima that k_replay_scan (kernels.hip) consumes to replay the
// reference's R-heap (flat/index.go:470-487) in id order.
//
// Layouts:
//   rq-8 data codes: 32-row tiles of 16-byte chunks, stored offset by 128:
//        chunk c of slot s is the uint4 at ((s/32) * (D/16) + c) * 32 + s%32
//        (rq_tile_u4) -> 32 rows' chunk = 512 contiguous bytes, a 32-row block
//        one contiguous run; meta[s] = {lower, step, codeSum, norm2} (float4),
//        code sums after the meta (rq_csum).
//   rq-1 data codes: word-major [W][cap] u64 (coalesced per word); meta[s] =
//        {step, squaredNorm, 0, 0}.
//   queries: group-tiled for uniform (scalar) loads in the distance kernels:
//        rq-8 chunk c of query q at ((q/RQ_QPB) * (D/16) + c) * RQ_QPB + q%RQ_QPB;
//        rq-1 plane p, word w of q at (((q/RQ_QPB) * W + w) * 5 + p) * RQ_QPB + q%RQ_QPB;
//        qmeta[q] = rq-8 {lower, step, codeSum, norm2}; rq-1 {step, sqn, dim, 0}.
#pragma once

namespace wv {
namespace {  // internal linkage: each runtime unit compiles the kernels it launches

constexpr int RQ_QPB = 32;      // queries per distance block (scalar operands)
constexpr int RQ_MAXD = 4096;   // rotation output dims supported (two LDS buffers)
constexpr int RQ_ROUNDS = 3;
constexpr size_t RQ_META_B = sizeof(float4) + sizeof(uint32_t);  // per slot: meta, then (rq-8) the code sum
// rq-8 codes (and the rq-1 +-1 plane): 32-row tiles of 16-byte chunks, the
// uint4 index of chunk c of slot s -- a 32-row block is one contiguous
// 32 D-byte run in [chunk][row] order (k_rq8_keys' LDS image, 1-KiB DMA
// pieces), and 32 consecutive rows read one chunk as 512 contiguous bytes
__host__ __device__ constexpr int64_t rq_tile_u4(int64_t s, int c, int nch) {
    return ((s >> 5) * nch + c) * 32 + (s & 31);
}    // rotationRounds (rotational_quantization.go:61, binary_...:27)

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// FastRotation.Rotate of row[0..d) zero-padded to D (a multiple of 64) into
// LDS; returns the buffer holding the result.  src/sign: [RQ_ROUNDS][D],
// new[i] = sign[i] * old[src[i]] (the round's disjoint swaps,
// fast_rotation.go:106-108).  Blocks: 256 entries while >= 256 remain, then 64
// (:110-119); each block is scaled by 1/16 or 1/8 first (fastWalshHadamardTransform16
// scales on load) and then butterflied with strides 1, 2, 4, ... (:154-288).
__device__ float* rq_rotate(float* bufA, float* bufB, const float* __restrict__ row, int d, int D,
                            const uint16_t* __restrict__ src, const float* __restrict__ sign) {
    const int tid = threadIdx.x;
    for (int i = tid; i < D; i += 256) bufA[i] = i < d ? row[i] : 0.f;
    __syncthreads();
    const int n256 = (D >> 8) << 8;
    float* cur = bufA;
    float* nxt = bufB;
    for (int r = 0; r < RQ_ROUNDS; r++) {
        const uint16_t* sr = src + r * D;
        const float* sg = sign + r * D;
        for (int i = tid; i < D; i += 256) {
            float v = sg[i] * cur[sr[i]];
            nxt[i] = (i < n256 ? 0.0625f : 0.125f) * v;
        }
        __syncthreads();
        for (int h = 1; h < 256; h <<= 1) {
            const int npairs = h < 64 ? (D >> 1) : (n256 >> 1);
            for (int p = tid; p < npairs; p += 256) {
                const int i = (p / h) * 2 * h + (p % h);
                const float a = nxt[i], b = nxt[i + h];
                nxt[i] = a + b;
                nxt[i + h] = a - b;
            }
            __syncthreads();
        }
        float* t = cur;
        cur = nxt;
        nxt = t;
    }
    return cur;
}

// Encode rows: row r reads rows[slot * ld ...] (slot = slots[r] or r), d floats.
// QUERY = 0: data layout (slot-indexed); QUERY = 1: query layout (index r).
template <int BITS, int VARIANT, int QUERY>
__global__ __launch_bounds__(256) void k_rq_encode(const float* __restrict__ rows, int64_t ld, int64_t n, int d,
                                                   const uint32_t* __restrict__ slots, int D,
                                                   const uint16_t* __restrict__ rot_src,
                                                   const float* __restrict__ rot_sign,
                                                   const float* __restrict__ rounding, void* __restrict__ codes,
                                                   int64_t cap, float4* __restrict__ meta,
                                                   uint32_t* __restrict__ csum_out,
                                                   unsigned char* __restrict__ pm_out) {
    extern __shared__ __attribute__((aligned(16))) float esm[];
    float* bufA = esm;
    float* bufB = esm + D;
    __shared__ float redf[2][4];
    __shared__ uint32_t redu[4];
    __shared__ float s_scal[4];
    const int64_t r = blockIdx.x;
    if (r >= n) return;
    const int tid = threadIdx.x, lane = tid & 63, wv_ = tid >> 6;
    const int64_t slot = QUERY ? r : (slots ? (int64_t)slots[r] : r);
    const float* row = rows + (QUERY ? r : slot) * ld;
    const float* rx = rq_rotate(bufA, bufB, row, d, D, rot_src, rot_sign);
    if (BITS == 8) {
        float lo = __builtin_inff(), hi = -__builtin_inff();
        for (int i = tid; i < D; i += 256) { lo = fminf(lo, rx[i]); hi = fmaxf(hi, rx[i]); }
        lo = wave_min(lo);
        hi = wave_max(hi);
        if (lane == 0) { redf[0][wv_] = lo; redf[1][wv_] = hi; }
        __syncthreads();
        lo = fminf(fminf(redf[0][0], redf[0][1]), fminf(redf[0][2], redf[0][3]));
        hi = fmaxf(fmaxf(redf[1][0], redf[1][1]), fmaxf(redf[1][2], redf[1][3]));
        const float step = (hi - lo) / 255.0f;
        const bool zero = step <= 0.f;  // ZeroRQCode (:196-199)
        // codes: thread handles 16-byte chunks
        uint32_t csum = 0;
        const int nch = D >> 4;
        uint4* out = reinterpret_cast<uint4*>(codes);
        for (int c = tid; c < nch; c += 256) {
            uint32_t w[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                uint32_t word = 0;
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    uint32_t cb = 0;
                    if (!zero) {
                        float t = (rx[c * 16 + j * 4 + b] - lo) / step;
                        t = t + 0.5f;
                        cb = (uint32_t)(int)t & 0xFFu;  // byte(...): truncation
                    }
                    csum += cb;
                    word |= cb << (8 * b);
                }
                w[j] = word;
            }
            const int64_t o = QUERY ? ((r / RQ_QPB) * nch + c) * RQ_QPB + (r % RQ_QPB)
                                    : rq_tile_u4(slot, c, nch);
            // data codes are stored offset by 128 (byte x ^ 0x80 = int8 x - 128:
            // the integer-MFMA operand of k_rq8_keys); query codes as they are
            constexpr uint32_t X = QUERY ? 0u : 0x80808080u;
            out[o] = make_uint4(w[0] ^ X, w[1] ^ X, w[2] ^ X, w[3] ^ X);
        }
        csum = wave_sum_u32(csum);
        if (lane == 0) redu[wv_] = csum;
        __syncthreads();
        if (tid == 0) {
            float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
            if (!zero) {
                const uint32_t cs = redu[0] + redu[1] + redu[2] + redu[3];  // exact: sum of float32(c) < 2^24
                // norm2 = dotProduct(x, x) (:176-180, :211): the SIMD dot kernel's order
                const float n2 = exact_raw<DOT, VARIANT>(row, row, d);
                m = make_float4(lo, step, step * (float)cs, n2);
            }
            meta[slot] = m;
            if (!QUERY && csum_out) csum_out[slot] = zero ? 0u : redu[0] + redu[1] + redu[2] + redu[3];
        }
    } else {
        const int W = D >> 6;
        uint64_t* out = reinterpret_cast<uint64_t*>(codes);
        if (!QUERY) {
            for (int w = tid; w < W; w += 256) {
                uint64_t bits = 0;
                for (int j = 0; j < 64; j++)
                    if (rx[w * 64 + j] > 0.f) bits |= 1ull << j;
                out[(int64_t)w * cap + slot] = bits;
            }
            // the +-1 plane of the same bits (integer-MFMA operand of
            // k_rq8_keys<.., 1>): byte 1 - 2 bit, tiled as the rq-8 codes
            if (pm_out) {
                const int nch = D >> 4;
                for (int c = tid; c < nch; c += 256) {
                    uint32_t wd[4];
#pragma unroll
                    for (int jj = 0; jj < 4; jj++) {
                        uint32_t word = 0;
#pragma unroll
                        for (int b = 0; b < 4; b++) word |= (rx[c * 16 + jj * 4 + b] > 0.f ? 0xFFu : 0x01u) << (8 * b);
                        wd[jj] = word;
                    }
                    reinterpret_cast<uint4*>(pm_out)[rq_tile_u4(slot, c, nch)] =
                        make_uint4(wd[0], wd[1], wd[2], wd[3]);
                }
            }
            if (tid == 0) {  // sequential l1 / l2 (:165-176)
                float l2 = 0.f, l1 = 0.f;
                for (int i = 0; i < D; i++) {
                    const float v = rx[i];
                    if (v > 0.f) l1 = l1 + v;
                    else l1 = l1 + (-v);
                    const float sq = v * v;
                    l2 = l2 + sq;
                }
                float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
                if (l1 != 0.f) m = make_float4(l2 / l1, l2, 0.f, 0.f);
                meta[slot] = m;
            }
        } else {
            float mx = 0.f;
            for (int i = tid; i < D; i += 256) mx = fmaxf(mx, fabsf(rx[i]));
            mx = wave_max(mx);
            if (lane == 0) redf[0][wv_] = mx;
            __syncthreads();
            mx = fmaxf(fmaxf(redf[0][0], redf[0][1]), fmaxf(redf[0][2], redf[0][3]));
            const bool zero = mx == 0.f;  // RQMultiBitCode{} (:257-260)
            const float step = mx / 31.0f;
            const float twostep = 2.0f * step;
            const int64_t g = r / RQ_QPB, ql = r % RQ_QPB;
            for (int w = tid; w < W; w += 256) {
                uint64_t pl[5] = {0, 0, 0, 0, 0};
                if (!zero) {
                    for (int j = 0; j < 64; j++) {
                        const int i = w * 64 + j;
                        float t = rx[i] + mx;
                        t = t / twostep;
                        t = t + rounding[i];
                        const uint64_t c = (uint64_t)t;
#pragma unroll
                        for (int p = 0; p < 5; p++)
                            if (c & (1ull << p)) pl[p] |= 1ull << j;
                    }
                }
#pragma unroll
                for (int p = 0; p < 5; p++) out[((g * W + w) * 5 + p) * RQ_QPB + ql] = pl[p];
            }
            if (tid == 0) {
                float sqn = 0.f;
                if (!zero)
                    for (int i = 0; i < D; i++) { const float sq = rx[i] * rx[i]; sqn = sqn + sq; }
                s_scal[0] = sqn;
                meta[r] = zero ? make_float4(0.f, 0.f, 0.f, 0.f) : make_float4(step, sqn, (float)D, 0.f);
            }
        }
    }
}

// Block-reduce the per-(query, row) distances of one 256-row tile into the
// tile minimum per query and write E.  dist[q] for this thread's row.
template <int QPB>
__device__ __forceinline__ void rq_emit(const float (&dist)[QPB], bool ok, int64_t slot, int64_t f0, int F,
                                        int64_t ld, int64_t tile, float* __restrict__ E,
                                        float* __restrict__ bmin, float (*red)[QPB]) {
    const int tid = threadIdx.x, lane = tid & 63, wv_ = tid >> 6;
#pragma unroll
    for (int q = 0; q < QPB; q++) {
        if (f0 + q < F) {
            if (slot < ld) E[(f0 + q) * ld + slot] = ok ? dist[q] : __builtin_inff();
            const float m = wave_min(ok ? dist[q] : __builtin_inff());
            if (lane == 0) red[wv_][q] = m;
        }
    }
    __syncthreads();
    if (tid < QPB && f0 + tid < F)
        bmin[(f0 + tid) * (ld / 256) + tile] = fminf(fminf(red[0][tid], red[1][tid]), fminf(red[2][tid], red[3][tid]));
}

// rq-8 distances of query group [q0 + RQ_QPB*blockIdx.x, +RQ_QPB) (codes in
// the group-tiled query layout) against the 256 rows of tile blockIdx.y.
// Thread = row.  Query bytes are wave-uniform: scalar loads, v_dot4_u32_u8
// with SGPR operands.  E / bmin rows are indexed f = query - q0.
__global__ __launch_bounds__(256) void k_rq8_dist(const uint4* __restrict__ codes, const float4* __restrict__ meta,
                                                  int D, const uint32_t* __restrict__ valid, int64_t nslots,
                                                  const uint4* __restrict__ qcodes, const float4* __restrict__ qmeta,
                                                  int64_t q0, int F, float fl2, float fcos, int64_t ld,
                                                  float* __restrict__ E, float* __restrict__ bmin) {
    __shared__ float red[4][RQ_QPB];
    const int tid = threadIdx.x;
    const int64_t tile = blockIdx.y;
    const int64_t g = (q0 / RQ_QPB) + blockIdx.x;  // q0 is a multiple of RQ_QPB
    const int64_t f0 = (int64_t)blockIdx.x * RQ_QPB;
    const int64_t slot = tile * 256 + tid;
    const int nch = D >> 4;
    uint32_t acc[RQ_QPB];
#pragma unroll
    for (int q = 0; q < RQ_QPB; q++) acc[q] = 0;
    const uint4* xr = codes + rq_tile_u4(slot, 0, nch);
    const uint4* qg = qcodes + g * nch * RQ_QPB;
    for (int c = 0; c < nch; c++) {
        uint4 x = xr[(int64_t)c * 32];
        x.x ^= 0x80808080u;  // stored offset by 128 (k_rq_encode)
        x.y ^= 0x80808080u;
        x.z ^= 0x80808080u;
        x.w ^= 0x80808080u;
        const uint4* qc = qg + c * RQ_QPB;
#pragma unroll
        for (int q = 0; q < RQ_QPB; q++) {
            const uint4 y = qc[q];
            uint32_t a = acc[q];
            a = __builtin_amdgcn_udot4(x.x, y.x, a, false);
            a = __builtin_amdgcn_udot4(x.y, y.y, a, false);
            a = __builtin_amdgcn_udot4(x.z, y.z, a, false);
            a = __builtin_amdgcn_udot4(x.w, y.w, a, false);
            acc[q] = a;
        }
    }
    const bool ok = slot < nslots && ((valid[slot >> 5] >> (slot & 31)) & 1u);
    const float4 xm = ok ? meta[slot] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float fD = (float)D;
    float dist[RQ_QPB];
#pragma unroll
    for (int q = 0; q < RQ_QPB; q++) {
        const float4 ym = qmeta[g * RQ_QPB + q];
        // a = D * x.lower * y.lower; b = x.lower * y.codeSum; c = y.lower * x.codeSum;
        // d = x.step * y.step * float32(dot); est = ((a + b) + c) + d
        float a = fD * xm.x;
        a = a * ym.x;
        const float b = xm.x * ym.z;
        const float cc = ym.x * xm.z;
        float dd = xm.y * ym.y;
        dd = dd * (float)acc[q];
        float est = a + b;
        est = est + cc;
        est = est + dd;
        float t = fl2 * (xm.w + ym.w);
        t = t + fcos;
        const float s = 1.0f + fl2;
        dist[q] = t - s * est;
    }
    rq_emit<RQ_QPB>(dist, ok, slot, f0, F, ld, tile, E, bmin, red);
}

// rq-1 distances (BinaryRQDistancer.Distance) -- same grid as k_rq8_dist.
__global__ __launch_bounds__(256) void k_rq1_dist(const uint64_t* __restrict__ codes, int64_t cap,
                                                  const float4* __restrict__ meta, int W,
                                                  const uint32_t* __restrict__ valid, int64_t nslots,
                                                  const uint64_t* __restrict__ qplanes,
                                                  const float4* __restrict__ qmeta, int64_t q0, int F, float fl2,
                                                  float fcos, int64_t ld, float* __restrict__ E,
                                                  float* __restrict__ bmin) {
    __shared__ float red[4][RQ_QPB];
    const int tid = threadIdx.x;
    const int64_t tile = blockIdx.y;
    const int64_t g = (q0 / RQ_QPB) + blockIdx.x;
    const int64_t f0 = (int64_t)blockIdx.x * RQ_QPB;
    const int64_t slot = tile * 256 + tid;
    uint32_t acc[RQ_QPB];
#pragma unroll
    for (int q = 0; q < RQ_QPB; q++) acc[q] = 0;
    const uint64_t* qg = qplanes + g * (int64_t)W * 5 * RQ_QPB;
    for (int w = 0; w < W; w++) {
        const uint64_t x = codes[(int64_t)w * cap + slot];
        const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
        const uint64_t* qw = qg + (int64_t)w * 5 * RQ_QPB;
#pragma unroll
        for (int q = 0; q < RQ_QPB; q++) {
            uint32_t a = acc[q];
#pragma unroll
            for (int p = 0; p < 5; p++) {
                const uint64_t y = qw[p * RQ_QPB + q];
                uint32_t h = __builtin_popcount(xl ^ (uint32_t)y);
                h += __builtin_popcount(xh ^ (uint32_t)(y >> 32));
                a += h << (p + 1);
            }
            acc[q] = a;
        }
    }
    const bool ok = slot < nslots && ((valid[slot >> 5] >> (slot & 31)) & 1u);
    const float4 xm = ok ? meta[slot] : make_float4(0.f, 0.f, 0.f, 0.f);
    float dist[RQ_QPB];
#pragma unroll
    for (int q = 0; q < RQ_QPB; q++) {
        const float4 ym = qmeta[g * RQ_QPB + q];  // {step, sqn, dim, 0}
        const int qdim = (int)ym.z;
        const int dot = qdim > 0 ? 31 * qdim - (int)acc[q] : 0;
        float est = ym.x * xm.x;
        est = est * (float)dot;
        float t = fl2 * (xm.y + ym.y);
        t = t + fcos;
        const float s = 1.0f + fl2;
        dist[q] = t - s * est;
    }
    rq_emit<RQ_QPB>(dist, ok, slot, f0, F, ld, tile, E, bmin, red);
}

}  // namespace
}  // namespace wv
