// kernels.hip -- gfx950 kernels of the flat-index hot path.
//
// The default exact search is the block-key path (qs_kernels.hip).  These are
// the row preparation, the fallback select path (d > 1536, hamming-free k <= 24
// without block keys, option kernel) and the exact replay shared by all paths
// (flat/index.go:423-448, :578-688), per GPU:
//   k_prepare_rows      normalise (cosine, distancer/normalize.go:16-32) and
//                       store rows + squared norms          [Add, :362-390]
//   k_mfma_select3      f32 MFMA (v_mfma_f32_32x32x2_f32) query x corpus tiles
//                       fused with per-(query, corpus span) top-KP selection
//                       on an approximate distance; the B x N distance matrix
//                       is never written (k_gemv_select: the same for <= 8
//                       queries, gemv_kernels.hip).
//   k_merge_spans       merge the span lists of a query       (wave per query)
//   k_rescore           exact-order distance of the KP candidates (lane per pair)
//   k_finalize          sort by exact distance, prove the result equals the
//                       reference heap's (margin + no ties), else flag
//   k_exact_rows +      flagged queries: exact-order distances of every row,
//   k_replay_scan       then an exact replay of the reference heap
//                       (priorityqueue NewMax + insertToHeap) over the id-ordered
//                       scan, skipping 256-row blocks that cannot insert.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wv_device.h"

namespace wv {
namespace {  // internal linkage: each runtime unit compiles the kernels it launches

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// row preparation
// ---------------------------------------------------------------------------

// One lane per row: out row = normalize(in row) for cosine, else a copy; pad
// columns [d, dpad) are zeroed.  norm2[row] = sum of squares of the stored row
// (any order: only feeds the approximate L2 and the error bound).
// maxnorm2_bits: atomicMax over the float bits of norm2 (non-negative floats
// order like their bit patterns).
template <int METRIC>
__global__ void k_prepare_rows(const float* __restrict__ in, int64_t n, int d, const uint32_t* __restrict__ slots,
                               float* __restrict__ out, int dpad, float* __restrict__ norm2,
                               uint32_t* __restrict__ present_bits, uint32_t* __restrict__ maxnorm2_bits) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* src = in + i * (int64_t)d;
    int64_t slot = slots ? (int64_t)slots[i] : i;
    float* dst = out + slot * (int64_t)dpad;
    float divisor = 1.f;
    bool zero = false;
    if (METRIC == COSINE) {
        float nrm = 0.f;
        for (int c = 0; c < d; c++) { float v = src[c]; float sq = v * v; nrm = nrm + sq; }
        if (nrm == 0.f) zero = true;
        else divisor = (float)sqrt((double)nrm);
    }
    float s2 = 0.f;
    for (int c = 0; c < d; c++) {
        float v = src[c];
        if (METRIC == COSINE) v = zero ? 0.f : v / divisor;
        dst[c] = v;
        s2 = fmaf(v, v, s2);
    }
    for (int c = d; c < dpad; c++) dst[c] = 0.f;
    if (norm2) norm2[slot] = s2;
    if (present_bits) atomicOr(&present_bits[slot >> 5], 1u << (slot & 31));
    if (maxnorm2_bits) atomicMax(maxnorm2_bits, __float_as_uint(s2));
}

// ---------------------------------------------------------------------------
// main MFMA + selection kernel
// ---------------------------------------------------------------------------
// Block: 256 threads = 4 waves in a 2 (queries) x 2 (corpus rows) layout over a
// 128-query x 128-row tile; each wave owns 64x64 = 2x2 MFMA 32x32 blocks.  The
// MFMA computes C^T: A = corpus rows (i = row), B = queries (j = query), so the
// accumulator layout puts the query on the lane (col = lane&31) and 16 corpus
// rows in registers (row = (r&3) + 8(r>>2) + 4(lane>>5)).
//
// LDS staging (per BK=32 slice): rows at a 36-float stride; a lane's 16
// k-values for the 16 MFMA k-steps are one contiguous 64 B run
// (4 x ds_read_b128), bank-conflict-free for reads and writes (see stage()).
constexpr int QB = 128;   // queries per workgroup tile
constexpr int BN = 128;   // corpus rows per tile
constexpr int BK = 32;    // k per staging step
constexpr int LDSROW = 36;

struct SelectArgs {
    const float* X;           // [cap][dpad]
    const float* xnorm2;      // [cap]
    const uint32_t* valid;    // bitmap over slots: present & allowed
    int64_t ntiles;           // tiles of BN rows to scan
    const float* Q;           // [nq_pad][dpad]
    const float* qnorm2;      // [nq_pad]
    int nq;
    int dpad;
    int tiles_per_span;
    int nspans;
    int nqb;
    int KP;
    int C;                    // candidate buffer per query (KP + C <= 64*R)
    int qgroup;               // query blocks per XCD cell (divides nqb)
    float* outA;              // [nq_pad][nspans][KP]
    uint32_t* outI;
    int dbg;                  // timing experiments only: 1 = skip selection, 2 = skip MFMA + selection
    int opt;                  // kernel tuning bits (option sel_opt), reserved for experiments
};

template <int R>
__device__ __forceinline__ void merge_query_list(float* listA, uint32_t* listI, const float* cbA,
                                                 const uint32_t* cbI, int KP, int C, int nc, int lane,
                                                 float* thr_slot) {
    float key[R];
    uint32_t id[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        int e = r * 64 + lane;
        if (e < KP) { key[r] = listA[e]; id[r] = listI[e]; }
        else if (e - KP < nc) { key[r] = cbA[e - KP]; id[r] = cbI[e - KP]; }
        else { key[r] = __builtin_inff(); id[r] = NO_ID; }
    }
    bitonic_sort<R>(key, id, lane);
#pragma unroll
    for (int r = 0; r < R; r++) {
        int e = r * 64 + lane;
        if (e < KP) { listA[e] = key[r]; listI[e] = id[r]; }
        if (e == KP - 1) *thr_slot = key[r];
    }
}

// 32-float rows with an XOR chunk swizzle f(r) = (r&3) ^ ((r>>2)&7): the
// 16-lane ds_read_b128 groups are conflict-free
__device__ __forceinline__ int swz(int r) { return ((r & 3) ^ ((r >> 2) & 7)); }

// ---------------------------------------------------------------------------
// k_mfma_select3: 8 waves, 128-query x 256-row tiles, direct global->LDS DMA
// (global_load_lds_dwordx4) into a 3-deep LDS ring: slice s+2 is in flight
// while slice s is multiplied; one raw s_barrier per BK slice behind a counted
// vmcnt (Guide §5 "Pipelining across barriers").  The DMA writes LDS
// lane-linearly, so the XOR chunk swizzle f(r) is applied to the per-lane
// SOURCE address and again on the read (rule 21).  Lists live in the output
// buffer (global), thresholds / counters / candidate buffer in LDS;
// ~156 KiB LDS, one workgroup (2 waves per SIMD) per CU.
// ---------------------------------------------------------------------------
constexpr int BN3 = 256;
constexpr int NBUF3 = 3;
constexpr int STG3 = (BN3 + QB) * BK;  // floats per ring slot
constexpr int GLDS_PER_WAVE = (BN3 + QB) * BK * 4 / 1024 / 8;  // 1 KiB pieces per wave per slice (= 6)

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(3))) const float lds_cfloat;

// ds_read_b128 from an LDS pointer, invisible to hipcc's waitcnt insertion:
// the caller waits with an explicit lgkmcnt + sched_barrier (rule 18).
__device__ __forceinline__ float4 lds_ld4(const float* p) {
    float4 v;
    const unsigned off = (unsigned)(size_t)((lds_cfloat*)p);
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(off));
    return v;
}
__device__ __forceinline__ float f4get(const float4& v, int t) { return t == 0 ? v.x : t == 1 ? v.y : t == 2 ? v.z : v.w; }

template <int METRIC, int R>
__global__ __launch_bounds__(512, 2) void k_mfma_select3(SelectArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int KP = a.KP;
    const int C = a.C;
    float* ring = smem;                                      // [NBUF3][STG3]
    float* thr = ring + NBUF3 * STG3;                        // QB
    int* cnt = reinterpret_cast<int*>(thr + QB);             // QB
    int* flags = cnt + QB;                                   // 4
    float* cbA = reinterpret_cast<float*>(flags + 4);        // QB*C
    uint32_t* cbI = reinterpret_cast<uint32_t*>(cbA + QB * C);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;          // 0..7
    const int wq = wave & 1, wx = wave >> 1;   // 2 query halves x 4 row quarters
    const int li = lane & 31, lh = lane >> 5;

    const int total = a.nqb * a.nspans;
    const int b = blockIdx.x;
    const int logical = (total % 8 == 0) ? (b % 8) * (total / 8) + (b / 8) : b;
    const int QG = a.qgroup;
    const int cell = logical / QG, qi = logical % QG;
    const int group = cell / a.nspans;
    const int span = cell % a.nspans;
    const int qb = group * QG + qi;
    const int q0 = qb * QB;

    for (int jq = 0; jq < QB / 8; jq++) {
        const int q = wave + 8 * jq;
        if (q0 + q >= a.nq) continue;
        const int64_t base = ((int64_t)(q0 + q) * a.nspans + span) * KP;
        for (int e = lane; e < KP; e += 64) { a.outA[base + e] = __builtin_inff(); a.outI[base + e] = NO_ID; }
    }
    if (tid < QB) { thr[tid] = __builtin_inff(); cnt[tid] = 0; }
    if (tid == 0) { flags[0] = 0; flags[1] = 0; }

    const int64_t t0 = (int64_t)span * a.tiles_per_span;
    int64_t t1 = t0 + a.tiles_per_span;
    if (t1 > a.ntiles) t1 = a.ntiles;
    const int nk = a.dpad / BK;
    const int64_t total_steps = t1 > t0 ? (t1 - t0) * nk : 0;

    // DMA piece p (0..5) of this wave covers 8 rows: pieces 0-3 -> X rows
    // 32*wave + 8p, pieces 4-5 -> Q rows 16*wave + 8(p-4).  Lane L writes LDS
    // row (L>>3), physical chunk (L&7), i.e. logical chunk (L&7) ^ f(row).
    const int prow = lane >> 3, pchunk = lane & 7;
    auto issue = [&](int64_t step) {
        const int64_t tile = t0 + step / nk;
        const int kb = (int)(step % nk);
        float* slot = ring + (int)(step % NBUF3) * STG3;
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const int row = 32 * wave + 8 * p + prow;
            const int c = pchunk ^ swz(row & 31);
            const float* src = a.X + (tile * BN3 + row) * (int64_t)a.dpad + kb * BK + 4 * c;
            __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(slot + (32 * wave + 8 * p) * BK), 16, 0, 0);
        }
#pragma unroll
        for (int p = 0; p < 2; p++) {
            const int row = 16 * wave + 8 * p + prow;
            const int c = pchunk ^ swz(row & 31);
            const float* src = a.Q + (int64_t)(q0 + row) * a.dpad + kb * BK + 4 * c;
            __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(slot + BN3 * BK + (16 * wave + 8 * p) * BK), 16, 0, 0);
        }
    };

    const int rsw = swz(li);
    f32x16 acc[2][2];
    int epoch = 0;
    if (total_steps > 0) issue(0);
    if (total_steps > 1) issue(1);

    for (int64_t step = 0; step < total_steps; step++) {
        const int64_t tile = t0 + step / nk;
        const int kb = (int)(step % nk);
        // this wave's pieces of `step` have landed (those of step+1 may fly)
        if (step + 1 < total_steps) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // everyone's pieces landed; slot (step+2)%3 is free
        __builtin_amdgcn_sched_barrier(0);
        if (step + 2 < total_steps) issue(step + 2);
        const float* cur = ring + (int)(step % NBUF3) * STG3;
        if (kb == 0) {
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 2; j++)
#pragma unroll
                    for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;
        }
        // fragment reads in inline asm: hipcc would otherwise put vmcnt(0) in
        // front of them (the DMA writes LDS) and drain the ring.  All 16
        // reads issue up front; half 0's MFMAs wait for the first 8.
        float4 X4[2][4], Y4[2][4];
#pragma unroll
        for (int hh = 0; hh < 2; hh++)
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const float* xr = cur + (64 * wx + 32 * i + li) * BK;
                const float* qr = cur + BN3 * BK + (64 * wq + 32 * i + li) * BK;
#pragma unroll
                for (int c = 0; c < 2; c++) {
                    const int cc = 2 * hh + c;
                    const int pc = (4 * lh + cc) ^ rsw;
                    X4[i][cc] = lds_ld4(xr + 4 * pc);
                    Y4[i][cc] = lds_ld4(qr + 4 * pc);
                }
            }
#pragma unroll
        for (int hh = 0; hh < 2; hh++) {
            if (hh == 0) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int c = 0; c < 2; c++) {
                const int cc = 2 * hh + c;
#pragma unroll
                for (int t = 0; t < 4; t++)
#pragma unroll
                    for (int i = 0; i < 2; i++)
#pragma unroll
                        for (int j = 0; j < 2; j++)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(X4[i][cc], t), f4get(Y4[j][cc], t),
                                                                             acc[i][j], 0, 0, 0);
            }
        }

        if (kb == nk - 1) {
            // ---------------- epilogue: selection over this 128 x 256 tile ----------------
            const int64_t row0 = tile * BN3;
            float qn[2];
            int qidx[2];
#pragma unroll
            for (int j = 0; j < 2; j++) {
                qidx[j] = 64 * wq + 32 * j + li;
                qn[j] = (METRIC == L2) ? a.qnorm2[q0 + qidx[j]] : 0.f;
            }
            const uint32_t* vb = a.valid + (row0 >> 5);
#pragma unroll
            for (int i = 0; i < 2; i++) {
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    int rt = 64 * wx + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    bool ok = (vb[rt >> 5] >> (rt & 31)) & 1u;
                    float xn = (METRIC == L2) ? a.xnorm2[row0 + rt] : 0.f;
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        float dot = acc[i][j][r];
                        float v;
                        if (METRIC == L2) v = (xn - 2.f * dot) + qn[j];
                        else if (METRIC == DOT) v = -dot;
                        else { v = 1.f - dot; v = v < 0.f ? 0.f : v; }
                        bool qok = (q0 + qidx[j]) < a.nq;
                        acc[i][j][r] = (ok && qok) ? v : __builtin_inff();
                    }
                }
            }
            uint64_t pending = ~0ull;
            for (;;) {
                ++epoch;
                float th[2] = {thr[qidx[0]], thr[qidx[1]]};
#pragma unroll
                for (int i = 0; i < 2; i++) {
#pragma unroll
                    for (int r = 0; r < 16; r++) {
#pragma unroll
                        for (int j = 0; j < 2; j++) {
                            const int vi = (i * 16 + r) * 2 + j;
                            if (!((pending >> vi) & 1ull)) continue;
                            float v = acc[i][j][r];
                            if (v < th[j]) {
                                int slot = atomicAdd(&cnt[qidx[j]], 1);
                                if (slot < C) {
                                    int rt = 64 * wx + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
                                    cbA[qidx[j] * C + slot] = v;
                                    cbI[qidx[j] * C + slot] = (uint32_t)(row0 + rt);
                                    pending &= ~(1ull << vi);
                                }
                                flags[0] = epoch;
                            } else {
                                pending &= ~(1ull << vi);
                            }
                        }
                    }
                }
                __syncthreads();
                if (flags[0] != epoch) break;
                for (int jq = 0; jq < QB / 8; jq++) {
                    const int q = wave + 8 * jq;
                    const int c = cnt[q];
                    if (c == 0) continue;
                    const int nc = c < C ? c : C;
                    const int64_t base = ((int64_t)(q0 + q) * a.nspans + span) * KP;
                    merge_query_list<R>(a.outA + base, a.outI + base, cbA + q * C, cbI + q * C, KP, C, nc, lane,
                                        &thr[q]);
                    if (lane == 0) {
                        if (c > C) flags[1] = epoch;
                        cnt[q] = 0;
                    }
                }
                __syncthreads();
                if (flags[1] != epoch) break;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// merge the per-span lists of each query (wave per query), keep KP best (A,id)
// ---------------------------------------------------------------------------
template <int R>
__global__ void k_merge_spans(const float* __restrict__ inA, const uint32_t* __restrict__ inI, int nq, int nspans,
                              int KP, float* __restrict__ outA, uint32_t* __restrict__ outI) {
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (q >= nq) return;
    float key[R];
    uint32_t id[R];
#pragma unroll
    for (int r = 0; r < R; r++) { key[r] = __builtin_inff(); id[r] = NO_ID; }
    // running best in e < KP; each round loads up to (64R-KP)/KP spans behind it
    const int per = (64 * R - KP) / KP;
    for (int s0 = 0; s0 < nspans; s0 += per) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            int e = r * 64 + lane;
            if (e >= KP) {
                int k = e - KP;
                int s = s0 + k / KP, w = k % KP;
                if (k / KP < per && s < nspans) {
                    int64_t off = ((int64_t)q * nspans + s) * KP + w;
                    key[r] = inA[off];
                    id[r] = inI[off];
                } else {
                    key[r] = __builtin_inff();
                    id[r] = NO_ID;
                }
            }
        }
        bitonic_sort<R>(key, id, lane);
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
        int e = r * 64 + lane;
        if (e < KP) { outA[(int64_t)q * KP + e] = key[r]; outI[(int64_t)q * KP + e] = id[r]; }
    }
}

// ---------------------------------------------------------------------------
// exact-order rescoring of the candidates (lane per (query, candidate))
// ---------------------------------------------------------------------------
template <int METRIC, int VARIANT>
__global__ __launch_bounds__(64) void k_rescore(const float* __restrict__ X, int dpad, const float* __restrict__ Q, int d,
                          const uint32_t* __restrict__ candI, int nq, int KP, float* __restrict__ outE) {
    int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)nq * KP) return;
    int q = (int)(p / KP);
    uint32_t id = candI[p];
    if (id == NO_ID) { outE[p] = __builtin_inff(); return; }
    outE[p] = exact_dist<METRIC, VARIANT>(Q + (int64_t)q * dpad, X + (int64_t)id * dpad, d);
}

// ---------------------------------------------------------------------------
// finalize: sort candidates by exact distance and prove equality with the
// reference heap result.  Proof obligations (DESIGN.md "exactness"):
//  * margin: every non-candidate j has A_j >= A_max and |A - E| <= eps, so if
//    E_(m) < A_max - eps the m smallest exact distances are all candidates;
//  * no ties among E_(1..m), m = min(k+1, n): then the heap (which keeps the
//    k smallest, flat/index.go:665-674) holds exactly these and extractHeap
//    returns them ascending.  Otherwise flag the query for k_replay.
// ---------------------------------------------------------------------------
template <int R>
__global__ void k_finalize(const float* __restrict__ candA, const uint32_t* __restrict__ candI,
                           const float* __restrict__ candE, const float* __restrict__ qnorm2, int nq, int KP,
                           int k, int kout, float eps_scale, float eps_base, int metric,
                           uint64_t id_base, uint64_t* __restrict__ out_ids, float* __restrict__ out_d,
                           int32_t* __restrict__ out_n, int32_t* __restrict__ flagged) {
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (q >= nq) return;
    float key[R];
    uint32_t id[R];
    float amax = -__builtin_inff();
    int nvalid = 0;
#pragma unroll
    for (int r = 0; r < R; r++) {
        int e = r * 64 + lane;
        if (e < KP) {
            key[r] = candE[(int64_t)q * KP + e];
            id[r] = candI[(int64_t)q * KP + e];
            if (id[r] != NO_ID) { amax = fmaxf(amax, candA[(int64_t)q * KP + e]); nvalid++; }
            else key[r] = __builtin_inff();
        } else { key[r] = __builtin_inff(); id[r] = NO_ID; }
    }
    // wave max / sum
    for (int o = 32; o > 0; o >>= 1) {
        amax = fmaxf(amax, __shfl_xor(amax, o));
        nvalid += __shfl_xor(nvalid, o);
    }
    bitonic_sort<R>(key, id, lane);
    const int m = (k + 1) < nvalid ? (k + 1) : nvalid;
    // eps: 2*gamma*(|q|*M + 1) for dot/cosine, 2*gamma*(|q| + M)^2 for l2
    float qn = sqrtf(qnorm2[q]);
    float eps;
    if (metric == L2) { float t = qn + eps_base; eps = eps_scale * t * t; }
    else eps = eps_scale * (qn * eps_base + 1.f);
    bool ok = true;
    if (nvalid >= KP) {
        // E_(m) is element m-1
        float em = 0.f;
#pragma unroll
        for (int r = 0; r < R; r++) {
            float v = __shfl(key[r], (m - 1) & 63);
            if (((m - 1) >> 6) == r) em = v;
        }
        ok = em < amax - eps;
    }
    // strict increase over elements 0..m-1
    bool inc = true;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const float up = __shfl_up(key[r], 1);
        const float wrap = (r > 0) ? __shfl(key[r > 0 ? r - 1 : 0], 63) : 0.f;
        const float pv = lane == 0 ? wrap : up;
        const int e = r * 64 + lane;
        if (e >= 1 && e < m && !(key[r] > pv)) inc = false;
    }
    inc = __all(inc);
    ok = ok && inc;
    if (!ok) {
        if (lane == 0) flagged[q] = 1;
        return;
    }
    if (lane == 0) flagged[q] = 0;
    const int nout = kout < nvalid ? kout : nvalid;
#pragma unroll
    for (int r = 0; r < R; r++) {
        int e = r * 64 + lane;
        if (e < nout) {
            out_ids[(int64_t)q * kout + e] = id_base + id[r];
            out_d[(int64_t)q * kout + e] = key[r];
        }
    }
    if (lane == 0) out_n[q] = nout;
}

// ---------------------------------------------------------------------------
// exact replay of the reference heap for flagged queries (one wave each)
// priorityqueue/queue.go:58-198 (NewMax), flat/index.go:578-619,665-688.
// ---------------------------------------------------------------------------
struct ReplayHeap {
    uint64_t* id;
    float* dist;
    int len;
};
__device__ __forceinline__ void rh_swap(ReplayHeap& h, int i, int j) {
    uint64_t ti = h.id[i]; h.id[i] = h.id[j]; h.id[j] = ti;
    float td = h.dist[i]; h.dist[i] = h.dist[j]; h.dist[j] = td;
}
__device__ void rh_insert(ReplayHeap& h, uint64_t id, float dist) {
    h.id[h.len] = id; h.dist[h.len] = dist; h.len++;
    int i = h.len - 1;
    while (i != 0 && h.dist[i] > h.dist[(i - 1) / 2]) { rh_swap(h, i, (i - 1) / 2); i = (i - 1) / 2; }
}
__device__ void rh_pop(ReplayHeap& h, uint64_t* id, float* dist) {
    *id = h.id[0]; *dist = h.dist[0];
    h.id[0] = h.id[h.len - 1]; h.dist[0] = h.dist[h.len - 1];
    h.len--;
    int i = 0;
    for (;;) {
        int l = 2 * i + 1, r = 2 * i + 2, s = i;
        if (l < h.len && h.dist[l] > h.dist[i]) s = l;
        if (r < h.len && h.dist[r] > h.dist[s]) s = r;
        if (s == i) break;
        rh_swap(h, i, s);
        i = s;
    }
}

// The same heap with each item one 16-byte LDS record (distance, id): a sift
// level reads both children with two ds_read_b128 issued together and moves
// one record with one ds_write_b128 -- one LDS round trip per level instead of
// ReplayHeap's separate distance / id loads and swaps.  Comparisons and final
// layout are rh_insert / rh_pop's (the hole moves instead of swapping, which
// leaves the same array).  Lane 0 runs it, like ReplayHeap.
struct __attribute__((aligned(16))) HeapRec {
    float d;
    uint32_t lo, hi, pad;
};
struct PHeap {
    HeapRec* r;
    int len;
};
// records move as one 4 x u32 vector (x = distance bits, y / z = id lo / hi):
// ds_read_b128 / ds_write_b128, selected with v_cndmask, never an aggregate
// copy (which the compiler put on the scratch stack)
typedef uint32_t hr_v4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint64_t hr_id(const HeapRec& x) { return ((uint64_t)x.hi << 32) | x.lo; }
__device__ __forceinline__ HeapRec hr_make(uint64_t id, float d) {
    HeapRec x;
    x.d = d;
    x.lo = (uint32_t)id;
    x.hi = (uint32_t)(id >> 32);
    x.pad = 0u;
    return x;
}
__device__ __forceinline__ hr_v4 hr_v(uint64_t id, float d) {
    return hr_v4{__float_as_uint(d), (uint32_t)id, (uint32_t)(id >> 32), 0u};
}
__device__ __forceinline__ void ph_insert(PHeap& h, uint64_t id, float v) {
    hr_v4* r = reinterpret_cast<hr_v4*>(h.r);
    int i = h.len++;
    while (i != 0) {  // up while dist[i] > dist[parent]
        const int p = (i - 1) >> 1;
        const hr_v4 rp = r[p];
        if (!(v > __uint_as_float(rp.x))) break;
        r[i] = rp;
        i = p;
    }
    r[i] = hr_v(id, v);
}
__device__ __forceinline__ void ph_pop(PHeap& h, uint64_t* id, float* dist) {
    hr_v4* r = reinterpret_cast<hr_v4*>(h.r);
    const hr_v4 top = r[0];
    *id = ((uint64_t)top.z << 32) | top.y;
    *dist = __uint_as_float(top.x);
    const int n = --h.len;
    const hr_v4 x = r[n];  // the last item moves to the root and sifts down
    const float xd = __uint_as_float(x.x);
    int i = 0;
    for (;;) {
        const int l = 2 * i + 1;
        if (l >= n) break;
        const bool hasr = l + 1 < n;
        const hr_v4 rl = r[l];
        const hr_v4 rr = r[hasr ? l + 1 : l];
        const float dl = __uint_as_float(rl.x), dr = __uint_as_float(rr.x);
        int s = i;
        float ds = xd;
        if (dl > ds) { s = l; ds = dl; }
        if (hasr && dr > ds) { s = l + 1; ds = dr; }
        if (s == i) break;
        r[i] = s == l ? rl : rr;
        i = s;
    }
    if (n > 0) r[i] = x;
}
// insertToHeap (flat/index.go:665-674): true when the item entered
__device__ __forceinline__ bool ph_offer(PHeap& h, int k, uint64_t id, float v) {
    if (h.len < k) { ph_insert(h, id, v); return true; }
    if (h.r[0].d > v) {
        uint64_t a;
        float b;
        ph_pop(h, &a, &b);
        ph_insert(h, id, v);
        return true;
    }
    return false;
}
// dynamic LDS of the packed replays: [k] records | [64] f32 | len (16 B)
__host__ __device__ constexpr size_t packed_replay_lds(int k) { return (size_t)k * sizeof(HeapRec) + 64 * sizeof(float) + 16; }

// (1) exact-order distances of every stored row to each listed query, plus
//     per-256-row block minima (valid rows only).  Block b handles query
//     f = b % F and rows [256*(b/F), +256): the F blocks of one row range are
//     dispatched back to back so the rows are re-read from cache.
constexpr int EBLK = 256;
template <int METRIC, int VARIANT>
__global__ __launch_bounds__(256) void k_exact_rows(const float* __restrict__ X, int dpad,
                                                    const uint32_t* __restrict__ valid, int64_t nslots,
                                                    const float* __restrict__ Q, int d,
                                                    const int32_t* __restrict__ qlist, int F, int64_t ld,
                                                    float* __restrict__ E, float* __restrict__ bmin) {
    __shared__ float red[4];
    const int f = blockIdx.x % F;
    const int64_t blk = blockIdx.x / F;
    const int64_t s = blk * EBLK + threadIdx.x;
    const float* qv = Q + (int64_t)qlist[f] * dpad;
    float e = __builtin_inff();
    bool ok = s < nslots && ((valid[s >> 5] >> (s & 31)) & 1u);
    if (ok) e = exact_dist<METRIC, VARIANT>(qv, X + s * dpad, d);
    if (s < ld) E[(int64_t)f * ld + s] = e;
    float m = ok ? e : __builtin_inff();
    for (int o = 32; o > 0; o >>= 1) m = fminf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float mm = fminf(fminf(red[0], red[1]), fminf(red[2], red[3]));
        bmin[(int64_t)f * (ld / EBLK) + blk] = mm;
    }
}

// (1b) k_exact_rows for QF queries per thread (the AVX2 accumulation order,
//      i.e. VARIANT AVX256, or AVX512 below 128 dims where both orders agree):
//      the thread's row is loaded once per 32-float block and stepped into the
//      QF queries' accumulators, cutting the uncoalesced row loads QF-fold.
//      Same order of operations per (query, row) as exact_raw's
//      32-block / 8-block / scalar-tail paths and reduce_ymm4.
template <int METRIC, int QF>
__device__ __forceinline__ void exact_raw_avx256_multi(const float* const (&q)[QF], const float* __restrict__ x, int n,
                                                       float (&out)[QF]) {
    float sum[QF];
    float acc[QF][4][8];
#pragma unroll
    for (int f = 0; f < QF; f++) {
        sum[f] = 0.f;
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int l = 0; l < 8; l++) acc[f][j][l] = 0.f;
    }
    if (n < 8) {
        for (int i = 0; i < n; i++) {
            const float xv = x[i];
#pragma unroll
            for (int f = 0; f < QF; f++) sum[f] = scalar_step<METRIC>(sum[f], q[f][i], xv);
        }
#pragma unroll
        for (int f = 0; f < QF; f++) out[f] = sum[f];
        return;
    }
    int e = 0;
    while (n - e >= 32) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
#pragma unroll
            for (int c = 0; c < 2; c++) {
                const float4 b = ld4(x + e + 8 * j + 4 * c);
#pragma unroll
                for (int f = 0; f < QF; f++) {
                    const float4 a = ld4(q[f] + e + 8 * j + 4 * c);
                    acc[f][j][4 * c + 0] = elem_step<METRIC>(acc[f][j][4 * c + 0], a.x, b.x);
                    acc[f][j][4 * c + 1] = elem_step<METRIC>(acc[f][j][4 * c + 1], a.y, b.y);
                    acc[f][j][4 * c + 2] = elem_step<METRIC>(acc[f][j][4 * c + 2], a.z, b.z);
                    acc[f][j][4 * c + 3] = elem_step<METRIC>(acc[f][j][4 * c + 3], a.w, b.w);
                }
            }
        }
        e += 32;
    }
    while (n - e >= 8) {
#pragma unroll
        for (int l = 0; l < 8; l++) {
            const float xv = x[e + l];
#pragma unroll
            for (int f = 0; f < QF; f++) acc[f][0][l] = elem_step<METRIC>(acc[f][0][l], q[f][e + l], xv);
        }
        e += 8;
    }
    for (; e < n; e++) {
        const float xv = x[e];
#pragma unroll
        for (int f = 0; f < QF; f++) sum[f] = scalar_step<METRIC>(sum[f], q[f][e], xv);
    }
#pragma unroll
    for (int f = 0; f < QF; f++) out[f] = sum[f] + reduce_ymm4(acc[f]);
}

template <int METRIC, int QF>
__global__ __launch_bounds__(256) void k_exact_rows_multi(const float* __restrict__ X, int dpad,
                                                          const uint32_t* __restrict__ valid, int64_t nslots,
                                                          const float* __restrict__ Q, int d,
                                                          const int32_t* __restrict__ qlist, int F, int64_t ld,
                                                          float* __restrict__ E, float* __restrict__ bmin) {
    __shared__ float red[4][QF];
    extern __shared__ __attribute__((aligned(16))) float qs[];  // [QF][dpad]: broadcast ds_reads, not VMEM
    const int FB = (F + QF - 1) / QF;
    const int fb = blockIdx.x % FB;
    const int64_t blk = blockIdx.x / FB;
    const int64_t s = blk * EBLK + threadIdx.x;
    for (int i = threadIdx.x; i < QF * dpad; i += 256) {
        const int f = i / dpad;
        const int ff = fb * QF + f < F ? fb * QF + f : fb * QF;  // duplicate a real query, never written
        qs[i] = Q[(int64_t)qlist[ff] * dpad + (i - f * dpad)];
    }
    __syncthreads();
    const float* qv[QF];
#pragma unroll
    for (int f = 0; f < QF; f++) qv[f] = qs + f * dpad;
    float e[QF];
#pragma unroll
    for (int f = 0; f < QF; f++) e[f] = __builtin_inff();
    const bool ok = s < nslots && ((valid[s >> 5] >> (s & 31)) & 1u);
    if (ok) {
        float r[QF];
        exact_raw_avx256_multi<METRIC == L2 ? L2 : DOT, QF>(qv, X + s * dpad, d, r);
#pragma unroll
        for (int f = 0; f < QF; f++) {
            if (METRIC == L2) e[f] = r[f];
            else if (METRIC == DOT) e[f] = -r[f];
            else { const float p = 1.f - r[f]; e[f] = p < 0.f ? 0.f : p; }
        }
    }
#pragma unroll
    for (int f = 0; f < QF; f++) {
        const int ff = fb * QF + f;
        if (ff < F && s < ld) E[(int64_t)ff * ld + s] = e[f];
        float m = e[f];
        for (int o = 32; o > 0; o >>= 1) m = fminf(m, __shfl_xor(m, o));
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][f] = m;
    }
    __syncthreads();
    if (threadIdx.x < QF) {
        const int f = threadIdx.x;
        const int ff = fb * QF + f;
        if (ff < F) bmin[(int64_t)ff * (ld / EBLK) + blk] = fminf(fminf(red[0][f], red[1][f]), fminf(red[2][f], red[3][f]));
    }
}

// (2) exact replay of the reference heap (priorityqueue NewMax +
//     insertToHeap, flat/index.go:578-688) over the precomputed distances, in
//     id order, one wave per listed query.  A 256-row block is skipped when the
//     heap is full and !(top > block_min): no row in it can pass insertToHeap's
//     `top.Dist > distance` test, and the top never increases.
// PK: the heap as packed 16-byte records (PHeap, default for k <= 8192); else ReplayHeap's split arrays
template <bool PK>
__global__ __launch_bounds__(64) void k_replay_scan(const float* __restrict__ E, const float* __restrict__ bmin,
                                                    const uint32_t* __restrict__ valid, int64_t nslots, int64_t ld,
                                                    const int32_t* __restrict__ qlist, int nlist, int k,
                                                    uint64_t id_base,
                                                    const uint64_t* __restrict__ in_hid,
                                                    const float* __restrict__ in_hd,
                                                    const int32_t* __restrict__ in_hlen, int extract,
                                                    int out_by_query, int kout, uint64_t* __restrict__ out_ids,
                                                    float* __restrict__ out_d, int32_t* __restrict__ out_n,
                                                    int in_by_query, int raw_by_query,
                                                    uint64_t* __restrict__ rec_i, float* __restrict__ rec_d,
                                                    int32_t* __restrict__ rec_n, int rec_cap) {
    // all LDS in the dynamic region (Guideline 17): PK: [k] records | [64] dists | len,
    // else [k] ids | [64] dists | [k] heap dists | len
    extern __shared__ __attribute__((aligned(16))) unsigned char rsm[];
    HeapRec* hr = reinterpret_cast<HeapRec*>(rsm);
    uint64_t* hid = reinterpret_cast<uint64_t*>(rsm);
    float* s_d = PK ? reinterpret_cast<float*>(hr + k) : reinterpret_cast<float*>(hid + k);
    float* hd = s_d + 64;
    int* s_len = PK ? reinterpret_cast<int*>(s_d + 64) : reinterpret_cast<int*>(hd + k);
    const int lane = threadIdx.x;
    const int li = blockIdx.x;
    if (li >= nlist) return;
    const int q = qlist[li];
    const float* Eq = E + (int64_t)li * ld;
    const float* Bq = bmin + (int64_t)li * (ld / EBLK);
    if (lane == 0) {
        int len = 0;
        if (in_hlen) {
            const int64_t ir = in_by_query ? q : li;
            len = in_hlen[ir];
            for (int i = 0; i < len; i++) {
                if (PK) hr[i] = hr_make(in_hid[ir * k + i], in_hd[ir * k + i]);
                else { hid[i] = in_hid[ir * k + i]; hd[i] = in_hd[ir * k + i]; }
            }
        }
        *s_len = len;
        if (rec_n) rec_n[li] = 0;
    }
    __syncthreads();
    const int64_t nblk = (nslots + EBLK - 1) / EBLK;
    for (int64_t b0 = 0; b0 < nblk; b0 += 64) {
        const float bm = (b0 + lane < nblk) ? Bq[b0 + lane] : __builtin_inff();
        int len = *s_len;
        float top = len > 0 ? (PK ? hr[0].d : hd[0]) : 0.f;
        uint64_t bmask = __ballot((b0 + lane < nblk) && (len < k || top > bm));
        while (bmask) {
            const int j = __builtin_ctzll(bmask);
            bmask &= bmask - 1;
            const float bmj = __shfl(bm, j);
            len = *s_len;
            top = len > 0 ? (PK ? hr[0].d : hd[0]) : 0.f;
            if (!(len < k || top > bmj)) continue;
            const int64_t r0 = (b0 + j) * EBLK;
            for (int sub = 0; sub < EBLK; sub += 64) {
                const int64_t s = r0 + sub + lane;
                const bool ok = s < nslots && ((valid[s >> 5] >> (s & 31)) & 1u);
                const float dist = ok ? Eq[s] : 0.f;
                len = *s_len;
                top = len > 0 ? (PK ? hr[0].d : hd[0]) : 0.f;
                uint64_t mask = __ballot(ok && (len < k || top > dist));
                if (mask == 0) continue;
                s_d[lane] = dist;
                __syncthreads();
                if (lane == 0) {
                    ReplayHeap h{hid, hd, *s_len};
                    PHeap ph{hr, *s_len};
                    while (mask) {
                        const int jj = __builtin_ctzll(mask);
                        mask &= mask - 1;
                        const float dj = s_d[jj];
                        const uint64_t idj = id_base + (uint64_t)(s - lane + jj);
                        bool ins = true;
                        if (PK) ins = ph_offer(ph, k, idj, dj);
                        else if (h.len < k) rh_insert(h, idj, dj);
                        else if (h.dist[0] > dj) { uint64_t a; float b; rh_pop(h, &a, &b); rh_insert(h, idj, dj); }
                        else ins = false;
                        if (ins && rec_n) {  // the parallel cross-shard replay's record (id order)
                            const int c = rec_n[li];
                            if (c < rec_cap) { rec_i[(int64_t)li * rec_cap + c] = idj; rec_d[(int64_t)li * rec_cap + c] = dj; }
                            rec_n[li] = c < rec_cap ? c + 1 : rec_cap + 1;
                        }
                    }
                    *s_len = PK ? ph.len : h.len;
                }
                __syncthreads();
            }
        }
    }
    if (lane == 0) {
        ReplayHeap h{hid, hd, *s_len};
        PHeap ph{hr, *s_len};
        if (extract) {
            // extractHeap (flat/index.go:676-688): pop max-first, fill from the back
            const int n = *s_len;
            const int64_t row = out_by_query ? q : li;
            for (int i = n - 1; i >= 0; i--) {
                uint64_t a; float b;
                if (PK) ph_pop(ph, &a, &b);
                else rh_pop(h, &a, &b);
                if (i < kout) { out_ids[row * kout + i] = a; out_d[row * kout + i] = b; }
            }
            out_n[row] = n < kout ? n : kout;
        } else {
            const int64_t row = raw_by_query ? q : li;
            const int n = *s_len;
            for (int i = 0; i < n; i++) {
                out_ids[row * k + i] = PK ? hr_id(hr[i]) : hid[i];
                out_d[row * k + i] = PK ? hr[i].d : hd[i];
            }
            out_n[row] = n;
        }
    }
}

// the worker-heap replay: packed records for k <= 8192, else the split layout (up to 13.6k)
constexpr int PACKED_REPLAY_MAX_K = 8192;
__host__ __forceinline__ size_t replay_scan_lds(int k) {
    return k <= PACKED_REPLAY_MAX_K ? packed_replay_lds(k)
                                    : (size_t)k * sizeof(uint64_t) + 64 * sizeof(float) + (size_t)k * sizeof(float) + 16;
}
template <class... A>
static inline hipError_t launch_replay_scan(int k, unsigned grid, hipStream_t st, A... args) {
    if (grid == 0) return hipSuccess;
    const size_t lds = replay_scan_lds(k);
    const void* fn = k <= PACKED_REPLAY_MAX_K ? (const void*)k_replay_scan<true> : (const void*)k_replay_scan<false>;
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    if (k <= PACKED_REPLAY_MAX_K) k_replay_scan<true><<<grid, 64, lds, st>>>(args...);
    else k_replay_scan<false><<<grid, 64, lds, st>>>(args...);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Provider.SingleDist over pairs, exact reference order (lane per pair)
// ---------------------------------------------------------------------------
template <int METRIC, int VARIANT>
__global__ __launch_bounds__(64) void k_distance_pairs(const float* __restrict__ A, const float* __restrict__ B, int64_t n, int d, int ld,
                                 float* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = exact_dist<METRIC, VARIANT>(A + i * ld, B + i * ld, d);
}

// exact normalisation of arbitrary rows into a padded buffer (queries):
// distancer.Normalize (normalize.go:16-32).  One wave per row: the squares are
// formed in parallel, the float32 sum runs serially in element order (every
// lane adds the same squares, read back from LDS by broadcast 16 at a time,
// so the sum is wave-uniform; a readlane per element cost 32 us per 768-d
// row in the dependent SGPR chain), then the divisions are parallel.
// rows [n, n_pad) of out are zeroed (the padded query group)
__global__ __launch_bounds__(256) void k_normalize_rows(const float* __restrict__ in, int64_t n, int d,
                                                        float* __restrict__ out, int ld, int64_t n_pad = 0) {
    __shared__ float ssq[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * 4 + w;
    if (i >= n) {
        if (i < n_pad)
            for (int c = lane; c < ld; c += 64) out[i * ld + c] = 0.f;
        return;
    }
    const float* src = in + i * d;
    float* dst = out + i * ld;
    float nrm = 0.f;
    for (int c0 = 0; c0 < d; c0 += 64) {
        const float v = c0 + lane < d ? src[c0 + lane] : 0.f;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the previous chunk's reads are done
        __builtin_amdgcn_wave_barrier();
        ssq[w][lane] = v * v;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int m = d - c0 < 64 ? d - c0 : 64;
        if (m == 64) {
#pragma unroll
            for (int j0 = 0; j0 < 64; j0 += 16) {
                float t[16];
#pragma unroll
                for (int j = 0; j < 16; j++) t[j] = ssq[w][j0 + j];
#pragma unroll
                for (int j = 0; j < 16; j++) nrm = nrm + t[j];
            }
        } else {
            for (int j = 0; j < m; j++) nrm = nrm + ssq[w][j];
        }
    }
    if (nrm == 0.f) {
        for (int c = lane; c < ld; c += 64) dst[c] = 0.f;
        return;
    }
    const float dv = (float)sqrt((double)nrm);
    for (int c = lane; c < ld; c += 64) dst[c] = c < d ? src[c] / dv : 0.f;
}

// hamming over uint64 words: popcount(a^b) summed, as float (distancer/hamming.go:63-68)
__global__ void k_hamming_pairs(const uint64_t* __restrict__ A, const uint64_t* __restrict__ B, int64_t n, int words,
                                float* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t s = 0;
    for (int w = 0; w < words; w++) s += (uint64_t)__popcll(A[i * words + w] ^ B[i * words + w]);
    out[i] = (float)s;
}

// BinaryQuantizer.Encode (compressionhelpers/binary_quantization.go:28-47)
__global__ void k_bq_encode(const float* __restrict__ in, int64_t n, int d, int ld, uint64_t* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int words = (d + 63) >> 6;
    if (i >= n * words) return;
    int64_t row = i / words;
    int w = (int)(i % words);
    const float* src = in + row * ld + 64 * w;
    int lim = d - 64 * w < 64 ? d - 64 * w : 64;
    uint64_t bits = 0;
    for (int b = 0; b < lim; b++)
        if (src[b] < 0.f) bits |= 1ull << b;
    out[i] = bits;
}

// copy rows into a zero-padded [n][ld] buffer (queries for l2 / dot)
__global__ void k_copy_pad_rows(const float* __restrict__ in, int64_t n, int d, float* __restrict__ out, int ld,
                                int64_t n_pad) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pad * ld) return;
    int64_t r = i / ld;
    int c = (int)(i % ld);
    out[i] = (r < n && c < d) ? in[r * d + c] : 0.f;
}

// squared norm of each padded row (approximate path + error bound only)
__global__ void k_row_norm2(const float* __restrict__ rows, int64_t n, int ld, float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r >= n) return;
    float s = 0.f;
    for (int c = lane; c < ld; c += 64) { float v = rows[r * ld + c]; s = fmaf(v, v, s); }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) out[r] = s;
}

// merge G shard lists [g][q][kin] (kin = k+1, ascending exact distances) into
// the final top-k; flag when a shard flagged q or the merged top k+1 tie.
template <int R>
__global__ void k_merge_shards(int G, int64_t nq, int k, const uint64_t* __restrict__ ids, const float* __restrict__ dd,
                               const int32_t* __restrict__ cnt, const int32_t* __restrict__ flg,
                               uint64_t* __restrict__ out_ids, float* __restrict__ out_d, int32_t* __restrict__ out_n,
                               int32_t* __restrict__ out_flags) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int kin = k + 1;
    float key[R];
    uint32_t pos[R];  // position g*kin + j
    int any_flag = 0;
    for (int g = lane; g < G; g += 64) any_flag |= flg[(int64_t)g * nq + q];
    any_flag = __any(any_flag);
#pragma unroll
    for (int r = 0; r < R; r++) {
        int e = r * 64 + lane;
        int g = e / kin, j = e % kin;
        if (g < G && j < cnt[(int64_t)g * nq + q]) { key[r] = dd[((int64_t)g * nq + q) * kin + j]; pos[r] = e; }
        else { key[r] = __builtin_inff(); pos[r] = NO_ID; }
    }
    // (dist, id) order; pos order == id order because shards hold ascending id ranges
    bitonic_sort<R>(key, pos, lane);
    int nvalid = 0;
#pragma unroll
    for (int r = 0; r < R; r++) nvalid += pos[r] != NO_ID;
    for (int o = 32; o > 0; o >>= 1) nvalid += __shfl_xor(nvalid, o);
    const int m = kin < nvalid ? kin : nvalid;
    bool inc = true;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const float up = __shfl_up(key[r], 1);
        const float wrap = (r > 0) ? __shfl(key[r > 0 ? r - 1 : 0], 63) : 0.f;
        const float pv = lane == 0 ? wrap : up;
        const int e = r * 64 + lane;
        if (e >= 1 && e < m && !(key[r] > pv)) inc = false;
    }
    inc = __all(inc);
    const int nout = k < nvalid ? k : nvalid;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int e = r * 64 + lane;
        if (e < nout) {
            const int g = pos[r] / kin, j = pos[r] % kin;
            out_ids[q * k + e] = ids[((int64_t)g * nq + q) * kin + j];
            out_d[q * k + e] = key[r];
        }
    }
    if (lane == 0) { out_n[q] = nout; out_flags[q] = (any_flag || !inc) ? 1 : 0; }
}

// synthetic data (same values as oracle or_gen_value)
__global__ void k_gen(int kind, uint64_t seed, uint64_t row0, int64_t rows, int d, float* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * d) return;
    int64_t r = i / d;
    int c = (int)(i % d);
    out[i] = gen_value(kind, seed, row0 + r, c);
}

}  // namespace
}  // namespace wv
