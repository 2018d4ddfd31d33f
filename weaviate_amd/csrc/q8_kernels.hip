// q8_kernels.hip -- int8 block keys for the exact fp32 flat search (DESIGN.md
// §3.1f).  The same pipeline as the bf16 block-key path (qs_kernels.hip:
// block keys -> k_blk_select -> k_blk_exact -> bounded replay), with the key
// pass on v_mfma_i32_16x16x64_i8: twice the bf16 MFMA rate per clock, and the
// integer products are exact, so the only approximation is the quantisation
// itself, bounded per row at Add time.
//
//   corpus   x^ = sb * X8, X8 in [-127, 127], one scale sb per 32-row block
//            (max |x| of the block / 127): the key epilogue stays one multiply
//            per (query, block) for dot / cosine.  k_block_q8 rebuilds a whole
//            block whenever one of its rows is written.
//   queries  q^ = sq * Q8, one scale per query (k_query_q8).
//   S        = fl(fl(sq * sb) * float(sum Q8 * X8)), the int32 sum exact.
//   |q.x - S| <= |q^| R + |q - q^| H + |q - q^| R + 4u |q^| H
//            (R = max |x - x^|, H = max |x^| over stored rows; the last term
//            the three roundings of S), i.e. qs_eps with gacc = 4u: the
//            selection, exact pass and replay of qs_kernels.hip apply as they
//            are.
//
// Plane layout: the bf16 plane's tiling with two int8 columns per bf16
// element (256-row tiles x 32-byte column chunks, q8_plane_byte), so the
// LDS-DMA pieces, ring slots and fragment addresses of k_qs_blockkey's
// one-block schedule carry over: a 64-column i8 MFMA chunk is a 32-column
// bf16 chunk's bytes.
#pragma once
#include "batch_row.h"

namespace wv {
namespace {

typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef int i32x16_t __attribute__((ext_vector_type(16)));
constexpr int Q8_NONE = (int)0x80000000;  // "no valid row" in the integer max

// (q8_plane_byte: qs_kernels.hip)

template <int OFF>
__device__ __forceinline__ i32x4_t lds_ld16_o(unsigned base) {
    i32x4_t v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(OFF));
    return v;
}

// valid bits of an allow list: slot = id - id_base, set when the slot is
// below hiwater and present; cnt counts the bits newly set (duplicate ids once)
__global__ void k_allow_bits(const uint64_t* __restrict__ ids, int64_t n, uint64_t id_base, int64_t hiwater,
                             const uint32_t* __restrict__ present, uint32_t* __restrict__ bits,
                             uint32_t* __restrict__ cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t id = ids[i];
    if (id < id_base || id - id_base >= (uint64_t)hiwater) return;
    const uint64_t sl = id - id_base;
    const uint32_t m = 1u << (sl & 31);
    if (!(present[sl >> 5] & m)) return;
    if (!(atomicOr(&bits[sl >> 5], m) & m)) atomicAdd(cnt, 1u);
}

// per-query allow bitmaps (wv_index_search_by_vector_batch_multi_allow): query
// q's vq words at bits + q * vq.  Queries without a list (qlist) take the
// present bitmap; a listed id sets its query's bit when the slot is present.
__global__ void k_pqa_present(const uint32_t* __restrict__ present, int64_t vq, const int32_t* __restrict__ qlist,
                              int64_t nl, uint32_t* __restrict__ bits) {
    const int64_t n = nl * vq;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = i / vq, w = i - j * vq;
        bits[(int64_t)qlist[j] * vq + w] = present[w];
    }
}

// ids [off[0], off[nq]) of all lists as given; thread per id, its query by
// binary search of the offsets (the last q with off[q] <= i)
__global__ void k_pqa_bits(const uint64_t* __restrict__ ids, const int64_t* __restrict__ off,
                           const int32_t* __restrict__ modes, int64_t nq, uint64_t id_base, int64_t hiwater,
                           const uint32_t* __restrict__ present, int64_t vq, uint32_t* __restrict__ bits) {
    const int64_t i = off[0] + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= off[nq]) return;
    int64_t lo = 0, hi = nq - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (off[mid] <= i) lo = mid; else hi = mid - 1;
    }
    if (modes[lo] == 0) return;
    const uint64_t id = ids[i - off[0]];
    if (id < id_base || id - id_base >= (uint64_t)hiwater) return;
    const uint64_t sl = id - id_base;
    const uint32_t m = 1u << (sl & 31);
    if (present[sl >> 5] & m) atomicOr(&bits[lo * vq + (int64_t)(sl >> 5)], m);
}

// per-query bitmaps from the caller's doc-id bitmaps (the bitmap form of the
// multi-allow call): raw holds each query's words from doc id (id_base & ~31)
// on (sw words per query, avail of them copied), so slot word w is the funnel
// shift of raw words w, w + 1 by id_base & 31; ANDed with present.  Unlisted
// queries (mode 0) take the present bitmap.  Thread per (query, word).
__global__ void k_pqa_from_bits(const uint32_t* __restrict__ raw, int64_t sw, int64_t avail,
                                const int32_t* __restrict__ modes, int64_t nq, int sh,
                                const uint32_t* __restrict__ present, int64_t vq, uint32_t* __restrict__ bits) {
    const int64_t n = nq * vq;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t q = i / vq, w = i - q * vq;
        uint32_t v = present[w];
        if (modes[q]) {
            const uint32_t* r = raw + q * sw;
            const uint32_t lo = w < avail ? r[w] : 0u, hi = w + 1 < avail ? r[w + 1] : 0u;
            v &= sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
        }
        bits[i] = v;
    }
}

// per-query bitmaps from the micro-batcher's slot-bitmap rows (batch_row.h:
// page-locked rows the callers filled, read in place); ANDed with present.
// Thread per (query, word).
__global__ void k_pqa_from_rows(const wv_batch_row* __restrict__ rows, const int32_t* __restrict__ modes, int64_t nq,
                                const uint32_t* __restrict__ present, int64_t vq, uint32_t* __restrict__ bits) {
    const int64_t n = nq * vq;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t q = i / vq, w = i - q * vq;
        uint32_t v = present[w];
        if (modes[q]) v &= w < rows[q].words ? rows[q].dev[w] : 0u;
        bits[i] = v;
    }
}

// union of the nq bitmaps (the block keys' row set), thread per word
__global__ void k_pqa_union(const uint32_t* __restrict__ bits, int64_t vq, int64_t nq, uint32_t* __restrict__ uni) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= vq) return;
    uint32_t u = 0;
    for (int64_t q = 0; q < nq; q++) u |= bits[q * vq + w];
    uni[w] = u;
}

// gathered allow-list search: stored rows slots[i] -> row i of a sub-index
// (fp32 row with its padding, |x|^2, and the bf16 plane row), thread per
// (row, 16-byte piece); rows in [n, n_pad) are zeroed
__global__ void k_gather_rows(const float* __restrict__ X, const float* __restrict__ xn2, int dpad,
                              const uint16_t* __restrict__ Xb, int dpb, const uint32_t* __restrict__ slots, int64_t n,
                              int64_t n_pad, float* __restrict__ Xo, float* __restrict__ xn2o, uint16_t* __restrict__ Xbo) {
    const int per = dpad / 4 + (Xb ? dpb / 8 : 0) + 1;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pad * per) return;
    const int64_t r = i / per;
    const int p = (int)(i % per);
    const bool live = r < n;
    const int64_t sl = live ? (int64_t)slots[r] : 0;
    if (p < dpad / 4) {
        const float4 v = live ? reinterpret_cast<const float4*>(X + sl * dpad)[p] : make_float4(0.f, 0.f, 0.f, 0.f);
        reinterpret_cast<float4*>(Xo + r * dpad)[p] = v;
    } else if (p < dpad / 4 + (Xb ? dpb / 8 : 0)) {
        const int c = (p - dpad / 4) * 8;  // 8 bf16 columns: one 16-byte half of a 32-byte chunk row
        const uint4 v = live ? *reinterpret_cast<const uint4*>(Xb + bf3_plane_index(sl, c, dpb)) : make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(Xbo + bf3_plane_index(r, c, dpb)) = v;
    } else {
        xn2o[r] = live ? xn2[sl] : 0.f;
    }
}

// ids[q][j] = id_base + slots[ids[q][j]] for j < counts[q] (sub-index positions -> doc ids)
__global__ void k_remap_ids(uint64_t* __restrict__ ids, const int32_t* __restrict__ counts, int64_t nq, int k,
                            const uint32_t* __restrict__ slots, uint64_t id_base) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq * k) return;
    const int64_t q = i / k;
    if ((int)(i % k) >= counts[q]) return;
    ids[i] = id_base + slots[ids[i]];
}

// n copies of a 32-bit word (e.g. +inf block minima of an empty shard)
__global__ void k_fill_u32(uint32_t* __restrict__ p, int64_t n, uint32_t v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

__device__ __forceinline__ int q8_code(float x, float inv) {
    const float c = rintf(x * inv);
    return (int)fminf(127.f, fmaxf(-127.f, c));
}

// ---------------------------------------------------------------------------
// k_block_q8: one workgroup (4 waves) per 32-row block: sb = max |x| / 127 over
// the block's 32 stored rows (present or not: a stale or zero row only costs
// precision), X8 = rint(x / sb) clamped to +-127, and per row
// |x - sb X8|^2, |sb X8|^2 into the index maxima qmax8[0], qmax8[1]
// (atomicMax on float bits); qmax8[2] = 1 once a block holds a non-finite
// value (the int8-only planes above 1536 dims have no bf16 plane to flag it).
// Blocks blist[i] or b0 + i.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_block_q8(const float* __restrict__ X, int dpad, int dims, int dpb8,
                                                  const uint32_t* __restrict__ blist, int64_t b0,
                                                  unsigned char* __restrict__ X8, float* __restrict__ sb8,
                                                  uint32_t* __restrict__ qmax8) {
    __shared__ float smax[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t blk = blist ? (int64_t)blist[blockIdx.x] : b0 + blockIdx.x;
    const int64_t r0 = blk * 32;
    float m = 0.f;
    bool bad = false;
    for (int r = 8 * w; r < 8 * w + 8; r++) {
        const float* x = X + (r0 + r) * dpad;
        for (int c = lane; c < dims; c += 64) {
            const float v = x[c];
            m = fmaxf(m, fabsf(v));
            bad |= !__builtin_isfinite(v);
        }
    }
    if (__any(bad) && lane == 0) atomicOr(&qmax8[2], 1u);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) smax[w] = m;
    __syncthreads();
    m = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
    const float sb = m / 127.f;
    const float inv = m > 0.f ? 127.f / m : 0.f;
    if (threadIdx.x == 0) sb8[blk] = sb;
    for (int r = 8 * w; r < 8 * w + 8; r++) {
        const int64_t row = r0 + r;
        const float* x = X + row * dpad;
        float sr = 0.f, sh = 0.f;
        for (int c4 = 4 * lane; c4 < dpb8; c4 += 256) {
            uint32_t word = 0;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int c = c4 + e;
                const float v = c < dims ? x[c] : 0.f;
                const int q = q8_code(v, inv);
                const float h = sb * (float)q;       // x^ component (one rounding)
                const float rv = fmaf(-sb, (float)q, v);  // x - x^ (one rounding)
                sr = fmaf(rv, rv, sr);
                sh = fmaf(h, h, sh);
                word |= (uint32_t)(q & 0xFF) << (8 * e);
            }
            *reinterpret_cast<uint32_t*>(X8 + q8_plane_byte(row, c4, dpb8)) = word;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            sr += __shfl_xor(sr, o);
            sh += __shfl_xor(sh, o);
        }
        if (lane == 0) {
            atomicMax(&qmax8[0], __float_as_uint(sr));
            atomicMax(&qmax8[1], __float_as_uint(sh));
        }
    }
}

// k_query_q8: wave per query row of Qn (rows [nq, nq_pad) are zero): sq =
// max |q| / 127, Q8 into the tiled query plane, qscale[q] = sq, and
// qinfo8[q] = (|q|^2, |q^|^2, |q - q^|^2, non-finite ? 1 : 0), |q|^2 and the
// non-finite flag taken from k_query_split's qinfo16 (one |q|^2 per query on
// every path).
__global__ void k_query_q8(const float* __restrict__ Qn, int dpad, int dims, int dpb8, int64_t nq, int64_t nq_pad,
                           const float4* __restrict__ qinfo16, unsigned char* __restrict__ Q8,
                           float* __restrict__ qscale, float4* __restrict__ qinfo8) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (q >= nq_pad) return;
    const float* x = Qn + q * dpad;
    float m = 0.f;
    bool bad = false;
    if (q < nq)
        for (int c = lane; c < dims; c += 64) {
            const float v = x[c];
            m = fmaxf(m, fabsf(v));
            bad |= !__builtin_isfinite(v);
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    bad = __any(bad);
    const float sq = m / 127.f;
    const float inv = m > 0.f ? 127.f / m : 0.f;
    float sh = 0.f, sr = 0.f;
    for (int c4 = 4 * lane; c4 < dpb8; c4 += 256) {
        uint32_t word = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int c = c4 + e;
            const float v = (q < nq && c < dims) ? x[c] : 0.f;
            const int cq = bad ? 0 : q8_code(v, inv);
            const float h = sq * (float)cq;
            const float rv = fmaf(-sq, (float)cq, v);
            sh = fmaf(h, h, sh);
            sr = fmaf(rv, rv, sr);
            word |= (uint32_t)(cq & 0xFF) << (8 * e);
        }
        *reinterpret_cast<uint32_t*>(Q8 + q8_plane_byte(q, c4, dpb8)) = word;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        sh += __shfl_xor(sh, o);
        sr += __shfl_xor(sr, o);
    }
    if (lane == 0) {
        const float4 q16 = qinfo16[q];
        qscale[q] = sq;
        qinfo8[q] = make_float4(q16.x, sh, sr, (bad || q16.w != 0.f || !(sh < 1e30f)) ? 1.f : 0.f);
    }
}

}  // namespace
// external linkage: the key-pass launcher (qs_runtime.hip) serves other units
struct Q8Args {
    const unsigned char* X8;   // corpus int8 plane, tiled (q8_plane_byte, dpb8 columns)
    const float* sb;           // [cap/32] block scales
    const float* xnorm2;       // [cap] |x|^2 of the stored fp32 rows (L2)
    const uint32_t* valid;     // [cap/32] slots to scan (present & allowed)
    const unsigned char* Q8;   // query int8 plane, tiled, nq_pad rows (multiple of 256)
    const float* qscale;       // [nq_pad]
    float* key;                // [nq_pad][ldk] block keys
    int64_t ldk;
    int64_t nslots;            // ring steps (RB 32-row blocks each) to scan
    int slots_per_span;
    int nspans;
    int nqg;                   // query groups of 256
    int bq_bits;               // BQ: code bits 64 * words (hamming = (bq_bits - dot) / 2)
    int64_t nq_live = 1ll << 62;  // k_q8_blockkey<.., LIVE>: the launch's real queries (the rest is padding)
    int prio = 0;                 // k_q8_blockkey: 1 = waves 4-7 at s_setprio 1 for the whole loop
    // k_q8_blockkey<.., MASK>: per-query row bitmaps (query q's word for block b
    // at qmask[q * qmask_ld + b]; queries past qmask_n read row qmask_n - 1)
    const uint32_t* qmask = nullptr;
    int64_t qmask_ld = 0;
    int64_t qmask_n = 1;
};
namespace {

// ---------------------------------------------------------------------------
// k_q8_blockkey<NC, RB, L2>: block keys of 256 queries (8 waves x 32) x one
// span of the corpus, NC 64-column chunks per 32-row block, RB blocks per LDS
// ring slot (3 slots, RB * 2NC KiB each, LDS-DMA filled two steps ahead).
//   key (L2)      = min over the block's valid rows of fl(xnorm2 - 2 S)
//   key (dot/cos) = -max over the block's valid rows of S
// S = fl(fl(sq * sb) * float(sum_k Q8 X8)); a block with no valid row: +inf.
// Per chunk: 2 A-fragment reads (row halves), 4 v_mfma_i32_16x16x64_i8 (2 row
// halves x 2 query halves), one DMA piece of the group two steps ahead.  The
// reduction over a block's rows runs beside the next block's MFMAs (RB = 2)
// or after the slot; the cross-lane combine + key store of a slot's last
// block is deferred into the next slot.  One barrier per slot.
// ---------------------------------------------------------------------------
// STAG (RB = 2): waves 4-7 -- each the SIMD partner of wave w - 4 -- run every
// block's reduction P0 chunks into the next block instead of right after it
// (MI355X_MICROARCH.md, two waves per SIMD, item 9: a stagger), so the two
// waves of a SIMD do not issue their epilogue VALU at the same time.
//
// BQ (bq_kernels.hip's block minima on the matrix cores): X8 / Q8 are the
// codes unpacked to +-1 (bit 0 -> +1, bit 1 -> -1; columns past the code bits
// 0), so sum s_q s_x = bq_bits - 2 hamming exactly in int32; the kernel writes
// the minimum hamming distance of every 32-row block (+inf without a valid
// row) -- 8x finer than the VALU kernels' 256-row minima, so the replay
// (k_bq_replay<.., 32>) recomputes 8x fewer rows per visited block.
// PF: A-fragment reads PF chunks ahead of their MFMAs (PF + 1 register sets).
// PAIR (RB = 2, in-order schedule): a slot's two blocks share one cross-lane
// combine and one 64-lane key store.  Each block's reduction leaves, per lane,
// the partial of its row group for both query halves -- raw int32 maxima for
// dot/cos/BQ (the positive scale commutes with the maximum, so it is applied
// once after the combine), fl(xnorm2 - 2S) minima for L2 -- and the combine is
// a transpose-reduction: permlane32 swaps pair (A half 0, A half 1) and (B half
// 0, B half 1), one permlane16 swap pairs the two results, three max/min ops
// in all, ending with lane group G = lane >> 4 holding block A / B (G & 1) of
// query half G >> 1.  The unpaired form takes five swaps and four ops per
// block and stores from 32 lanes.
// DBG (timing experiments in a -DWV_QS_DBG build only, wrong results): bit 0
// drops the plane DMA, bit 1 the MFMAs, bit 2 the block reductions and stores,
// bit 3 the key stores only.
// MASK (PAIR, dot / cosine): per-query allow bitmaps (the multi-allow batch):
// a block's key for query q is the maximum over the rows of q's own list only
// (a.qmask word of q and the block ANDed with the valid word), so each query's
// keys bound its own rows -- the plain select and proof then apply per query.
// One more LDS-DMA op per wave and group: the 64 mask words of the wave's 32
// queries x the slot's 2 blocks, laid out [block][query j][half n] so a lane
// reads its two queries' words of a block with one ds_read_b64.
// LIVE (PAIR schedule; a batch that is not a multiple of 256 queries): a wave
// whose 32 queries all lie at or past a.nq_live -- the padding of the last
// query group -- reads no fragments and issues no MFMA or reduction; it still
// issues its share of every slot's DMA and its key stores (+inf), so each
// wave's vector-memory counts, which the ring's vmcnt waits rely on, are those
// of the full schedule.  A batch of 64 queries runs the MFMAs of 2 waves
// instead of 8 (the HBM stream of the plane is then the bound).
template <int NC, int RB, bool ISL2, bool STAG = false, bool BQ = false, int PF = 1, int DBG = 0, bool LIVE = false,
          bool MASK = false>
__global__ __launch_bounds__(512, 2) void k_q8_blockkey(Q8Args a) {
    constexpr int NPB = 2 * NC;                     // 1 KiB pieces per 32-row block
    constexpr int SLOT = RB * NPB * 1024;           // bytes per ring slot
    constexpr int P = RB * NPB / 8;                 // pieces per wave per slot
    static_assert((RB * NPB) % 8 == 0, "pieces per slot must split over 8 waves");
    static_assert(RB == 1 || RB == 2, "RB must be 1 or 2");
    constexpr int64_t TILE_B = (int64_t)NPB * 8192;  // bytes per 256-row tile of a plane
    constexpr int NT = RB * NC;                     // chunks per slot
    constexpr int P0 = P + 2 + (ISL2 ? 1 : 0) + (MASK ? 1 : 0);  // vector-memory ops per group, per wave
    static_assert(P0 < NC, "the deferred key store must follow the slot's DMA pieces");
    static_assert(PF >= 1 && PF + 1 < NC, "prefetch distance");
    static_assert(!STAG || RB == 2, "the stagger defers a slot's second block");
    static_assert(!BQ || (!ISL2 && !STAG), "BQ: integer maxima, in-order schedule");
    static_assert(!LIVE || (RB == 2 && !STAG && !BQ && DBG == 0), "LIVE: the paired in-order schedule");
    static_assert(!MASK || (RB == 2 && !STAG && !BQ && !ISL2 && DBG == 0), "MASK: paired dot / cosine keys");
    constexpr int X0 = 1;                           // chunk of the slot's extra LDS reads
    constexpr int XE = 2 + (ISL2 ? 2 * RB : 0) + (MASK ? 2 : 0);  // extra reads: valid words, scales (+ norms / masks)
    constexpr int NBUF = 3;
    extern __shared__ __attribute__((aligned(16))) unsigned char qsm[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int total = a.nqg * a.nspans;
    const int b = blockIdx.x;
    // XCD-aware order: the query groups of one span share an XCD (its L2)
    const int logical = (total % 8 == 0) ? (b % 8) * (total / 8) + (b / 8) : b;
    const int span = logical / a.nqg, grp = logical % a.nqg;
    // uniform: grp from blockIdx, wave readfirstlane'd
    const bool act = !LIVE || (int64_t)grp * 256 + wave * 32 < a.nq_live;

    // this wave's 32 queries as B fragments: Qf[2c + n] = chunk c, query half
    // n: lane (j = lane & 15, kq = lane >> 4) holds query wave*32 + 16n + j,
    // columns 64c + 16kq .. +15
    i32x4_t Qf[2 * NC];
    const int64_t q0 = (int64_t)grp * 256 + wave * 32;
    if (act) {
        const int j = lane & 15, kq = lane >> 4;
        const unsigned char* qp =
            a.Q8 + (int64_t)grp * TILE_B + (kq >> 1) * 8192 + (wave * 32 + j) * 32 + 16 * (kq & 1);
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int n = 0; n < 2; n++)
                Qf[2 * c + n] = *reinterpret_cast<const i32x4_t*>(qp + (2 * c) * 8192 + n * 16 * 32);
    }
    const float sqA = BQ ? 1.f : a.qscale[q0 + (lane & 15)];
    const float sqB = BQ ? 1.f : a.qscale[q0 + 16 + (lane & 15)];
    constexpr bool PAIR = RB == 2 && !STAG;
    // PAIR: the query of the lane's combined key (group G: half G >> 1)
    const float sqO = (BQ || !PAIR) ? 1.f : a.qscale[q0 + (lane & 15) + 16 * (lane >> 5)];
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): retire the query loads before the DMA ring

    const int64_t s0 = (int64_t)span * a.slots_per_span;
    int64_t s1 = s0 + a.slots_per_span;
    if (s1 > a.nslots) s1 = a.nslots;
    const int nsteps = s1 > s0 ? (int)(s1 - s0) : 0;

    const uint32_t src_lane = (uint32_t)(16 * lane);
    const unsigned ring = lds_addr(qsm);
    // per-wave rings of 4 entries (step & 3): valid words [8][4][16 B], block
    // scales [8][4][16 B], L2 norms [8][4][RB * 128 B]; every wave loads its own
    // copy, so every wave issues the same vector-memory ops per step
    const unsigned vring = ring + NBUF * SLOT + (unsigned)wave * 64u;
    const unsigned sring = ring + NBUF * SLOT + 512u + (unsigned)wave * 64u;
    const unsigned xnring = ring + NBUF * SLOT + 1024u + (unsigned)wave * (unsigned)(4 * RB * 128);
    // MASK: [8 waves][4 steps][64 words] per-query mask words (after the valid / scale rings)
    const unsigned mring = ring + NBUF * SLOT + 1024u + (unsigned)wave * 1024u;
    const int64_t tile0 = (s0 * RB * 32) >> 8;
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.X8 + tile0 * TILE_B), (short)0, -1, 0x00020000);
    int64_t igb = s0 * RB;
    uint32_t ioff = (uint32_t)(((igb >> 3) - tile0) * TILE_B + (igb & 7) * 1024);
    auto issue_piece = [&](int j, int t, int slot) {
        if (j < P) {
            if constexpr (DBG & 1) return;
            const int p = wave + 8 * j;
            const int rb = p / NPB, c = p % NPB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(size_t)(ring + (unsigned)(slot * SLOT + (rb * NPB + c) * 1024)),
                                                     16, src_lane, ioff + (uint32_t)(rb * 1024 + c * 8192), 0, 0);
        } else if (j == P) {
            if (lane < RB)
                __builtin_amdgcn_global_load_lds(a.valid + igb + lane, (lds_ptr_t)(size_t)(vring + (unsigned)((t & 3) * 16)), 4,
                                                 0, 0);
        } else if (j == P + 1) {
            if (lane < RB)
                __builtin_amdgcn_global_load_lds(a.sb + igb + lane, (lds_ptr_t)(size_t)(sring + (unsigned)((t & 3) * 16)), 4,
                                                 0, 0);
        } else if constexpr (MASK) {
            // lane (block rb, query j, half n) -> LDS word rb * 32 + 2 j + n
            const int rbm = lane >> 5, jq = (lane >> 1) & 15, hn = lane & 1;
            int64_t qq = q0 + 16 * hn + jq;
            if (qq >= a.qmask_n) qq = a.qmask_n - 1;
            __builtin_amdgcn_global_load_lds(a.qmask + qq * a.qmask_ld + igb + rbm,
                                             (lds_ptr_t)(size_t)(mring + (unsigned)((t & 3) * 256)), 4, 0, 0);
        } else {
            if (lane < RB * 8)
                __builtin_amdgcn_global_load_lds(a.xnorm2 + igb * 32 + 4 * lane,
                                                 (lds_ptr_t)(size_t)(xnring + (unsigned)((t & 3) * RB * 128)), 16, 0, 0);
        }
        if (j == P0 - 1) {
            igb += RB;
            ioff += RB * 1024;
            if ((igb & 7) == 0) ioff += (uint32_t)(TILE_B - 8192);
        }
    };
    auto issue_group = [&](int t, int slot) {
#pragma unroll
        for (int j = 0; j < P0; j++) issue_piece(j, t, slot);
    };

    const int64_t qrow = q0 + (lane & 31);
    float* krow = a.key + qrow * a.ldk;
    // lane (i = lane&15, kq = lane>>4) reads row 16m+i, columns 64c+16kq..+15
    // = piece 2c + (kq>>1), bytes 16(kq&1).. of the row (linear image)
    const unsigned l16 = (unsigned)(((lane >> 5) & 1) * 1024 + (lane & 15) * 32 + 16 * ((lane >> 4) & 1));
    constexpr int NB2 = PF + 1;
    i32x4_t B2[NB2][2];  // A fragments [chunk % NB2][row half m]
    // the first PF chunks of a slot, right after its barrier
    auto head_reads = [&](unsigned sbh) {
        static_for<0, PF>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if constexpr (j < NT) {
                constexpr int o = (j / NC * NPB + 2 * (j % NC)) * 1024;
                B2[j % NB2][0] = lds_ld16_o<o>(sbh);
                B2[j % NB2][1] = lds_ld16_o<o + 512>(sbh);
            }
        });
    };
    if (nsteps > 0) {
        issue_group(0, 0);
        if (nsteps > 1) issue_group(1, 1);
        qs_wait_vm(nsteps > 1 ? P0 : 0);  // group 0 landed, group 1 may stay in flight
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (act) head_reads(ring + l16);
    }
    // the pending block (a slot's last): per query half n the lane's partial
    // key before the cross-lane combine
    float mp0 = 0.f, mp1 = 0.f;
    int64_t gbp = 0;
    int dbg_sink = 0;  // DBG & 4: keeps the MFMAs live without the reductions; DBG & 8: the keys without stores
    auto finish = [&](float p0, float p1, int64_t gb) {
        // lanes g*16 + j (g = 0..3) hold partial keys of query 16n + j
        float m0 = p0, m1 = p1;
        const auto a0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m0), __float_as_uint(m0), false, false);
        const auto a1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m1), __float_as_uint(m1), false, false);
        m0 = ISL2 ? fminf(m0, __uint_as_float(a0[1])) : fmaxf(m0, __uint_as_float(a0[1]));
        m1 = ISL2 ? fminf(m1, __uint_as_float(a1[1])) : fmaxf(m1, __uint_as_float(a1[1]));
        const auto b0 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m0), __float_as_uint(m0), false, false);
        const auto b1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m1), __float_as_uint(m1), false, false);
        m0 = ISL2 ? fminf(m0, __uint_as_float(b0[1])) : fmaxf(m0, __uint_as_float(b0[1]));
        m1 = ISL2 ? fminf(m1, __uint_as_float(b1[1])) : fmaxf(m1, __uint_as_float(b1[1]));
        // lanes 0-15: queries j (n = 0) in m0, 16 + j in m1 -> lanes 16-31 take m1
        const auto c01 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m0), __float_as_uint(m1), false, false);
        const float m = __uint_as_float(c01[0]);
        if constexpr ((DBG & 8) != 0) {
            dbg_sink ^= __float_as_int(m);
            return;
        }
        if constexpr (BQ) {
            if (lane < 32) krow[gb] = m == -__builtin_inff() ? __builtin_inff() : 0.5f * ((float)a.bq_bits - m);
        } else {
            if (lane < 32) krow[gb] = ISL2 ? m : -m;
        }
    };
    // PAIR: the combine of a slot's two blocks (raw partials rA*, rB*, block
    // scales sbA_, sbB_) and the 64-lane store of blocks gbA, gbA + 1
    auto finish2 = [&](uint32_t rA0, uint32_t rA1, uint32_t rB0, uint32_t rB1, float sbA_, float sbB_, int64_t gbA) {
        auto op = [](uint32_t x, uint32_t y) -> uint32_t {
            if constexpr (ISL2) return __float_as_uint(fminf(__uint_as_float(x), __uint_as_float(y)));
            else return (uint32_t)max((int)x, (int)y);
        };
        const auto sa = __builtin_amdgcn_permlane32_swap(rA0, rA1, false, false);
        const auto sb2 = __builtin_amdgcn_permlane32_swap(rB0, rB1, false, false);
        const uint32_t w = op(sa[0], sa[1]), u = op(sb2[0], sb2[1]);
        const auto sw = __builtin_amdgcn_permlane16_swap(w, u, false, false);
        const uint32_t r = op(sw[0], sw[1]);
        float key;
        if constexpr (ISL2) {
            key = __uint_as_float(r);
        } else {
            const int mi = (int)r;
            if constexpr (BQ) {
                key = mi == Q8_NONE ? __builtin_inff() : 0.5f * ((float)a.bq_bits - (float)mi);
            } else {
                const float s = sqO * (((lane >> 4) & 1) ? sbB_ : sbA_);
                key = mi == Q8_NONE ? __builtin_inff() : -(s * (float)mi);
            }
        }
        if constexpr ((DBG & 8) != 0) {
            dbg_sink ^= __float_as_int(key);
            return;
        }
        a.key[(q0 + (lane & 15) + 16 * (lane >> 5)) * a.ldk + gbA + ((lane >> 4) & 1)] = key;
    };
    // stores issued in slot t (the deferred finish + block 0's), for vmcnt
    auto stores_in = [&](int t) -> int { return (t > 0 ? 1 : 0) + (PAIR ? 0 : RB - 1); };
    constexpr int SPS = PAIR ? 1 : RB;  // key stores per slot
    // a block's reduction over its rows (accumulators ac, valid word vw_, scale
    // sb_, L2 norms xa_/xb_) -> the lane's partial keys (p0, p1)
    auto reduce = [&](const i32x4_t (&ac)[2][2], uint32_t vw_, float sb_, const f32x4_t& xa_, const f32x4_t& xb_,
                      float& p0, float& p1) {
        const uint32_t vw = __builtin_amdgcn_readfirstlane(vw_);
        const float sbf = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(sb_)));
        // ac[m][n][r] is row 16m + 4g + r (g = lane>>4) of query 16n + (lane&15)
        const uint32_t vl = vw >> (4 * ((lane >> 4) & 3));
        const float s0f = sqA * sbf, s1f = sqB * sbf;
        float mn[2];
        // the all-valid case (every block but a span's ragged tail, deletions and
        // allow lists) is one uniform branch around both query halves, so the
        // masked form's bit tests are not computed for it
        if (vw == 0xFFFFFFFFu) {
#pragma unroll
            for (int n = 0; n < 2; n++) {
                if constexpr (ISL2) {
                    const float cn = -2.f * (n ? s1f : s0f);
                    float m = __builtin_inff();
#pragma unroll
                    for (int mm = 0; mm < 2; mm++)
#pragma unroll
                        for (int r = 0; r < 4; r++)
                            m = fminf(m, fmaf(cn, (float)ac[mm][n][r], mm ? xb_[r] : xa_[r]));
                    mn[n] = m;
                } else {
                    const int mi = max(max(max(ac[0][n][0], ac[0][n][1]), max(ac[0][n][2], ac[0][n][3])),
                                       max(max(ac[1][n][0], ac[1][n][1]), max(ac[1][n][2], ac[1][n][3])));
                    if constexpr (BQ) mn[n] = (float)mi;
                    else mn[n] = (n ? s1f : s0f) * (float)mi;
                }
            }
        } else {
#pragma unroll
            for (int n = 0; n < 2; n++) {
                if constexpr (ISL2) {
                    const float cn = -2.f * (n ? s1f : s0f);
                    float m = __builtin_inff();
#pragma unroll
                    for (int mm = 0; mm < 2; mm++)
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            const float v = fmaf(cn, (float)ac[mm][n][r], mm ? xb_[r] : xa_[r]);
                            m = fminf(m, ((vl >> (16 * mm + r)) & 1u) ? v : __builtin_inff());
                        }
                    mn[n] = m;
                } else {
                    int mi = Q8_NONE;
#pragma unroll
                    for (int mm = 0; mm < 2; mm++)
#pragma unroll
                        for (int r = 0; r < 4; r++)
                            mi = max(mi, ((vl >> (16 * mm + r)) & 1u) ? ac[mm][n][r] : Q8_NONE);
                    // the scale is positive: the largest S is the largest product
                    if constexpr (BQ) mn[n] = mi == Q8_NONE ? -__builtin_inff() : (float)mi;
                    else mn[n] = mi == Q8_NONE ? -__builtin_inff() : (n ? s1f : s0f) * (float)mi;
                }
            }
        }
        p0 = mn[0];
        p1 = mn[1];
    };
    // PAIR: a block's raw per-lane partials (see finish2)
    auto reduce_raw = [&](const i32x4_t (&ac)[2][2], uint32_t vw_, float sb_, const f32x4_t& xa_, const f32x4_t& xb_,
                          uint32_t& r0, uint32_t& r1, uint2 mw = uint2{0u, 0u}) {
        const uint32_t vw = __builtin_amdgcn_readfirstlane(vw_);
        const uint32_t vl = vw >> (4 * ((lane >> 4) & 3));
        uint32_t rr[2];
        if constexpr (MASK) {  // each query half its own rows (per-lane bits)
#pragma unroll
            for (int n = 0; n < 2; n++) {
                const uint32_t vq_ = ((n ? mw.y : mw.x) & vw) >> (4 * ((lane >> 4) & 3));
                int mi = Q8_NONE;
#pragma unroll
                for (int mm = 0; mm < 2; mm++)
#pragma unroll
                    for (int r = 0; r < 4; r++) mi = max(mi, ((vq_ >> (16 * mm + r)) & 1u) ? ac[mm][n][r] : Q8_NONE);
                rr[n] = (uint32_t)mi;
            }
        } else if constexpr (ISL2) {
            float p0, p1;
            reduce(ac, vw_, sb_, xa_, xb_, p0, p1);
            rr[0] = __float_as_uint(p0);
            rr[1] = __float_as_uint(p1);
        } else if (vw == 0xFFFFFFFFu) {
#pragma unroll
            for (int n = 0; n < 2; n++)
                rr[n] = (uint32_t)max(max(max(ac[0][n][0], ac[0][n][1]), max(ac[0][n][2], ac[0][n][3])),
                                      max(max(ac[1][n][0], ac[1][n][1]), max(ac[1][n][2], ac[1][n][3])));
        } else {
#pragma unroll
            for (int n = 0; n < 2; n++) {
                int mi = Q8_NONE;
#pragma unroll
                for (int mm = 0; mm < 2; mm++)
#pragma unroll
                    for (int r = 0; r < 4; r++) mi = max(mi, ((vl >> (16 * mm + r)) & 1u) ? ac[mm][n][r] : Q8_NONE);
                rr[n] = (uint32_t)mi;
            }
        }
        r0 = rr[0];
        r1 = rr[1];
    };
    // PAIR: the pending slot's raw partials ("no valid row" until a block is
    // reduced: a LIVE wave without queries stores +inf keys)
    constexpr uint32_t PNONE = ISL2 ? 0x7f800000u : (uint32_t)Q8_NONE;
    uint32_t pA0 = PNONE, pA1 = PNONE, pB0 = PNONE, pB1 = PNONE;
    float psA = 0.f, psB = 0.f;                    // and its block scales
    i32x4_t acc[RB][2][2];
    // STAG, waves 4-7: the previous slot's last block is reduced late, from its
    // accumulators (kept: acc[1] is rewritten only from chunk NC on) and these
    const bool late = STAG && wave >= 4;
    uint32_t dvw = 0;
    float dsb = 0.f;
    f32x4_t dxa = {0.f, 0.f, 0.f, 0.f}, dxb = {0.f, 0.f, 0.f, 0.f};
    // static priority for the younger half of the SIMD pairs (MI355X_MICROARCH.md,
    // two waves per SIMD, item 4): one s_setprio before the loop, none inside
    if (a.prio && wave >= 4) __builtin_amdgcn_s_setprio(1);
    // the slot loop; LIVE: a second copy for a wave without queries (ACT false:
    // no fragment reads, MFMAs or reductions; the same DMA, key stores and
    // barriers), so neither copy branches around its MFMAs
    auto slot_loop = [&](auto actc) {
    constexpr bool ACT = decltype(actc)::value;
    int cur = 0;
    for (int t = 0; t < nsteps; t++) {
        const int nxt = cur == NBUF - 1 ? 0 : cur + 1;
        const int gslot = cur == 0 ? NBUF - 1 : cur - 1;  // slot of group t+2
        const unsigned sbase = ring + (unsigned)(cur * SLOT) + l16;
        const int dma = __builtin_amdgcn_readfirstlane(t + 2 < nsteps ? 1 : 0);  // uniform: a scalar branch
        const unsigned sm = (unsigned)(t & 3);
        uint2 vwv;
        float2 sbv;
        uint2 mw0 = uint2{0u, 0u}, mw1 = uint2{0u, 0u};  // MASK: this lane's two queries' words of blocks 0, 1
        f32x4_t xa[RB], xb[RB];
        if constexpr (!ISL2) {
#pragma unroll
            for (int r = 0; r < RB; r++) xa[r] = xb[r] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        }
        static_for<0, NT>([&](auto ttc) {
            constexpr int tt = decltype(ttc)::value;
            constexpr int rb = tt / NC, c = tt % NC;
            if constexpr (tt == X0 && ACT) {  // this slot's valid words, scales (+ L2 norms)
                asm volatile("ds_read_b64 %0, %1" : "=v"(vwv) : "v"(vring + sm * 16u));
                asm volatile("ds_read_b64 %0, %1" : "=v"(sbv) : "v"(sring + sm * 16u));
                if constexpr (MASK) {
                    const unsigned mb = mring + sm * 256u + (unsigned)((lane & 15) * 8);
                    asm volatile("ds_read_b64 %0, %1" : "=v"(mw0) : "v"(mb));
                    asm volatile("ds_read_b64 %0, %1 offset:128" : "=v"(mw1) : "v"(mb));
                }
                if constexpr (ISL2) {
                    // rows 4g..4g+3 and 16+4g..+3 of block rb, g = lane>>4
                    const unsigned xbase = xnring + sm * (unsigned)(RB * 128) + (unsigned)(16 * ((lane >> 4) & 3));
                    xa[0] = lds_ld4f_o<0>(xbase);
                    xb[0] = lds_ld4f_o<64>(xbase);
                    if constexpr (RB == 2) {
                        xa[RB - 1] = lds_ld4f_o<128>(xbase);
                        xb[RB - 1] = lds_ld4f_o<192>(xbase);
                    }
                }
            }
            if constexpr (tt + PF < NT && ACT) {
                constexpr int o1 = ((tt + PF) / NC * NPB + 2 * ((tt + PF) % NC)) * 1024;
                B2[(tt + PF) % NB2][0] = lds_ld16_o<o1>(sbase);
                B2[(tt + PF) % NB2][1] = lds_ld16_o<o1 + 512>(sbase);
            }
            // reads younger than chunk tt's: the chunks up to tt + PF, and the
            // extras (issued at the start of step X0) while tt < X0 + PF
            constexpr int ahead = (NT - 1 - tt) < PF ? (NT - 1 - tt) : PF;
            qs_wait_lgkm<2 * ahead + ((tt >= X0 && tt < X0 + PF) ? XE : 0)>();
            asm volatile("" : "+v"(B2[tt % NB2][0]), "+v"(B2[tt % NB2][1]));
            if constexpr (tt == X0 + PF) {
                if constexpr (ISL2) {
                    asm volatile("" : "+v"(vwv), "+v"(sbv), "+v"(xa[0]), "+v"(xb[0]));
                    if constexpr (RB == 2) asm volatile("" : "+v"(xa[RB - 1]), "+v"(xb[RB - 1]));
                } else {
                    asm volatile("" : "+v"(vwv), "+v"(sbv));
                    if constexpr (MASK) asm volatile("" : "+v"(mw0), "+v"(mw1));
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ACT)
#pragma unroll
            for (int m = 0; m < 2; m++)
#pragma unroll
                for (int n = 0; n < 2; n++) {
                    if constexpr (DBG & 2) { acc[rb][m][n] = B2[tt % NB2][m]; continue; }
                    if constexpr (c == 0)
                        acc[rb][m][n] = __builtin_amdgcn_mfma_i32_16x16x64_i8(B2[tt % NB2][m], Qf[2 * c + n],
                                                                              i32x4_t{0, 0, 0, 0}, 0, 0, 0);
                    else
                        acc[rb][m][n] = __builtin_amdgcn_mfma_i32_16x16x64_i8(B2[tt % NB2][m], Qf[2 * c + n],
                                                                              acc[rb][m][n], 0, 0, 0);
                }
            // DMA of group t+2: one piece per chunk
            if constexpr (tt < P0) {
                if (dma) issue_piece(tt, t + 2, gslot);
            }
            // the previous slot's last block: cross-lane combine + key store
            if constexpr (tt == P0 && !(DBG & 4)) {
                if (t > 0) {
                    if constexpr (PAIR) {
                        finish2(pA0, pA1, pB0, pB1, psA, psB, gbp);
                    } else {
                        if (late) reduce(acc[RB - 1], dvw, dsb, dxa, dxb, mp0, mp1);
                        finish(mp0, mp1, gbp);
                    }
                }
            }
            // PAIR: block 0's partials beside block 1's MFMAs (stored with block 1)
            if constexpr (PAIR && tt == NC + 1 && !(DBG & 4) && ACT) reduce_raw(acc[0], vwv.x, sbv.x, xa[0], xb[0], pA0, pA1, mw0);
            // RB = 2: block 0 is reduced and stored beside block 1's MFMAs
            if constexpr (RB == 2 && !PAIR && tt == NC + 1 && !(DBG & 4)) {
                if (!late) {
                    float p0, p1;
                    reduce(acc[0], vwv.x, sbv.x, xa[0], xb[0], p0, p1);
                    finish(p0, p1, (s0 + t) * RB);
                }
            }
            if constexpr (STAG && tt == NC + P0) {
                if (late) {
                    float p0, p1;
                    reduce(acc[0], vwv.x, sbv.x, xa[0], xb[0], p0, p1);
                    finish(p0, p1, (s0 + t) * RB);
                }
            }
        });
        if (late) {
            dvw = vwv.y;
            dsb = sbv.y;
            dxa = xa[RB - 1];
            dxb = xb[RB - 1];
        } else if constexpr (PAIR && !(DBG & 4)) {
            if constexpr (ACT) {
                reduce_raw(acc[1], vwv.y, sbv.y, xa[1], xb[1], pB0, pB1, mw1);
                psA = sbv.x;
                psB = sbv.y;
            }
        } else if constexpr (!(DBG & 4)) {
            reduce(acc[RB - 1], RB == 2 ? vwv.y : vwv.x, RB == 2 ? sbv.y : sbv.x, xa[RB - 1], xb[RB - 1], mp0, mp1);
        } else {
#pragma unroll
            for (int r = 0; r < RB; r++)
                dbg_sink ^= acc[r][0][0][0] ^ acc[r][0][1][0] ^ acc[r][1][0][0] ^ acc[r][1][1][0];
        }
        gbp = (s0 + t) * RB + (PAIR ? 0 : RB - 1);
        // ---- end of the slot: the next group must have landed (every wave) ----
        if (t + 1 < nsteps) {
            // this wave's vector-memory ops after group t+1, in issue order: the
            // stores of slot t-1, the pieces of group t+2, the stores of slot t
            // (RB per slot; slot 0 has RB - 1)
            if constexpr (DBG != 0) {
                qs_wait_vm_c<0>();
            } else if (t >= 2 && t + 2 < nsteps) {
                qs_wait_vm_c<2 * SPS + P0>();
            } else {
                const int y = (t >= 1 ? stores_in(t - 1) : 0) + stores_in(t) + (t + 2 < nsteps ? P0 : 0);
                qs_wait_vm(y);
            }
            __builtin_amdgcn_s_barrier();  // slot t is free; slot t+1 has landed for every wave
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ACT) head_reads(ring + (unsigned)(nxt * SLOT) + l16);
        }
        cur = nxt;
    }
    };
    if constexpr (LIVE) {
        if (act) slot_loop(std::true_type{});
        else slot_loop(std::false_type{});
    } else {
        slot_loop(std::true_type{});
    }
    if (nsteps > 0 && !(DBG & 4)) {
        if constexpr (PAIR) {
            finish2(pA0, pA1, pB0, pB1, psA, psB, gbp);
        } else {
            if (late) reduce(acc[RB - 1], dvw, dsb, dxa, dxb, mp0, mp1);
            finish(mp0, mp1, gbp);
        }
    }
    if constexpr ((DBG & 12) != 0) {
        if (a.ldk == -1234567) krow[0] = (float)dbg_sink;  // never true: the sink stays live
    }
}

// ---------------------------------------------------------------------------
// k_q8_blockkey32<NC, RB, L2>: the same int8 block keys on
// v_mfma_i32_32x32x32_i8 (NC = dpb8 / 32 chunks of 32 columns per block, one
// MFMA per chunk and wave: 32 rows x the wave's 32 queries).  The 32x32
// accumulator holds 16 rows of ONE query per lane, so a block's reduction is
// 15 lane-local maxima and one permlane32 swap (the 16x16x64 layout spreads a
// query over four lane groups: two more swap levels and twice the selects).
// The schedule is k_qs_blockkey's multi-block one (32x32x16 bf16 for d <= 384):
// A fragments four chunks ahead, RB blocks per slot, the slot's DMA group three
// steps ahead issued after its barrier, the half-swapped 1 KiB pieces that make
// the 16-lane ds_read_b128 groups conflict-free.
// ---------------------------------------------------------------------------
template <int NC, int RB, bool ISL2>
__global__ __launch_bounds__(512, 2) void k_q8_blockkey32(Q8Args a) {
    constexpr int SLOT = RB * NC * 1024;           // bytes per ring slot
    constexpr int P = RB * NC / 8;                 // 1 KiB DMA pieces per wave per slot
    static_assert((RB * NC) % 8 == 0, "pieces per slot must split over 8 waves");
    constexpr int64_t TILE_B = (int64_t)NC * 8192;  // bytes per 256-row tile of the plane
    constexpr int NBUF = 3;
    extern __shared__ __attribute__((aligned(16))) unsigned char qsm[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 31, lh = lane >> 5;
    const int total = a.nqg * a.nspans;
    const int b = blockIdx.x;
    const int logical = (total % 8 == 0) ? (b % 8) * (total / 8) + (b / 8) : b;
    const int span = logical / a.nqg, grp = logical % a.nqg;

    // B fragments: Qf[c] = lane (li, lh): query wave*32 + li, columns 32c + 16lh .. +15
    i32x4_t Qf[NC];
    {
        const unsigned char* qp = a.Q8 + (int64_t)grp * TILE_B + (wave * 32 + li) * 32 + 16 * lh;
#pragma unroll
        for (int c = 0; c < NC; c++) Qf[c] = *reinterpret_cast<const i32x4_t*>(qp + c * 8192);
    }
    const int64_t qrow = (int64_t)grp * 256 + wave * 32 + li;
    const float sq = a.qscale[qrow];
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): retire the query loads before the DMA ring

    const int64_t s0 = (int64_t)span * a.slots_per_span;
    int64_t s1 = s0 + a.slots_per_span;
    if (s1 > a.nslots) s1 = a.nslots;
    const int nsteps = s1 > s0 ? (int)(s1 - s0) : 0;

    // LDS-DMA: lane L writes bytes [16L, 16L+16) of a 1 KiB piece = row L>>1,
    // physical half L&1 holding source half (L&1) ^ ((row>>3)&1)
    const int prow = lane >> 1;
    const uint32_t src_lane = (uint32_t)(prow * 32 + 16 * ((lane & 1) ^ ((prow >> 3) & 1)));
    const unsigned ring = lds_addr(qsm);
    // per-wave rings of 4 entries: valid words [8][4][16 B], scales [8][4][16 B],
    // L2 norms [8][4][RB * 128 B]
    const unsigned vring = ring + NBUF * SLOT + (unsigned)wave * 64u;
    const unsigned sring = ring + NBUF * SLOT + 512u + (unsigned)wave * 64u;
    const unsigned xnring = ring + NBUF * SLOT + 1024u + (unsigned)wave * (unsigned)(4 * RB * 128);
    constexpr int P0 = P + 2 + (ISL2 ? 1 : 0);  // vector-memory ops per group, per wave
    const int64_t tile0 = (s0 * RB * 32) >> 8;
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.X8 + tile0 * TILE_B), (short)0, -1, 0x00020000);
    int64_t igb = s0 * RB;
    uint32_t ioff = (uint32_t)(((igb >> 3) - tile0) * TILE_B + (igb & 7) * 1024);
    auto issue = [&](int t, int slot) {
        const unsigned sbs = ring + (unsigned)(slot * SLOT);
#pragma unroll
        for (int i = 0; i < P; i++) {
            const int p = wave + 8 * i;
            const int rb = p / NC, c = p % NC;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(size_t)(sbs + (unsigned)((rb * NC + c) * 1024)), 16,
                                                     src_lane, ioff + (uint32_t)(rb * 1024 + c * 8192), 0, 0);
        }
        if (lane < RB)
            __builtin_amdgcn_global_load_lds(a.valid + igb + lane, (lds_ptr_t)(size_t)(vring + (unsigned)((t & 3) * 16)), 4, 0, 0);
        if (lane < RB)
            __builtin_amdgcn_global_load_lds(a.sb + igb + lane, (lds_ptr_t)(size_t)(sring + (unsigned)((t & 3) * 16)), 4, 0, 0);
        if (ISL2 && lane < RB * 8)
            __builtin_amdgcn_global_load_lds(a.xnorm2 + igb * 32 + 4 * lane,
                                             (lds_ptr_t)(size_t)(xnring + (unsigned)((t & 3) * RB * 128)), 16, 0, 0);
        igb += RB;
        ioff += RB * 1024;
        if ((igb & 7) == 0) ioff += (uint32_t)(TILE_B - 8192);
    };

    const unsigned lane_off = (unsigned)(li * 32 + 16 * (lh ^ ((li >> 3) & 1)));
    float* krow = a.key + qrow * a.ldk;
    i32x4_t A[4];
    if (nsteps > 0) {
        issue(0, 0);
        if (nsteps > 1) issue(1, 1);
        qs_wait_vm(nsteps > 1 ? P0 : 0);  // group 0 landed, group 1 may stay in flight
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (nsteps > 2) issue(2, 2);
        const unsigned sb0 = ring + lane_off;
        A[0] = lds_ld16_o<0>(sb0);
        A[1] = lds_ld16_o<1024>(sb0);
        A[2] = lds_ld16_o<2048>(sb0);
        A[3] = lds_ld16_o<3072>(sb0);
    }
    int cur = 0;
    for (int t = 0; t < nsteps; t++) {
        const int nxt = cur == NBUF - 1 ? 0 : cur + 1;
        const unsigned sbase = ring + (unsigned)(cur * SLOT) + lane_off;
        const unsigned sbn = ring + (unsigned)(nxt * SLOT) + lane_off;
        const unsigned sm = (unsigned)(t & 3);
        static_for<0, RB>([&](auto rbc) {
            constexpr int rb = decltype(rbc)::value;
            // ---- the block's 32 rows x this wave's 32 queries: NC MFMAs, A fragments 4 ahead ----
            i32x16_t acc;
            static_for<0, NC>([&](auto cc) {
                constexpr int c = decltype(cc)::value;
                qs_wait_lgkm<(NC - 1 - c) < 3 ? (NC - 1 - c) : 3>();
                asm volatile("" : "+v"(A[c & 3]));
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (c == 0)
                    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[c & 3], Qf[c], i32x16_t{}, 0, 0, 0);
                else
                    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[c & 3], Qf[c], acc, 0, 0, 0);
                if constexpr (c + 4 < NC) A[c & 3] = lds_ld16_o<(rb * NC + c + 4) * 1024>(sbase);
            });
            // ---- end of the slot: the next group must have landed (every wave) ----
            if constexpr (rb == RB - 1) {
                if (t + 1 < nsteps) {
                    if (t >= 2 && t + 2 < nsteps) {
                        qs_wait_vm_c<2 * RB + P0>();  // steady state
                    } else {
                        const int y = (RB - 1) + (t >= 1 ? RB : 0) + (t >= 2 ? 1 : 0) + (t + 2 < nsteps ? P0 : 0);
                        qs_wait_vm(y);
                    }
                    __builtin_amdgcn_s_barrier();  // slot t is free: every wave's chain over it is done
                    __builtin_amdgcn_sched_barrier(0);
                    if (t + 3 < nsteps) issue(t + 3, cur);
                }
            }
            // ---- epilogue: the block's key for this lane's query ----
            const int64_t gb = (s0 + t) * RB + rb;
            uint32_t vwv;
            float sbv;
            asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(vwv) : "v"(vring + sm * 16u), "i"(rb * 4));
            asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(sbv) : "v"(sring + sm * 16u), "i"(rb * 4));
            // next block's first fragments (in flight during the epilogue)
            const unsigned pb = rb + 1 < RB ? sbase : sbn;
            constexpr int pr = rb + 1 < RB ? rb + 1 : 0;
            float m;
            if constexpr (ISL2) {
                const unsigned xb = xnring + sm * (unsigned)(RB * 128) + (unsigned)(rb * 128 + 16 * lh);
                f32x4_t x0 = lds_ld4f_o<0>(xb), x1 = lds_ld4f_o<32>(xb), x2 = lds_ld4f_o<64>(xb), x3 = lds_ld4f_o<96>(xb);
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vwv), "+v"(sbv), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
                A[0] = lds_ld16_o<(pr * NC + 0) * 1024>(pb);
                A[1] = lds_ld16_o<(pr * NC + 1) * 1024>(pb);
                A[2] = lds_ld16_o<(pr * NC + 2) * 1024>(pb);
                A[3] = lds_ld16_o<(pr * NC + 3) * 1024>(pb);
                const uint32_t vw = __builtin_amdgcn_readfirstlane(vwv);
                const float c2 = -2.f * (sq * __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(sbv))));
                const uint32_t vl = vw >> (4 * lh);
                const float xn[16] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3],
                                      x2[0], x2[1], x2[2], x2[3], x3[0], x3[1], x3[2], x3[3]};
                m = __builtin_inff();
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    float v = fmaf(c2, (float)acc[r], xn[r]);
                    if (vw != 0xFFFFFFFFu) v = ((vl >> ((r & 3) + 8 * (r >> 2))) & 1u) ? v : __builtin_inff();
                    m = fminf(m, v);
                }
                const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
                m = fminf(m, __uint_as_float(sw[1]));
            } else {
                A[0] = lds_ld16_o<(pr * NC + 0) * 1024>(pb);
                A[1] = lds_ld16_o<(pr * NC + 1) * 1024>(pb);
                A[2] = lds_ld16_o<(pr * NC + 2) * 1024>(pb);
                A[3] = lds_ld16_o<(pr * NC + 3) * 1024>(pb);
                asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(vwv), "+v"(sbv));
                const uint32_t vw = __builtin_amdgcn_readfirstlane(vwv);
                const float s = sq * __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(sbv)));
                const uint32_t vl = vw >> (4 * lh);
                int mi;
                if (vw == 0xFFFFFFFFu) {
                    mi = acc[0];
#pragma unroll
                    for (int r = 1; r < 16; r++) mi = max(mi, acc[r]);
                } else {
                    mi = Q8_NONE;
#pragma unroll
                    for (int r = 0; r < 16; r++)
                        mi = max(mi, ((vl >> ((r & 3) + 8 * (r >> 2))) & 1u) ? acc[r] : Q8_NONE);
                }
                // one query per lane: the halves' maxima combine across lh before the scale
                const auto sw = __builtin_amdgcn_permlane32_swap((uint32_t)mi, (uint32_t)mi, false, false);
                mi = max(mi, (int)sw[1]);
                m = mi == Q8_NONE ? __builtin_inff() : -(s * (float)mi);
            }
            if (lh == 0) krow[gb] = m;
        });
        cur = nxt;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the last (unused) prefetch
}

// ---------------------------------------------------------------------------
// k_q8_blockkey_cp<NCS, L2>: int8 block keys above 1536 dims (dpb8 = 2 NCS
// 64-column chunks: 2048 / 2560 / 3072).  A wave's 32-query fragments would
// need 4 NCS i32x4 (> 256 VGPRs), so a wave holds 16 queries (2 NCS i32x4, up
// to 192 VGPRs; 128 queries per workgroup of 8 waves, two per SIMD) and a
// 32-row block streams through the LDS ring in two column parts of NCS chunks
// (3 slots of 2 NCS KiB, the next-but-one part's LDS-DMA group issued one
// piece per chunk).  Per chunk: 2 A-fragment reads (row halves) and 2
// v_mfma_i32_16x16x64_i8 (row halves x the wave's 16 queries); the block's
// accumulators carry from part 0 into part 1, whose end reduces the block (the
// valid word, scale and L2 norms ride with every part's DMA group, read in
// part 1).  The cross-lane combine and key store of a block are deferred into
// the next block's part 0.  Keys are k_q8_blockkey's, so select / exact /
// replay apply unchanged.
// NP > 2 column parts (3072 < d <= 6144: NP x 16 chunks): the fragments of
// 16 queries take up to 384 registers, so NW = 4 waves (one per SIMD, 64
// queries per workgroup) own the unified VGPR/AGPR file; the block's
// accumulators carry through all NP parts, the last one reduces the block and
// carries the valid word, scale and norms; the key store of a block rides in
// the next block's part 0 as before.
// ---------------------------------------------------------------------------
template <int NCS, bool ISL2, int NP = 2, int NW = 8>
__global__ __launch_bounds__(64 * NW, NW == 8 ? 2 : 1) void k_q8_blockkey_cp(Q8Args a) {
    constexpr int NC = NP * NCS;                    // 64-column chunks per block
    constexpr int NPB = 2 * NC;                     // 1 KiB pieces per block
    constexpr int SPC = 2 * NCS;                    // pieces per step (one column part)
    constexpr int SLOT = SPC * 1024;
    constexpr int P = SPC / NW;                     // pieces per wave per step
    static_assert(SPC % NW == 0, "a part's pieces split over the waves");
    constexpr int64_t TILE_B = (int64_t)NPB * 8192;  // bytes per 256-row tile of a plane
    constexpr int P0 = P + 2 + (ISL2 ? 1 : 0);      // vector-memory ops per group, per wave
    static_assert(P0 < NCS, "the deferred key store follows the step's DMA pieces");
    constexpr int X0 = 1;                           // chunk of part 1's extra LDS reads
    constexpr int XE = 2 + (ISL2 ? 2 : 0);
    constexpr int NBUF = 3;
    extern __shared__ __attribute__((aligned(16))) unsigned char qsm[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int total = a.nqg * a.nspans;
    const int b = blockIdx.x;
    const int logical = (total % 8 == 0) ? (b % 8) * (total / 8) + (b / 8) : b;  // a span's groups share an XCD
    const int span = logical / a.nqg, grp = logical % a.nqg;

    // the wave's 16 queries (group grp of 16 NW rows of the 256-row query tiles)
    i32x4_t Qf[NC];
    const int64_t q0 = (int64_t)grp * (16 * NW) + wave * 16;
    {
        const int j = lane & 15, kq = lane >> 4;
        const int64_t qr = q0 + j;
        const unsigned char* qp = a.Q8 + (qr >> 8) * TILE_B + (kq >> 1) * 8192 + (qr & 255) * 32 + 16 * (kq & 1);
#pragma unroll
        for (int c = 0; c < NC; c++) Qf[c] = *reinterpret_cast<const i32x4_t*>(qp + (2 * c) * 8192);
    }
    const float sq = a.qscale[q0 + (lane & 15)];
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the query loads retire before the DMA ring

    const int64_t s0 = (int64_t)span * a.slots_per_span;  // blocks (one per two steps)
    int64_t s1 = s0 + a.slots_per_span;
    if (s1 > a.nslots) s1 = a.nslots;
    const int nblk = s1 > s0 ? (int)(s1 - s0) : 0;
    const int nsteps = NP * nblk;

    const uint32_t src_lane = (uint32_t)(16 * lane);
    const unsigned ring = lds_addr(qsm);
    const unsigned vring = ring + NBUF * SLOT + (unsigned)wave * 64u;
    const unsigned sring = ring + NBUF * SLOT + 512u + (unsigned)wave * 64u;
    const unsigned xnring = ring + NBUF * SLOT + 1024u + (unsigned)wave * 512u;
    const int64_t tile0 = (s0 * 32) >> 8;
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.X8 + tile0 * TILE_B), (short)0, -1, 0x00020000);
    int64_t igb = s0;  // block of the next DMA group
    uint32_t ioff = (uint32_t)(((igb >> 3) - tile0) * TILE_B + (igb & 7) * 1024);
    // piece j of the group of step u (part PT), into ring slot `slot`
    auto issue_piece = [&](auto ptc, int j, int u, int slot) {
        constexpr int PT = decltype(ptc)::value;
        if (j < P) {
            const int pi = wave + NW * j;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(size_t)(ring + (unsigned)(slot * SLOT + pi * 1024)),
                                                     16, src_lane, ioff + (uint32_t)((PT * SPC + pi) * 8192), 0, 0);
        } else if (j == P) {
            if (lane < 1)
                __builtin_amdgcn_global_load_lds(a.valid + igb, (lds_ptr_t)(size_t)(vring + (unsigned)((u & 3) * 16)), 4, 0,
                                                 0);
        } else if (j == P + 1) {
            if (lane < 1)
                __builtin_amdgcn_global_load_lds(a.sb + igb, (lds_ptr_t)(size_t)(sring + (unsigned)((u & 3) * 16)), 4, 0, 0);
        } else {
            if (lane < 8)
                __builtin_amdgcn_global_load_lds(a.xnorm2 + igb * 32 + 4 * lane,
                                                 (lds_ptr_t)(size_t)(xnring + (unsigned)((u & 3) * 128)), 16, 0, 0);
        }
        if (PT == NP - 1 && j == P0 - 1) {  // the block's last part issued: on to the next block
            igb += 1;
            ioff += 1024;
            if ((igb & 7) == 0) ioff += (uint32_t)(TILE_B - 8192);
        }
    };
    // lane (i = lane&15, kq = lane>>4) reads row 16m + i, columns 64c + 16kq..+15
    const unsigned l16 = (unsigned)(((lane >> 5) & 1) * 1024 + (lane & 15) * 32 + 16 * ((lane >> 4) & 1));
    i32x4_t B2[2][2];  // A fragments [chunk & 1][row half m]
    i32x4_t acc[2];    // [row half m]: element r is row 16m + 4g + r (g = lane >> 4) of query lane & 15
    if (nsteps > 0) {
        static_for<0, P0>([&](auto jc) { issue_piece(std::integral_constant<int, 0>{}, decltype(jc)::value, 0, 0); });
        static_for<0, P0>([&](auto jc) { issue_piece(std::integral_constant<int, 1 % NP>{}, decltype(jc)::value, 1, 1); });
        qs_wait_vm_c<P0>();  // group 0 landed, group 1 may stay in flight
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        B2[0][0] = lds_ld16_o<0>(ring + l16);
        B2[0][1] = lds_ld16_o<512>(ring + l16);
    }
    // the pending block: the lane's partial (raw int max, or L2 float bits) and its scale
    uint32_t pend = 0;
    float psb = 0.f;
    auto op = [](uint32_t x, uint32_t y) -> uint32_t {
        if constexpr (ISL2) return __float_as_uint(fminf(__uint_as_float(x), __uint_as_float(y)));
        else return (uint32_t)max((int)x, (int)y);
    };
    auto finish = [&](uint32_t r, float sbp, int64_t gb) {
        const auto x32 = __builtin_amdgcn_permlane32_swap(r, r, false, false);
        r = op(r, x32[1]);
        const auto x16 = __builtin_amdgcn_permlane16_swap(r, r, false, false);
        r = op(r, x16[1]);  // lanes 0-15: the block's key partial over all 32 rows, query lane
        float key;
        if constexpr (ISL2) {
            key = __uint_as_float(r);
        } else {
            const int mi = (int)r;
            key = mi == Q8_NONE ? __builtin_inff() : -((sq * sbp) * (float)mi);
        }
        if (lane < 16) a.key[(q0 + lane) * a.ldk + gb] = key;
    };
    int cur = 0;
    for (int t = 0; t < nblk; t++) {
        static_for<0, NP>([&](auto pc) {
            constexpr int PT = decltype(pc)::value;
            constexpr int PG = (PT + 2) % NP;  // the part of group u + 2
            const int u = NP * t + PT;
            const int nxt = cur == NBUF - 1 ? 0 : cur + 1;
            const int gslot = cur == 0 ? NBUF - 1 : cur - 1;  // slot of group u+2
            const unsigned sbase = ring + (unsigned)(cur * SLOT) + l16;
            const int dma = __builtin_amdgcn_readfirstlane(u + 2 < nsteps ? 1 : 0);
            const unsigned sm = (unsigned)(u & 3);
            uint32_t vw = 0;
            float sbv = 0.f;
            f32x4_t xa = {0.f, 0.f, 0.f, 0.f}, xb = {0.f, 0.f, 0.f, 0.f};
            static_for<0, NCS>([&](auto ttc) {
                constexpr int tt = decltype(ttc)::value;
                if constexpr (PT == NP - 1 && tt == X0) {  // the block's valid word, scale (+ L2 norms)
                    asm volatile("ds_read_b32 %0, %1" : "=v"(vw) : "v"(vring + sm * 16u));
                    asm volatile("ds_read_b32 %0, %1" : "=v"(sbv) : "v"(sring + sm * 16u));
                    if constexpr (ISL2) {
                        const unsigned xbase = xnring + sm * 128u + (unsigned)(16 * ((lane >> 4) & 3));
                        xa = lds_ld4f_o<0>(xbase);
                        xb = lds_ld4f_o<64>(xbase);
                    }
                }
                if constexpr (tt + 1 < NCS) {
                    constexpr int o1 = 2 * (tt + 1) * 1024;
                    B2[(tt + 1) & 1][0] = lds_ld16_o<o1>(sbase);
                    B2[(tt + 1) & 1][1] = lds_ld16_o<o1 + 512>(sbase);
                }
                constexpr int ahead = tt + 1 < NCS ? 1 : 0;
                qs_wait_lgkm<2 * ahead + ((PT == NP - 1 && tt == X0) ? XE : 0)>();
                asm volatile("" : "+v"(B2[tt & 1][0]), "+v"(B2[tt & 1][1]));
                if constexpr (PT == NP - 1 && tt == X0 + 1) {  // the extras are older than chunk tt's reads
                    if constexpr (ISL2) asm volatile("" : "+v"(vw), "+v"(sbv), "+v"(xa), "+v"(xb));
                    else asm volatile("" : "+v"(vw), "+v"(sbv));
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int m = 0; m < 2; m++) {
                    if constexpr (PT == 0 && tt == 0)
                        acc[m] = __builtin_amdgcn_mfma_i32_16x16x64_i8(B2[0][m], Qf[0], i32x4_t{0, 0, 0, 0}, 0, 0, 0);
                    else
                        acc[m] = __builtin_amdgcn_mfma_i32_16x16x64_i8(B2[tt & 1][m], Qf[PT * NCS + tt], acc[m], 0, 0, 0);
                }
                if constexpr (tt < P0) {
                    if (dma) issue_piece(std::integral_constant<int, PG>{}, tt, u + 2, gslot);
                }
                if constexpr (PT == 0 && tt == P0) {
                    if (t > 0) finish(pend, psb, s0 + t - 1);
                }
            });
            if constexpr (PT == NP - 1) {  // the block's reduction over its 32 rows
                const uint32_t w = __builtin_amdgcn_readfirstlane(vw);
                const float sbf = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(sbv)));
                const uint32_t vl = w >> (4 * ((lane >> 4) & 3));
                if constexpr (ISL2) {
                    const float cn = -2.f * (sq * sbf);
                    float m = __builtin_inff();
#pragma unroll
                    for (int mm = 0; mm < 2; mm++)
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            const float v = fmaf(cn, (float)acc[mm][r], mm ? xb[r] : xa[r]);
                            m = fminf(m, ((vl >> (16 * mm + r)) & 1u) ? v : __builtin_inff());
                        }
                    pend = __float_as_uint(m);
                } else if (w == 0xFFFFFFFFu) {
                    pend = (uint32_t)max(max(max(acc[0][0], acc[0][1]), max(acc[0][2], acc[0][3])),
                                         max(max(acc[1][0], acc[1][1]), max(acc[1][2], acc[1][3])));
                } else {
                    int mi = Q8_NONE;
#pragma unroll
                    for (int mm = 0; mm < 2; mm++)
#pragma unroll
                        for (int r = 0; r < 4; r++) mi = max(mi, ((vl >> (16 * mm + r)) & 1u) ? acc[mm][r] : Q8_NONE);
                    pend = (uint32_t)mi;
                }
                psb = sbf;
            }
            // ---- end of the step: the next group must have landed (every wave) ----
            if (u + 1 < nsteps) {
                // this wave's vector-memory ops after group u+1, in issue order: the
                // store of step u-1 or u (one per block, in part 0, from block 1 on:
                // after group u+1 when step u or u-1 is a part 0), the pieces of
                // group u+2
                qs_wait_vm((t > 0 && (PT == 0 || PT == 1) ? 1 : 0) + (dma ? P0 : 0));
                __builtin_amdgcn_s_barrier();  // slot cur is free; slot nxt has landed for every wave
                __builtin_amdgcn_sched_barrier(0);
                B2[0][0] = lds_ld16_o<0>(ring + (unsigned)(nxt * SLOT) + l16);
                B2[0][1] = lds_ld16_o<512>(ring + (unsigned)(nxt * SLOT) + l16);
            }
            cur = nxt;
        });
    }
    if (nblk > 0) finish(pend, psb, s0 + nblk - 1);
}

// BQ codes unpacked to +-1 int8 for k_q8_blockkey<..., BQ>: bit b of word w
// (column 64 w + b) -> -1 if set, +1 if not; columns >= 64 * words -> 0.
// Corpus rows (listed slots or [0, n)) from the word-major store codes[w * ccap
// + slot]; thread per (row, 4 columns).
__global__ void k_bq_unpack8(const uint64_t* __restrict__ codes, int64_t ccap, int words, int64_t n,
                             const uint32_t* __restrict__ slots, int dpb8, unsigned char* __restrict__ X8) {
    const int nw4 = dpb8 >> 2;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * nw4) return;
    const int64_t r = i / nw4;
    const int c4 = (int)(i % nw4) * 4;
    const int64_t slot = slots ? (int64_t)slots[r] : r;
    uint32_t word = 0;
    if (c4 < 64 * words) {
        const uint64_t bits = codes[(int64_t)(c4 >> 6) * ccap + slot] >> (c4 & 63);
#pragma unroll
        for (int e = 0; e < 4; e++) word |= (((bits >> e) & 1ull) ? 0xFFu : 0x01u) << (8 * e);
    }
    *reinterpret_cast<uint32_t*>(X8 + q8_plane_byte(slot, c4, dpb8)) = word;
}

// ---------------------------------------------------------------------------
// k_q8_gemv<NC, QG, L2>: the block keys of a small batch (16 QG <= 32
// queries) by streaming the int8 plane once through registers.  The 256-query
// kernel pads a small batch to a full query group and keeps one workgroup per
// CU (its LDS ring), which leaves the plane stream latency-bound (C3, B = 1:
// 3.4 ms for 7.7 GB).  Here every wave owns whole 32-row blocks: per row half
// m the A fragments come straight from the tiled plane (lane (i, kq): row
// 16m + i, columns 64c + 16kq.., 16 contiguous bytes; 1 KiB per wave per
// chunk), the queries' B fragments stay in VGPRs, no LDS, many waves per SIMD
// in flight.  Products, scales and the key formula are k_q8_blockkey's (the
// same v_mfma_i32_16x16x64_i8 integer sums, fl(sq sb), one fma for L2), so the
// keys are bit-identical.
// ---------------------------------------------------------------------------
template <int NC, int QG, bool ISL2>
__global__ __launch_bounds__(256) void k_q8_gemv(Q8Args a, int64_t nb) {
    const int lane = threadIdx.x & 63;
    const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int j = lane & 15, kq = lane >> 4;
    const int64_t lofs = (int64_t)(kq >> 1) * 8192 + 16 * (kq & 1);
    i32x4_t Qf[QG][NC];
#pragma unroll
    for (int g = 0; g < QG; g++)
#pragma unroll
        for (int c = 0; c < NC; c++)
            Qf[g][c] = *reinterpret_cast<const i32x4_t*>(a.Q8 + (int64_t)(2 * c) * 8192 + lofs + (16 * g + j) * 32);
    float sq[QG];
#pragma unroll
    for (int g = 0; g < QG; g++) sq[g] = a.qscale[16 * g + j];
    constexpr int64_t TILE_B = (int64_t)NC * 2 * 8192;
    for (int64_t b = wave0; b < nb; b += nwaves) {
        const int64_t r0 = b * 32;
        const unsigned char* base = a.X8 + (r0 >> 8) * TILE_B + (r0 & 255) * 32 + lofs;
        i32x4_t acc[2][QG];
#pragma unroll
        for (int m = 0; m < 2; m++) {
            i32x4_t A[NC];
#pragma unroll
            for (int c = 0; c < NC; c++)
                A[c] = *reinterpret_cast<const i32x4_t*>(base + (int64_t)(2 * c) * 8192 + (16 * m + j) * 32);
#pragma unroll
            for (int g = 0; g < QG; g++) {
                acc[m][g] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], Qf[g][0], i32x4_t{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
                for (int c = 1; c < NC; c++) acc[m][g] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[c], Qf[g][c], acc[m][g], 0, 0, 0);
            }
        }
        // acc[m][g][r]: row 16m + 4 (lane >> 4) + r of query 16g + (lane & 15)
        const uint32_t vw = a.valid[b];
        const float sb = a.sb[b];
        const int rg = 4 * (lane >> 4);
        f32x4_t xn[2];
        if constexpr (ISL2) {
            xn[0] = *reinterpret_cast<const f32x4_t*>(a.xnorm2 + r0 + rg);
            xn[1] = *reinterpret_cast<const f32x4_t*>(a.xnorm2 + r0 + 16 + rg);
        }
#pragma unroll
        for (int g = 0; g < QG; g++) {
            const float s = sq[g] * sb;
            float key;
            if constexpr (ISL2) {
                const float cn = -2.f * s;
                float mn = __builtin_inff();
#pragma unroll
                for (int m = 0; m < 2; m++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const float v = fmaf(cn, (float)acc[m][g][r], xn[m][r]);
                        mn = fminf(mn, ((vw >> (16 * m + rg + r)) & 1u) ? v : __builtin_inff());
                    }
                mn = fminf(mn, __shfl_xor(mn, 16));
                mn = fminf(mn, __shfl_xor(mn, 32));
                key = mn;
            } else {
                int mi = Q8_NONE;
#pragma unroll
                for (int m = 0; m < 2; m++)
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        mi = max(mi, ((vw >> (16 * m + rg + r)) & 1u) ? acc[m][g][r] : Q8_NONE);
                mi = max(mi, __shfl_xor(mi, 16));
                mi = max(mi, __shfl_xor(mi, 32));
                key = mi == Q8_NONE ? __builtin_inff() : -(s * (float)mi);
            }
            if (lane < 16) a.key[(int64_t)(16 * g + lane) * a.ldk + b] = key;
        }
    }
}

}  // namespace
}  // namespace wv
