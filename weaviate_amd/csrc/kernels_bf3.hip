// kernels_bf3.hip -- the approximate-distance select kernel on bf16 MFMA with
// a three-term split ("bf16x3"): every fp32 value v is stored as
// vh = bf16(v) and vl = bf16(v - vh), and
//     q.x  ~  qh.xh + qh.xl + ql.xh       (three v_mfma_f32_32x32x16_bf16)
// whose error against the exact dot product is bounded by
//     (3.05 * 2^-16 + gamma'_{3d+16}) * sum|q_i||x_i|,
// so k_finalize's exactness proof carries over with a wider eps.  Per 32x32
// block and 16 k this is 3 x 32 MFMA cycles instead of 8 x 64 for the f32-in
// MFMA (5.3x less matrix-core time).
//
// Structure = k_mfma_select3 (8 waves, 128-query x 256-row tiles, 3-deep LDS
// ring filled by global_load_lds_dwordx4, one barrier per BK=32 slice, the
// same fused top-KP selection epilogue).  A ring slot holds, per plane, the
// BK=32 slice of every row as 64 B = four 16-B chunks (8 bf16 each); chunk c
// of row r sits at physical chunk c ^ ((r >> 2) & 3), which makes the
// 16-lane ds_read_b128 groups (16 consecutive rows) conflict-free.
#pragma once

namespace wv {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int SLOT_BF3 = (BN3 + QB) * BK * 2 * 2;  // bytes per ring slot: 2 planes x bf16 = 48 KiB

__device__ __forceinline__ int swz_bf3(int r) { return (r >> 2) & 3; }

// element index of (row, col) in a tiled bf16 plane (see k_split_bf16)
__host__ __device__ __forceinline__ int64_t bf3_plane_index(int64_t row, int col, int dpad) {
    return (((row >> 8) * (dpad >> 4) + (col >> 4)) << 12) + ((row & 255) << 4) + (col & 15);
}

__device__ __forceinline__ bf16x8_t lds_ld8bf(const unsigned char* p) {
    bf16x8_t v;
    const unsigned off = (unsigned)(size_t)((__attribute__((address_space(3))) const unsigned char*)p);
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(off));
    return v;
}

// Epilogue LDS traffic in inline asm: the LDS-DMA ring (global_load_lds)
// counts as pending LDS writes for the compiler, which then puts vmcnt(0) --
// a full drain of the ring -- before every LDS atomic/store and on every
// __syncthreads fence.  The candidate buffer, counters and flags are never a
// DMA target, so LDS ordering (lgkmcnt) is all these accesses need.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)((__attribute__((address_space(3))) const void*)p);
}
__device__ __forceinline__ int lds_add_rtn(int* p, int v) {
    int r;
    asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(lds_addr(p)), "v"(v) : "memory");
    return r;
}
__device__ __forceinline__ void lds_st(void* p, uint32_t v) {
    asm volatile("ds_write_b32 %0, %1" : : "v"(lds_addr(p)), "v"(v) : "memory");
}
// workgroup barrier ordering LDS only (no vmcnt drain of the DMA ring)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

// wave-uniform 8-byte read through the scalar cache (address 8-B aligned)
__device__ __forceinline__ uint64_t sload_u64(const void* p) {
    // p is wave-uniform but derived from threadIdx: move it to SGPRs
    const uint64_t pi = (uint64_t)p;
    const uint64_t up = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(pi >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)pi);
    uint64_t v;
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(up) : "memory");
    return v;
}

// ds_read_b128 at LDS byte address base + OFF (immediate offset field)
template <int OFF>
__device__ __forceinline__ bf16x8_t lds_ld8bf_o(unsigned base) {
    bf16x8_t v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(OFF));
    return v;
}

template <int METRIC, int R>
__global__ __launch_bounds__(512, 2) void k_mfma_select_bf3(SelectArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int KP = a.KP;
    const int C = a.C;
    unsigned char* ring = reinterpret_cast<unsigned char*>(smem);  // [NBUF3][SLOT_BF3]
    float* thr = reinterpret_cast<float*>(ring + NBUF3 * SLOT_BF3);  // QB
    int* cnt = reinterpret_cast<int*>(thr + QB);                     // QB
    int* flags = cnt + QB;                                           // 4
    float* cbA = reinterpret_cast<float*>(flags + 4);                // QB*C
    uint32_t* cbI = reinterpret_cast<uint32_t*>(cbA + QB * C);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;  // 0..7
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

    // 32-bit loop state (tile < 2^24, steps < 2^31): fewer SGPRs, no spills
    const int t0 = span * a.tiles_per_span;
    int t1 = t0 + a.tiles_per_span;
    if ((int64_t)t1 > a.ntiles) t1 = (int)a.ntiles;
    const int nk = a.dpad / BK;
    const int total_steps = t1 > t0 ? (t1 - t0) * nk : 0;

    // DMA pieces (1 KiB = 16 rows x 64 B) of this wave per slice: 2 of Xh, 2 of
    // Xl (rows 32w .. 32w+31), 1 of Qh, 1 of Ql (rows 16w .. 16w+15).  Lane L
    // writes LDS row L>>2, physical chunk L&3 = logical chunk (L&3) ^ swz(row).
    // Per-lane source offsets are fixed; a slice adds kb*64 B, a tile BN3 rows.
    const int prow = lane >> 2, pchunk = lane & 3;
    // tiled planes (bf3_plane_index): a 256-row tile is dpad/16 blocks of 8 KiB;
    // logical 16-B chunk lc of a BK=32 slice is k group 2*kb + (lc >> 1), half lc & 1
    const int64_t tile_b = (int64_t)(a.dpad >> 4) * 8192;  // bytes per 256-row tile of a plane
    int xoff[2];
#pragma unroll
    for (int p = 0; p < 2; p++) {
        const int row = 32 * wave + 16 * p + prow;
        const int lc = pchunk ^ swz_bf3(row);
        xoff[p] = (lc >> 1) * 8192 + row * 32 + 16 * (lc & 1);
    }
    const int qrow = (q0 & 255) + 16 * wave + prow;  // q0 is a multiple of 128
    const int qlc = pchunk ^ swz_bf3(16 * wave + prow);
    const int64_t qoff = (int64_t)(q0 >> 8) * tile_b + (qlc >> 1) * 8192 + qrow * 32 + 16 * (qlc & 1);
    const unsigned char* Xh8 = reinterpret_cast<const unsigned char*>(a.Xh);
    const unsigned char* Xl8 = reinterpret_cast<const unsigned char*>(a.Xl);
    const unsigned char* Qh8 = reinterpret_cast<const unsigned char*>(a.Qh);
    const unsigned char* Ql8 = reinterpret_cast<const unsigned char*>(a.Ql);
    // issue position (tile, kb, slot) runs two slices ahead of the compute position
    int itile = t0;
    int ikb = 0, islot = 0;
    auto issue = [&]() {
        unsigned char* slot = ring + islot * SLOT_BF3;
        const int64_t tb = (int64_t)itile * tile_b + ikb * 16384;
#pragma unroll
        for (int p = 0; p < 2; p++) {
            __builtin_amdgcn_global_load_lds(Xh8 + tb + xoff[p], (lds_ptr_t)(slot + (32 * wave + 16 * p) * 64), 16, 0, 0);
            __builtin_amdgcn_global_load_lds(Xl8 + tb + xoff[p], (lds_ptr_t)(slot + BN3 * 64 + (32 * wave + 16 * p) * 64),
                                             16, 0, 0);
        }
        __builtin_amdgcn_global_load_lds(Qh8 + ikb * 16384 + qoff, (lds_ptr_t)(slot + 2 * BN3 * 64 + (16 * wave) * 64),
                                         16, 0, 0);
        __builtin_amdgcn_global_load_lds(Ql8 + ikb * 16384 + qoff,
                                         (lds_ptr_t)(slot + 2 * BN3 * 64 + QB * 64 + (16 * wave) * 64), 16, 0, 0);
        if (++ikb == nk) { ikb = 0; itile++; }
        if (++islot == NBUF3) islot = 0;
    };

    f32x16 acc[2][2];
    int epoch = 0;
    if (total_steps > 0) issue();
    if (total_steps > 1) issue();

    int tile = t0;
    int kb = 0, cslot = 0;
    for (int step = 0; step < total_steps; step++) {
        if (step + 1 < total_steps) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // everyone's pieces landed; slot (step+2)%3 is free
        __builtin_amdgcn_sched_barrier(0);
        if (step + 2 < total_steps) issue();
        const unsigned char* cur = ring + cslot * SLOT_BF3;
        if (kb == 0) {
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 2; j++)
#pragma unroll
                    for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;
        }
        // all 16 fragment reads up front (invisible to hipcc's waitcnt logic);
        // k16 step 0's MFMAs wait for its 8 reads
        bf16x8_t XH[2][2], XL[2][2], QH[2][2], QL[2][2];  // [kk][block]
#pragma unroll
        for (int kk = 0; kk < 2; kk++)
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int xr = 64 * wx + 32 * i + li;
                const int qr = 64 * wq + 32 * i + li;
                const int xc = (2 * kk + lh) ^ swz_bf3(xr);
                const int qc = (2 * kk + lh) ^ swz_bf3(qr);
                XH[kk][i] = lds_ld8bf(cur + xr * 64 + 16 * xc);
                XL[kk][i] = lds_ld8bf(cur + BN3 * 64 + xr * 64 + 16 * xc);
                QH[kk][i] = lds_ld8bf(cur + 2 * BN3 * 64 + qr * 64 + 16 * qc);
                QL[kk][i] = lds_ld8bf(cur + 2 * BN3 * 64 + QB * 64 + qr * 64 + 16 * qc);
            }
#pragma unroll
        for (int kk = 0; kk < 2; kk++) {
            if (a.dbg == 2) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); break; }
            if (kk == 0) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(XH[kk][i], QH[kk][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(XH[kk][i], QL[kk][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(XL[kk][i], QH[kk][j], acc[i][j], 0, 0, 0);
                }
        }
        const bool last_k = kb == nk - 1;
        if (++cslot == NBUF3) cslot = 0;
        if (++kb == nk) kb = 0;

        if (last_k && a.dbg) tile++;
        if (last_k && !a.dbg) {
            // ---------------- epilogue: selection over this 128 x 256 tile (as k_mfma_select3) ----------------
            const int64_t row0 = (int64_t)tile * BN3;
            float qn[2];
            int qidx[2];
#pragma unroll
            for (int j = 0; j < 2; j++) {
                qidx[j] = 64 * wq + 32 * j + li;
                qn[j] = (METRIC == L2) ? a.qnorm2[q0 + qidx[j]] : 0.f;
            }
            // rows 64wx + 32i + [0, 32) of the tile share one word of the valid bitmap
            // scalar read: a vector load here would be retired by the
            // compiler's vmcnt(0), which also drains the DMA ring
            const uint64_t vb2 = sload_u64(a.valid + (row0 >> 5) + 2 * wx);
            const uint32_t vbw[2] = {(uint32_t)vb2, (uint32_t)(vb2 >> 32)};
            // the candidate mask against the current thresholds is built
            // branch-free; a wave with no candidate skips the selection loop
            uint64_t pending = 0;
            {
                const float th0[2] = {thr[qidx[0]], thr[qidx[1]]};
#pragma unroll
                for (int i = 0; i < 2; i++) {
#pragma unroll
                    for (int r = 0; r < 16; r++) {
                        const int rr = (r & 3) + 8 * (r >> 2) + 4 * lh;  // row within the 32-row block
                        const bool ok = (vbw[i] >> rr) & 1u;
                        const float xn = (METRIC == L2) ? a.xnorm2[row0 + 64 * wx + 32 * i + rr] : 0.f;
#pragma unroll
                        for (int j = 0; j < 2; j++) {
                            const float dot = acc[i][j][r];
                            float v;
                            if (METRIC == L2) v = (xn - 2.f * dot) + qn[j];
                            else if (METRIC == DOT) v = -dot;
                            else { v = 1.f - dot; v = v < 0.f ? 0.f : v; }
                            const bool qok = (q0 + qidx[j]) < a.nq;
                            v = (ok && qok) ? v : __builtin_inff();
                            acc[i][j][r] = v;
                            const int vi = (i * 16 + r) * 2 + j;
                            pending |= (uint64_t)(v < th0[j]) << vi;
                        }
                    }
                }
            }
            // Candidates accumulate in the LDS buffer across tiles; the lists
            // (global) are merged only when a buffer overflows or at the span's
            // last tile.  Stale thresholds only admit more candidates, never
            // drop one of the KP best.
            const bool last_tile = tile == t1 - 1;
            for (;;) {
                ++epoch;
                float th[2] = {thr[qidx[0]], thr[qidx[1]]};
                if (__any(pending != 0))
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
                                int slot = lds_add_rtn(&cnt[qidx[j]], 1);
                                if (slot < C) {
                                    int rt = 64 * wx + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
                                    lds_st(&cbA[qidx[j] * C + slot], __float_as_uint(v));
                                    lds_st(&cbI[qidx[j] * C + slot], (uint32_t)(row0 + rt));
                                    pending &= ~(1ull << vi);
                                } else {
                                    lds_st(&flags[1], (uint32_t)epoch);  // overflow: merge, then retry
                                }
                            } else {
                                pending &= ~(1ull << vi);
                            }
                        }
                    }
                }
                lds_barrier();
                const bool overflow = flags[1] == epoch;
                if (!overflow && !last_tile) break;
                for (int jq = 0; jq < QB / 8; jq++) {
                    const int q = wave + 8 * jq;
                    const int c = cnt[q];
                    if (c == 0) continue;
                    const int nc = c < C ? c : C;
                    const int64_t base = ((int64_t)(q0 + q) * a.nspans + span) * KP;
                    merge_query_list<R>(a.outA + base, a.outI + base, cbA + q * C, cbI + q * C, KP, C, nc, lane,
                                        &thr[q]);
                    if (lane == 0) cnt[q] = 0;
                }
                lds_barrier();
                if (!overflow) break;
            }
            tile++;
        }
    }
}

// ---------------------------------------------------------------------------
// k_mfma_select_bf3w: the same math on 256-query x 256-row tiles (half the
// staged bytes per MFMA of the 128 x 256 form: the LDS-DMA stream is the
// bound there).  BK = 16 slices (32 B per row and plane), a 4-slot ring
// (3 slices in flight), 8 waves = 4 row quarters x 2 query halves, each wave
// 2 x 4 blocks of 32 x 32 (128 accumulator registers).  Chunk c of row r of a
// slice sits at physical chunk c ^ ((r >> 3) & 1): the 16-row ds_read_b128
// groups are conflict-free.
// ---------------------------------------------------------------------------
constexpr int QBW = 256;                      // queries per workgroup tile
constexpr int NBUFW = 4;
constexpr int SLOT_BW = (BN3 + QBW) * 32 * 2; // bytes per ring slot: 2 planes x 16 bf16 = 32 KiB
__device__ __forceinline__ int swz_bw(int r) { return (r >> 3) & 1; }

template <int METRIC, int R>
__global__ __launch_bounds__(512, 2) void k_mfma_select_bf3w(SelectArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int KP = a.KP;
    const int C = a.C;
    unsigned char* ring = reinterpret_cast<unsigned char*>(smem);    // [NBUFW][SLOT_BW]
    float* thr = reinterpret_cast<float*>(ring + NBUFW * SLOT_BW);    // QBW
    int* cnt = reinterpret_cast<int*>(thr + QBW);                     // QBW
    int* flags = cnt + QBW;                                           // 4
    float* cbA = reinterpret_cast<float*>(flags + 4);                 // QBW*C
    uint32_t* cbI = reinterpret_cast<uint32_t*>(cbA + QBW * C);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;  // 0..7
    const int wq = wave & 1, wx = wave >> 1;   // 2 query halves (128) x 4 row quarters (64)
    const int li = lane & 31, lh = lane >> 5;

    const int total = a.nqb * a.nspans;
    const int b = blockIdx.x;
    const int logical = (total % 8 == 0) ? (b % 8) * (total / 8) + (b / 8) : b;
    const int QG = a.qgroup;
    const int cell = logical / QG, qi = logical % QG;
    const int group = cell / a.nspans;
    const int span = cell % a.nspans;
    const int qb = group * QG + qi;
    const int q0 = qb * QBW;

    for (int jq = 0; jq < QBW / 8; jq++) {
        const int q = wave + 8 * jq;
        if (q0 + q >= a.nq) continue;
        const int64_t base = ((int64_t)(q0 + q) * a.nspans + span) * KP;
        for (int e = lane; e < KP; e += 64) { a.outA[base + e] = __builtin_inff(); a.outI[base + e] = NO_ID; }
    }
    if (tid < QBW) { thr[tid] = __builtin_inff(); cnt[tid] = 0; }
    if (tid == 0) { flags[0] = 0; flags[1] = 0; }

    const int t0 = span * a.tiles_per_span;
    int t1 = t0 + a.tiles_per_span;
    if ((int64_t)t1 > a.ntiles) t1 = (int)a.ntiles;
    const int nk = a.dpad / 16;
    const int total_steps = t1 > t0 ? (t1 - t0) * nk : 0;

    // DMA pieces (1 KiB = 32 rows x 32 B): Xh, Xl rows [32w, 32w+32), Qh, Ql
    // rows [32w, 32w+32).  Lane L writes LDS row L>>1, physical chunk L&1.
    const int prow = lane >> 1, pchunk = lane & 1;
    const int64_t tile_b = (int64_t)(a.dpad >> 4) * 8192;  // bytes per 256-row tile of a plane (bf3_plane_index)
    const int row = 32 * wave + prow;
    const int xoff = row * 32 + 16 * (pchunk ^ swz_bw(row));
    // the query tile's plane base is wave-uniform (q0 is a multiple of 256):
    // the only per-lane DMA state is xoff
    // Lean per-slice state (the scalar work between two slices' MFMAs is
    // exposed: both waves of a SIMD reach it together after the barrier).
    // In the tiled planes slice g of the span starts at (t0*nk + g) * 8 KiB
    // of X and at (g mod nk) * 8 KiB of the query tile.
    const unsigned char* Xh8 = reinterpret_cast<const unsigned char*>(a.Xh) + (int64_t)t0 * tile_b;
    const unsigned char* Xl8 = reinterpret_cast<const unsigned char*>(a.Xl) + (int64_t)t0 * tile_b;
    const unsigned char* Qh8 = reinterpret_cast<const unsigned char*>(a.Qh) + (int64_t)(q0 >> 8) * tile_b;
    const unsigned char* Ql8 = reinterpret_cast<const unsigned char*>(a.Ql) + (int64_t)(q0 >> 8) * tile_b;
    const unsigned ring_a = lds_addr(ring) + (unsigned)(32 * wave) * 32u;
    uint32_t xg = 0, qg = 0;  // byte offsets of the next slice to issue (X, query tile)
    int islot = 0;
    const uint32_t qwrap = (uint32_t)nk * 8192u;
    auto issue = [&]() {
        const unsigned sa = ring_a + (unsigned)islot * SLOT_BW;
        __builtin_amdgcn_global_load_lds(Xh8 + xg + xoff, (lds_ptr_t)(size_t)sa, 16, 0, 0);
        __builtin_amdgcn_global_load_lds(Xl8 + xg + xoff, (lds_ptr_t)(size_t)(sa + BN3 * 32), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(Qh8 + qg + xoff, (lds_ptr_t)(size_t)(sa + 2 * BN3 * 32), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(Ql8 + qg + xoff, (lds_ptr_t)(size_t)(sa + 2 * BN3 * 32 + QBW * 32), 16, 0, 0);
        xg += 8192u;
        qg += 8192u;
        if (qg == qwrap) qg = 0;
        islot = (islot + 1) & (NBUFW - 1);
    };

    f32x16 acc[2][4];
    int epoch = 0;
    for (int p = 0; p < NBUFW - 1; p++)
        if (p < total_steps) issue();

    int tile = t0;
    int kb = 0, cslot = 0;

    for (int step = 0; step < total_steps; step++) {
        // slices step+1, step+2 may stay in flight (4 pieces each)
        if (step + 2 < total_steps) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (step + 1 < total_steps) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // everyone's pieces landed; slot (step+3)%4 is free
        __builtin_amdgcn_sched_barrier(0);
        if (step + NBUFW - 1 < total_steps) issue();
        const unsigned char* cur = ring + cslot * SLOT_BW;
        if (kb == 0) {
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 4; j++)
#pragma unroll
                    for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;
        }
        // All 12 fragment reads of the slice are issued up front: X (4) and
        // query blocks 0-1 (4) are waited for before the first 12 MFMAs,
        // blocks 2-3 (4) land behind them.  Row r = 32*blk + li of any block
        // has swizzle (li >> 3) & 1, so every fragment address is one per-lane
        // VGPR plus an immediate offset (no address registers live across the
        // loop: spills here forced vmcnt(0) on the DMA ring).
        const unsigned lane_off = (unsigned)(li * 32 + 16 * (lh ^ ((li >> 3) & 1)));
        const unsigned cur_a = (unsigned)(size_t)((__attribute__((address_space(3))) const unsigned char*)cur);
        const unsigned xa = cur_a + 2048u * wx + lane_off;
        const unsigned qa = cur_a + 2u * BN3 * 32 + 4096u * wq + lane_off;
        bf16x8_t XH[2], XL[2], QH[4], QL[4];
        XH[0] = lds_ld8bf_o<0>(xa);
        XH[1] = lds_ld8bf_o<1024>(xa);
        XL[0] = lds_ld8bf_o<BN3 * 32>(xa);
        XL[1] = lds_ld8bf_o<BN3 * 32 + 1024>(xa);
        QH[0] = lds_ld8bf_o<0>(qa);
        QH[1] = lds_ld8bf_o<1024>(qa);
        QL[0] = lds_ld8bf_o<QBW * 32>(qa);
        QL[1] = lds_ld8bf_o<QBW * 32 + 1024>(qa);
        QH[2] = lds_ld8bf_o<2048>(qa);
        QH[3] = lds_ld8bf_o<3072>(qa);
        QL[2] = lds_ld8bf_o<QBW * 32 + 2048>(qa);
        QL[3] = lds_ld8bf_o<QBW * 32 + 3072>(qa);
#pragma unroll
        for (int jh = 0; jh < 2; jh++) {
            if (jh == 0) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if (a.dbg == 2) continue;
#pragma unroll
            for (int jj = 0; jj < 2; jj++)
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    const int j = 2 * jh + jj;
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(XH[i], QH[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(XH[i], QL[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(XL[i], QH[j], acc[i][j], 0, 0, 0);
                }
            __builtin_amdgcn_sched_barrier(0);
        }
        const bool last_k = kb == nk - 1;
        if (++cslot == NBUFW) cslot = 0;
        if (++kb == nk) kb = 0;
        if (last_k && a.dbg) tile++;
        if (last_k && !a.dbg) {
            // ---------------- epilogue: selection over this 256 x 256 tile ----------------
            const int64_t row0 = (int64_t)tile * BN3;
            float qn[4];
            int qidx[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                qidx[j] = 128 * wq + 32 * j + li;
                qn[j] = (METRIC == L2) ? a.qnorm2[q0 + qidx[j]] : 0.f;
            }
            // scalar read: a vector load here would be retired by the
            // compiler's vmcnt(0), which also drains the DMA ring
            const uint64_t vb2 = sload_u64(a.valid + (row0 >> 5) + 2 * wx);
            const uint32_t vbw[2] = {(uint32_t)vb2, (uint32_t)(vb2 >> 32)};
            // No pending bitmask (its 128 single-bit constants were hoisted
            // out of the main loop and pushed it into scratch): a value is a
            // candidate while it is below its query's threshold, and an
            // inserted value is set to +inf in its accumulator.  Thresholds
            // only decrease, so this admits exactly the values the mask did.
#pragma unroll
            for (int i = 0; i < 2; i++) {
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int rr = (r & 3) + 8 * (r >> 2) + 4 * lh;
                    const bool ok = (vbw[i] >> rr) & 1u;
                    const float xn = (METRIC == L2) ? a.xnorm2[row0 + 64 * wx + 32 * i + rr] : 0.f;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const float dot = acc[i][j][r];
                        float v;
                        if (METRIC == L2) v = (xn - 2.f * dot) + qn[j];
                        else if (METRIC == DOT) v = -dot;
                        else { v = 1.f - dot; v = v < 0.f ? 0.f : v; }
                        const bool qok = (q0 + qidx[j]) < a.nq;
                        acc[i][j][r] = (ok && qok) ? v : __builtin_inff();
                    }
                }
            }
            const bool last_tile = tile == t1 - 1;
            for (;;) {
                ++epoch;
                float th[4];
#pragma unroll
                for (int j = 0; j < 4; j++) th[j] = thr[qidx[j]];
                bool anyc = false;
#pragma unroll
                for (int i = 0; i < 2; i++)
#pragma unroll
                    for (int r = 0; r < 16; r++)
#pragma unroll
                        for (int j = 0; j < 4; j++) anyc |= acc[i][j][r] < th[j];
                if (__any(anyc))
#pragma unroll
                for (int i = 0; i < 2; i++) {
#pragma unroll
                    for (int r = 0; r < 16; r++) {
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            const float v = acc[i][j][r];
                            if (v < th[j]) {
                                const int slot = lds_add_rtn(&cnt[qidx[j]], 1);
                                if (slot < C) {
                                    const int rt = 64 * wx + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
                                    lds_st(&cbA[qidx[j] * C + slot], __float_as_uint(v));
                                    lds_st(&cbI[qidx[j] * C + slot], (uint32_t)(row0 + rt));
                                    acc[i][j][r] = __builtin_inff();
                                } else {
                                    lds_st(&flags[1], (uint32_t)epoch);
                                }
                            }
                        }
                    }
                }
                lds_barrier();
                const bool overflow = flags[1] == epoch;
                if (!overflow && !last_tile) break;
                for (int jq = 0; jq < QBW / 8; jq++) {
                    const int q = wave + 8 * jq;
                    const int c = cnt[q];
                    if (c == 0) continue;
                    const int nc = c < C ? c : C;
                    const int64_t base = ((int64_t)(q0 + q) * a.nspans + span) * KP;
                    merge_query_list<R>(a.outA + base, a.outI + base, cbA + q * C, cbI + q * C, KP, C, nc, lane,
                                        &thr[q]);
                    if (lane == 0) cnt[q] = 0;
                }
                lds_barrier();
                if (!overflow) break;
            }
            tile++;
        }
    }
}

// Plane layout (both kernels): 256-row tiles, 16-element k groups, so every
// slice a ring slot receives is one contiguous 8 KiB block per plane:
// element (row, col) at ((row / 256) * (dpad / 16) + col / 16) * 4096 +
// (row % 256) * 16 + col % 16.  (A row-major plane made the DMA re-fetch each
// 128-B line once per slice it spans: L2 could not hold 256 rows x d.)
//
// bf16 hi/lo split of fp32 rows: hi = bf16(v) (round to nearest even),
// lo = bf16(v - hi) (v - hi is exact in fp32).  Thread per element of the
// listed rows (slots) or of rows [0, n).
__global__ void k_split_bf16(const float* __restrict__ src, int64_t n, int dpad, const uint32_t* __restrict__ slots,
                             uint16_t* __restrict__ hi, uint16_t* __restrict__ lo) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * dpad) return;
    const int64_t r = i / dpad;
    const int c = (int)(i % dpad);
    const int64_t row = slots ? (int64_t)slots[r] : r;
    const float v = src[row * dpad + c];
    const __bf16 h = (__bf16)v;
    const float hf = (float)h;
    const __bf16 l = (__bf16)(v - hf);
    const int64_t o = bf3_plane_index(row, c, dpad);
    hi[o] = __builtin_bit_cast(uint16_t, h);
    lo[o] = __builtin_bit_cast(uint16_t, l);
}

}  // namespace wv
