// qs_kernels.hip -- the exact fp32 flat search on a bf16 block-key pass
// (DESIGN.md §3.1d).  Pipeline for a batch of queries (flat/index.go:423-448,
// :578-688):
//
//   k_qs_blockkey   query-stationary bf16 MFMA pass: every wave holds 32
//                   queries' bf16 fragments (all d) in VGPRs and streams the
//                   corpus' bf16 plane through an LDS ring; per (query,
//                   32-row block) it writes ONE float, the block's smallest
//                   approximate distance ("block key").  No selection state.
//   k_blk_select    wave per query: the (k+1)-th smallest block key M and
//                   every block whose key is within 2 eps of M -- the only
//                   blocks that can hold a top-(k+1) row (proof: DESIGN.md).
//   k_blk_exact     wave per query: reference-order exact distances of the
//                   candidate blocks' rows, top-(k+1) by (distance, id);
//                   strictly increasing -> the reference heap's answer,
//                   else the query is flagged.
//   k_blk_replay    flagged queries: the reference heap (priorityqueue NewMax
//                   + insertToHeap + extractHeap) replayed in id order,
//                   computing exact distances only for blocks whose key
//                   lower bound (key - eps) can still beat the heap top.
//
// Error model: A (from the bf16 hi planes, fp32 MFMA accumulation) and E (the
// reference's fp32 SingleDist) differ per pair by at most eps(q) (runtime:
// qs_eps), computed from per-row residual norms kept at Add time.
#pragma once
#include <type_traits>

namespace wv {
// the int8 plane of an index whose block keys came from it (k_blk_exact's row
// filter then bounds rows from the int8 codes); X8 == nullptr: the bf16 plane.
// External linkage: the exact pass's launcher (qs_exact.hip) takes it.
struct Q8Filter {
    const unsigned char* X8;
    const float* sb8;
    int dpb8;
    const unsigned char* Q8;   // the batch's query codes (tiled plane)
    const float* qscale;
    const float4* qinfo8;
    const uint32_t* qmax8;
    float gacc8;
};

namespace {  // internal linkage: each runtime unit compiles the kernels it launches

// compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N)
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

constexpr int QS_NBUF = 3;    // LDS ring slots
constexpr int QS_QPB = 256;   // queries per workgroup (8 waves x 32)

// 32-row blocks per ring slot: a slot is RB x NK KiB (<= 48 KiB)
__host__ __device__ constexpr int qs_rb(int nk) { return nk <= 8 ? 4 : nk <= 24 ? 2 : 1; }

struct QsArgs {
    const unsigned char* Xb;   // corpus bf16 hi plane, tiled (bf3_plane_index with dpb = NK*16)
    const float* xnorm2;       // [cap] sum of squares of the stored fp32 rows (L2)
    const uint32_t* valid;     // [cap/32] slots to scan (present & allowed)
    const unsigned char* Qb;   // query bf16 hi plane, tiled, nq_pad rows (multiple of 256)
    float* key;                // [nq_pad][ldk] block keys
    int64_t ldk;               // key row length (>= nslots * RB)
    int64_t nslots;            // ring slots (32 * RB rows each) to scan
    int slots_per_span;
    int nspans;
    int nqg;                   // query groups of 256
    int dbg;                   // reserved for timing experiments
};

__device__ __forceinline__ uint32_t sload_u32(const void* p) {
    const uint64_t pi = (uint64_t)p;
    const uint64_t up = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(pi >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)pi);
    uint32_t v;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(up) : "memory");
    return v;
}

// s_waitcnt vmcnt(y) for a run-time wave-uniform y (0..40; larger: vmcnt(0))
__device__ __forceinline__ void qs_wait_vm(int y) {
#define QS_VM(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    switch (y) {
        QS_VM(0) QS_VM(1) QS_VM(2) QS_VM(3) QS_VM(4) QS_VM(5) QS_VM(6) QS_VM(7) QS_VM(8) QS_VM(9) QS_VM(10)
        QS_VM(11) QS_VM(12) QS_VM(13) QS_VM(14) QS_VM(15) QS_VM(16) QS_VM(17) QS_VM(18) QS_VM(19) QS_VM(20)
        QS_VM(21) QS_VM(22) QS_VM(23) QS_VM(24) QS_VM(25) QS_VM(26) QS_VM(27) QS_VM(28) QS_VM(29) QS_VM(30)
        QS_VM(31) QS_VM(32) QS_VM(33) QS_VM(34) QS_VM(35) QS_VM(36) QS_VM(37) QS_VM(38) QS_VM(39) QS_VM(40)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
#undef QS_VM
}

template <int N>
__device__ __forceinline__ void qs_wait_vm_c() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int N>
__device__ __forceinline__ void qs_wait_lgkm() {
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

// LDS writes of this wave visible to its other lanes
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));  // packed fp32 (v_pk_mul_f32 / v_pk_add_f32)
template <int OFF>
__device__ __forceinline__ f32x4_t lds_ld4f_o(unsigned base) {
    f32x4_t v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(OFF));
    return v;
}

// ---------------------------------------------------------------------------
// k_qs_blockkey<NK, L2>: block keys of 256 queries x one span of the corpus.
//   key (L2)      = min over the block's valid rows of fl(xnorm2 - 2 S)   (A = fl(key + |q|^2))
//   key (dot/cos) = -max over the block's valid rows of S                 (A = key / max(0, fl(1 + key)))
// with S = sum_k bf16(q_k) bf16(x_k) (fp32 MFMA accumulation); a block with no
// valid row gets +inf.
// ---------------------------------------------------------------------------
// DBG (timing experiments only, never the product path): bit 0 drops the
// MFMAs, bit 1 the LDS-DMA pieces (every wait then vmcnt(0)), bit 2 the
// A-fragment LDS reads of the one-block schedule
template <int NK, bool ISL2, int DBG = 0>
__global__ __launch_bounds__(512, 2) void k_qs_blockkey(QsArgs a) {
    constexpr int RB = qs_rb(NK);
    constexpr int SLOT = RB * NK * 1024;        // bytes per ring slot
    constexpr int P = RB * NK / 8;              // 1 KiB DMA pieces per wave per slot
    constexpr int64_t TILE_B = (int64_t)NK * 8192;  // bytes per 256-row tile of a plane
    extern __shared__ __attribute__((aligned(16))) unsigned char qsm[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 31, lh = lane >> 5;
    const int total = a.nqg * a.nspans;
    const int b = blockIdx.x;
    // XCD-aware order: consecutive logical ids (the query groups of one span)
    // share an XCD and so read the span's rows through one L2
    const int logical = (total % 8 == 0) ? (b % 8) * (total / 8) + (b / 8) : b;
    const int span = logical / a.nqg, grp = logical % a.nqg;

    // One 32-row block per slot (d > 384) runs the 16x16x32 schedule below
    // (IL), smaller d the 32x32x16 schedule with several blocks per slot.
    constexpr bool IL = RB == 1;
    // this wave's 32 queries as MFMA B fragments for all of d.
    //  32x32x16: Qf[c] for 16-column chunk c: lane (li, lh) holds query
    //            wave*32+li, columns 16c + 8lh .. +7;
    //  16x16x32: Qf[2c+n] for 32-column chunk c and query half n: lane
    //            (j = lane&15, kq = lane>>4) holds query wave*32+16n+j,
    //            columns 32c + 8kq .. +7.
    bf16x8_t Qf[NK];
    if constexpr (IL) {
        const int j = lane & 15, kq = lane >> 4;
        const unsigned char* qp =
            a.Qb + (int64_t)grp * TILE_B + (kq >> 1) * 8192 + (wave * 32 + j) * 32 + 16 * (kq & 1);
#pragma unroll
        for (int c = 0; c < NK / 2; c++)
#pragma unroll
            for (int n = 0; n < 2; n++)
                Qf[2 * c + n] = *reinterpret_cast<const bf16x8_t*>(qp + (2 * c) * 8192 + n * 16 * 32);
    } else {
        const unsigned char* qp = a.Qb + (int64_t)grp * TILE_B + (wave * 32 + li) * 32 + 16 * lh;
#pragma unroll
        for (int c = 0; c < NK; c++) Qf[c] = *reinterpret_cast<const bf16x8_t*>(qp + c * 8192);
    }
    // retire the query loads in the compiler's books before any LDS-DMA is in
    // flight (otherwise its first use would drain the ring every iteration)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt/lgkmcnt untouched

    const int64_t s0 = (int64_t)span * a.slots_per_span;
    int64_t s1 = s0 + a.slots_per_span;
    if (s1 > a.nslots) s1 = a.nslots;
    const int nsteps = s1 > s0 ? (int)(s1 - s0) : 0;

    // LDS-DMA: lane L writes bytes [16L, 16L+16) of a 1 KiB piece = row L>>1,
    // physical half L&1, holding source half (L&1) ^ ((row>>3)&1): the
    // 16-lane groups of ds_read_b128 are then conflict-free
    // (the 16x16x32 schedule reads the image unswizzled: its 16-lane groups
    // are conflict-free on the linear layout)
    const int prow = lane >> 1;
    const uint32_t src_lane = IL ? (uint32_t)(16 * lane) : (uint32_t)(prow * 32 + 16 * ((lane & 1) ^ ((prow >> 3) & 1)));
    const unsigned ring = lds_addr(qsm);
    // per-wave rings with 4 entries (step & 3: never the entry being refilled
    // while an epilogue reads it): valid words [8][4][4] u32, L2 norms
    // [8][4][RB*32] floats.  Every wave loads its own copy, so every wave
    // issues the same number of vector-memory ops per step (one compile-time
    // vmcnt for the steady state).
    const unsigned vring = ring + QS_NBUF * SLOT + (unsigned)wave * 64u;
    const unsigned xnring = ring + QS_NBUF * SLOT + 512u + (unsigned)wave * (unsigned)(4 * RB * 128);
    constexpr int P0 = P + (ISL2 ? 2 : 1);  // vector-memory ops per step group, per wave
    // the span's rows through one buffer resource (the host keeps a span's
    // plane bytes below 4 GiB): per piece an SGPR offset + the lane's VGPR
    const int64_t tile0 = (s0 * RB * 32) >> 8;
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.Xb + tile0 * TILE_B), (short)0, -1, 0x00020000);
    // piece i of this wave: block rb_i of the slot, k chunk c_i -> source
    // offset K_i from the slot's first block, LDS offset Ld_i in the slot
    // source offset of the next group to issue: ((gb>>3) - tile0) * TILE_B + (gb&7) * 1024
    int64_t igb = s0 * RB;
    uint32_t ioff = (uint32_t)(((igb >> 3) - tile0) * TILE_B + (igb & 7) * 1024);
    auto issue = [&](int t, int slot) {
        const unsigned sb = ring + (unsigned)(slot * SLOT);
#pragma unroll
        for (int i = 0; i < P; i++) {
            const int p = wave + 8 * i;
            const int rb = p / NK, c = p % NK;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(size_t)(sb + (unsigned)((rb * NK + c) * 1024)), 16,
                                                     src_lane, ioff + (uint32_t)(rb * 1024 + c * 8192), 0, 0);
        }
        if (lane < RB)
            __builtin_amdgcn_global_load_lds(a.valid + igb + lane, (lds_ptr_t)(size_t)(vring + (unsigned)((t & 3) * 16)), 4, 0, 0);
        if (ISL2 && lane < RB * 8)
            __builtin_amdgcn_global_load_lds(a.xnorm2 + igb * 32 + 4 * lane,
                                             (lds_ptr_t)(size_t)(xnring + (unsigned)((t & 3) * RB * 128)), 16, 0, 0);
        igb += RB;
        ioff += RB * 1024;
        if ((igb & 7) == 0) ioff += (uint32_t)(TILE_B - 8192);
    };

    const unsigned lane_off = (unsigned)(li * 32 + 16 * (lh ^ ((li >> 3) & 1)));
    const int64_t qrow = (int64_t)grp * QS_QPB + wave * 32 + li;
    float* krow = a.key + qrow * a.ldk;
    bf16x8_t A[4];
    if (nsteps > 0) {
        issue(0, 0);
        if (nsteps > 1) issue(1, 1);
        qs_wait_vm(nsteps > 1 ? P0 : 0);  // group 0 landed, group 1 may stay in flight
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!IL) {  // the one-block schedule issues group 2 in its first chain
            if (nsteps > 2) issue(2, 2);
            const unsigned sb0 = ring + lane_off;
            A[0] = lds_ld8bf_o<0>(sb0);
            A[1] = lds_ld8bf_o<1024>(sb0);
            A[2] = lds_ld8bf_o<2048>(sb0);
            A[3] = lds_ld8bf_o<3072>(sb0);
        }
    }
    // ---------------------------------------------------------------------
    // One 32-row block per slot (d > 384): the epilogue of block t-1 and the
    // DMA of group t+2 run as fillers between block t's MFMAs, so the matrix
    // pipe never waits for them; one barrier per block.
    // ---------------------------------------------------------------------
    // ---------------------------------------------------------------------
    // One 32-row block per slot (d > 384), v_mfma_f32_16x16x32_bf16: per
    // 32-column chunk c, two row halves m x two query halves n.  The DMA of
    // group t+2 and the previous block's key store run as fillers between
    // block t's MFMAs; one barrier per block.
    // ---------------------------------------------------------------------
    if constexpr (IL) {
        constexpr int NC = NK / 2;
        // lane (i = lane&15, kq = lane>>4) reads row 16m+i, columns 32c+8kq..+7
        // = piece 2c + (kq>>1), half kq&1 of the linear image
        const unsigned l16 = (unsigned)(((lane >> 5) & 1) * 1024 + (lane & 15) * 32 + 16 * ((lane >> 4) & 1));
        auto issue_piece = [&](int j, int t, int slot) {
            if (j < P) {
                if constexpr (DBG & 2) return;
                const int c = wave + 8 * j;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(size_t)(ring + (unsigned)(slot * SLOT + c * 1024)),
                                                         16, src_lane, ioff + (uint32_t)(c * 8192), 0, 0);
            } else if (j == P) {
                if (lane == 0)
                    __builtin_amdgcn_global_load_lds(a.valid + igb, (lds_ptr_t)(size_t)(vring + (unsigned)((t & 3) * 16)), 4,
                                                     0, 0);
            } else {
                if (lane < 8)
                    __builtin_amdgcn_global_load_lds(a.xnorm2 + igb * 32 + 4 * lane,
                                                     (lds_ptr_t)(size_t)(xnring + (unsigned)((t & 3) * 128)), 16, 0, 0);
            }
            if (j == P0 - 1) {
                igb += 1;
                ioff += 1024;
                if ((igb & 7) == 0) ioff += (uint32_t)(TILE_B - 8192);
            }
        };
        bf16x8_t B2[2][2];  // A fragments [chunk & 1][m]
        if (nsteps > 0) {
            const unsigned sb0 = ring + l16;
            B2[0][0] = lds_ld8bf_o<0>(sb0);
            B2[0][1] = lds_ld8bf_o<512>(sb0);
        }
        // per query half n: the block's key before the cross-lane combine
        float mp0 = 0.f, mp1 = 0.f;
        int64_t gbp = 0;
        int cur = 0;
        auto finish = [&]() {
            // lanes g*16 + j (g = 0..3) hold partial keys of query 16n + j
            float m0 = mp0, m1 = mp1;
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
            if (lane < 32) krow[gbp] = ISL2 ? m : -m;
        };
        for (int t = 0; t < nsteps; t++) {
            const int nxt = cur == QS_NBUF - 1 ? 0 : cur + 1;
            const int gslot = cur == 0 ? QS_NBUF - 1 : cur - 1;  // slot of group t+2
            const unsigned sb = ring + (unsigned)(cur * SLOT) + l16;
            const bool dma = t + 2 < nsteps;
            const unsigned sm = (unsigned)(t & 3);
            f32x4_t acc[2][2];
#pragma unroll
            for (int m = 0; m < 2; m++)
#pragma unroll
                for (int n = 0; n < 2; n++) acc[m][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            uint32_t vwv = 0;
            f32x4_t x0, x1;
            // extra LDS reads (valid word, L2 norms) issued in chunk XC: the next
            // chunk's wait leaves them in flight, later waits retire them
            constexpr int XC = NC - 4;
            constexpr int XE = ISL2 ? 3 : 1;
            static_for<0, NC>([&](auto cc) {
                constexpr int c = decltype(cc)::value;
                if constexpr (c + 1 < NC && !(DBG & 4)) {
                    B2[(c + 1) & 1][0] = lds_ld8bf_o<(2 * (c + 1)) * 1024>(sb);
                    B2[(c + 1) & 1][1] = lds_ld8bf_o<(2 * (c + 1)) * 1024 + 512>(sb);
                }
                qs_wait_lgkm<(c + 1 < NC ? 2 : 0) + (c == XC + 1 ? XE : 0)>();
                asm volatile("" : "+v"(B2[c & 1][0]), "+v"(B2[c & 1][1]));
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (!(DBG & 1)) {
#pragma unroll
                    for (int m = 0; m < 2; m++)
#pragma unroll
                        for (int n = 0; n < 2; n++)
                            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B2[c & 1][m], Qf[2 * c + n], acc[m][n], 0, 0, 0);
                }
                // DMA of group t+2: one piece per chunk
                if constexpr (c < P0) {
                    if (dma) issue_piece(c, t + 2, gslot);
                }
                // previous block: cross-lane combine + key store
                if constexpr (c == P0 + 1) {
                    if (t > 0) finish();
                }
                if constexpr (c == XC) {
                    asm volatile("ds_read_b32 %0, %1" : "=v"(vwv) : "v"(vring + sm * 16u));
                    if constexpr (ISL2) {
                        // rows 4g..4g+3 and 16+4g..+3 of the block, g = lane>>4
                        const unsigned xb = xnring + sm * 128u + (unsigned)(16 * ((lane >> 4) & 3));
                        x0 = lds_ld4f_o<0>(xb);
                        x1 = lds_ld4f_o<64>(xb);
                    }
                }
            });
            // retired by the chunk waits after XC + 1
            if constexpr (ISL2) asm volatile("" : "+v"(vwv), "+v"(x0), "+v"(x1));
            else asm volatile("" : "+v"(vwv));
            {
                const uint32_t vw = __builtin_amdgcn_readfirstlane(vwv);
                // acc[m][n][r] is row 16m + 4g + r (g = lane>>4) of query 16n + (lane&15)
                const uint32_t vl = vw >> (4 * ((lane >> 4) & 3));
                float mn[2];
#pragma unroll
                for (int n = 0; n < 2; n++) {
                    if constexpr (ISL2) {
                        float m = __builtin_inff();
#pragma unroll
                        for (int mm = 0; mm < 2; mm++)
#pragma unroll
                            for (int r = 0; r < 4; r++) {
                                const float v = fmaf(-2.f, acc[mm][n][r], mm ? x1[r] : x0[r]);
                                m = fminf(m, ((vl >> (16 * mm + r)) & 1u) ? v : __builtin_inff());
                            }
                        mn[n] = m;
                    } else if (vw == 0xFFFFFFFFu) {
                        float m = fmaxf(fmaxf(acc[0][n][0], acc[0][n][1]), fmaxf(acc[0][n][2], acc[0][n][3]));
                        m = fmaxf(m, fmaxf(fmaxf(acc[1][n][0], acc[1][n][1]), fmaxf(acc[1][n][2], acc[1][n][3])));
                        mn[n] = m;
                    } else {
                        float m = -__builtin_inff();
#pragma unroll
                        for (int mm = 0; mm < 2; mm++)
#pragma unroll
                            for (int r = 0; r < 4; r++)
                                m = fmaxf(m, ((vl >> (16 * mm + r)) & 1u) ? acc[mm][n][r] : -__builtin_inff());
                        mn[n] = m;
                    }
                }
                mp0 = mn[0];
                mp1 = mn[1];
                gbp = s0 + t;
            }
            // ---- end of the block: the next group must have landed (every wave) ----
            if (t + 1 < nsteps) {
                // vector-memory ops of this wave after group t+1, in issue order:
                // store(t-2), the pieces of group t+2, store(t-1)
                if constexpr (DBG & 2) {
                    qs_wait_vm_c<0>();
                } else if (t >= 2 && t + 2 < nsteps) {
                    qs_wait_vm_c<P0 + 2>();
                } else {
                    const int y = (t >= 1 ? 1 : 0) + (t >= 2 ? 1 : 0) + (t + 2 < nsteps ? P0 : 0);
                    qs_wait_vm(y);
                }
                __builtin_amdgcn_s_barrier();  // slot t is free; slot t+1 has landed for every wave
                __builtin_amdgcn_sched_barrier(0);
                const unsigned sbn = ring + (unsigned)(nxt * SLOT) + l16;
                B2[0][0] = lds_ld8bf_o<0>(sbn);
                B2[0][1] = lds_ld8bf_o<512>(sbn);
            }
            cur = nxt;
        }
        if (nsteps > 0) finish();
        return;
    }
    int cur = 0;
    for (int t = 0; t < nsteps; t++) {
        const int nxt = cur == QS_NBUF - 1 ? 0 : cur + 1;
        const unsigned sb = ring + (unsigned)(cur * SLOT) + lane_off;
        const unsigned sbn = ring + (unsigned)(nxt * SLOT) + lane_off;
        const unsigned sm = (unsigned)(t & 3);
        static_for<0, RB>([&](auto rbc) {
            constexpr int rb = decltype(rbc)::value;
            // ---- the block's 32 rows x this wave's 32 queries: NK MFMAs, A fragments 4 ahead ----
            f32x16 acc;
#pragma unroll
            for (int r = 0; r < 16; r++) acc[r] = 0.f;
            static_for<0, NK>([&](auto cc) {
                constexpr int c = decltype(cc)::value;
                qs_wait_lgkm<(NK - 1 - c) < 3 ? (NK - 1 - c) : 3>();
                asm volatile("" : "+v"(A[c & 3]));
                __builtin_amdgcn_sched_barrier(0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[c & 3], Qf[c], acc, 0, 0, 0);
                if constexpr (c + 4 < NK) A[c & 3] = lds_ld8bf_o<(rb * NK + c + 4) * 1024>(sb);
            });
            // ---- end of the slot: the next group must have landed (every wave) ----
            if constexpr (rb == RB - 1) {
                if (t + 1 < nsteps) {
                    // ops of this wave issued after group t+1, in issue order (vmcnt
                    // counts the LDS-DMA pieces and the key stores together)
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
            asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(vwv) : "v"(vring + sm * 16u), "i"(rb * 4));
            float m;
            if constexpr (ISL2) {
                const unsigned xb = xnring + sm * (unsigned)(RB * 128) + (unsigned)(rb * 128 + 16 * lh);
                f32x4_t x0 = lds_ld4f_o<0>(xb), x1 = lds_ld4f_o<32>(xb), x2 = lds_ld4f_o<64>(xb), x3 = lds_ld4f_o<96>(xb);
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vwv), "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
                const uint32_t vw = __builtin_amdgcn_readfirstlane(vwv);
                const uint32_t vl = vw >> (4 * lh);
                const float xn[16] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3],
                                      x2[0], x2[1], x2[2], x2[3], x3[0], x3[1], x3[2], x3[3]};
                m = __builtin_inff();
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    float v = fmaf(-2.f, acc[r], xn[r]);
                    if (vw != 0xFFFFFFFFu) v = ((vl >> ((r & 3) + 8 * (r >> 2))) & 1u) ? v : __builtin_inff();
                    m = fminf(m, v);
                }
                // next block's first fragments (after the epilogue reads: registers)
                const unsigned pb = rb + 1 < RB ? sb : sbn;
                constexpr int pr = rb + 1 < RB ? rb + 1 : 0;
                A[0] = lds_ld8bf_o<(pr * NK + 0) * 1024>(pb);
                A[1] = lds_ld8bf_o<(pr * NK + 1) * 1024>(pb);
                A[2] = lds_ld8bf_o<(pr * NK + 2) * 1024>(pb);
                A[3] = lds_ld8bf_o<(pr * NK + 3) * 1024>(pb);
                const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
                m = fminf(m, __uint_as_float(sw[1]));
            } else {
                // next block's first fragments, in flight during the epilogue
                const unsigned pb = rb + 1 < RB ? sb : sbn;
                constexpr int pr = rb + 1 < RB ? rb + 1 : 0;
                A[0] = lds_ld8bf_o<(pr * NK + 0) * 1024>(pb);
                A[1] = lds_ld8bf_o<(pr * NK + 1) * 1024>(pb);
                A[2] = lds_ld8bf_o<(pr * NK + 2) * 1024>(pb);
                A[3] = lds_ld8bf_o<(pr * NK + 3) * 1024>(pb);
                asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(vwv));
                const uint32_t vw = __builtin_amdgcn_readfirstlane(vwv);
                const uint32_t vl = vw >> (4 * lh);
                m = -__builtin_inff();
                if (vw == 0xFFFFFFFFu) {
#pragma unroll
                    for (int r = 0; r < 16; r++) m = fmaxf(m, acc[r]);
                } else {
#pragma unroll
                    for (int r = 0; r < 16; r++)
                        m = fmaxf(m, ((vl >> ((r & 3) + 8 * (r >> 2))) & 1u) ? acc[r] : -__builtin_inff());
                }
                const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
                m = -fmaxf(m, __uint_as_float(sw[1]));
            }
            if (lh == 0) krow[gb] = m;
        });
        cur = nxt;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the last (unused) prefetch
}

// ---------------------------------------------------------------------------
// k_qs_blockkey_w4<NK, L2, NB>: the same block keys for 768 < d <= 1536 (dpb
// 1024 or 1536, NK = dpb / 16 in {64, 96}).  32 queries x dpb bf16 are NK x 4
// registers per lane -- more than two waves per SIMD leave -- so the
// workgroup is 4 waves, one per SIMD (512-entry register file: the stationary
// query fragments go to AGPRs), 128 queries.  A 32-row block is staged in
// NP = NK / 32 column parts of 512 columns (32 KiB per ring slot), one ring
// step per part; the accumulators run across the parts and the key epilogue
// follows the last.  NB ring slots: the DMA of the group NB - 1 steps ahead is
// issued during a step (128 queries per workgroup read the corpus at twice
// the per-flop rate of the 256-query k_qs_blockkey, so the L2 latency needs
// the deeper ring).  Per 32-column chunk: 2 A reads, 4
// v_mfma_f32_16x16x32_bf16 (2 row halves x 2 query halves), the DMA pieces
// and the previous block's key store as fillers.
// ---------------------------------------------------------------------------
template <int NK, bool ISL2, int NP, int NB>
__global__ __launch_bounds__(256, 1) void k_qs_blockkey_w4(QsArgs a) {
    constexpr int QH = 2;                           // query halves (16 queries) per wave
    constexpr int NCP = NK / (2 * NP);              // 32-column chunks per part
    constexpr int SLOT = NCP * 2048;                // bytes per ring slot (32 rows x the part's columns)
    constexpr int AF = 3;                           // A-fragment sets in flight (chunks c .. c+2)
    constexpr int P = NCP / 2;                      // 1 KiB DMA pieces per wave per step (2 NCP / 4 waves)
    constexpr int PX = ISL2 ? 2 : 1;                // valid word (+ the L2 norms): with a block's first part
    constexpr int64_t TILE_B = (int64_t)NK * 8192;  // bytes per 256-row tile of a plane
    constexpr int QPB = 64 * QH;                    // queries per workgroup
    constexpr int XC = NCP - 4;                     // chunk of the last part that reads valid / norms
    constexpr int XE = ISL2 ? 3 : 1;
    static_assert(NK % (2 * NP) == 0 && NCP % 2 == 0, "parts of whole 32-column chunk pairs");
    static_assert(P + PX + 1 < XC, "filler chunks overlap");
    extern __shared__ __attribute__((aligned(16))) unsigned char qsm[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int total = a.nqg * a.nspans;
    const int b = blockIdx.x;
    const int logical = (total % 8 == 0) ? (b % 8) * (total / 8) + (b / 8) : b;
    const int span = logical / a.nqg, grp = logical % a.nqg;

    // Qf[QH c + n]: lane (j = lane&15, kq = lane>>4) holds query q0 + 16n + j,
    // columns 32c + 8kq .. +7 (the 16x16x32 B fragment)
    bf16x8_t Qf[NK / 2 * QH];
    const int64_t q0 = (int64_t)grp * QPB + wave * 16 * QH;
    {
        const int j = lane & 15, kq = lane >> 4;
        const unsigned char* qp = a.Qb + (q0 >> 8) * TILE_B + (kq >> 1) * 8192 + ((q0 & 255) + j) * 32 + 16 * (kq & 1);
#pragma unroll
        for (int c = 0; c < NK / 2; c++)
#pragma unroll
            for (int n = 0; n < QH; n++)
                Qf[QH * c + n] = *reinterpret_cast<const bf16x8_t*>(qp + (2 * c) * 8192 + n * 16 * 32);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the query loads retire before any LDS-DMA

    const int64_t s0 = (int64_t)span * a.slots_per_span;
    int64_t s1 = s0 + a.slots_per_span;
    if (s1 > a.nslots) s1 = a.nslots;
    const int nblk = s1 > s0 ? (int)(s1 - s0) : 0;
    const int G = NP * nblk;  // ring steps

    const unsigned ring = lds_addr(qsm);
    const unsigned vring = ring + NB * SLOT + (unsigned)wave * 64u;           // [4] x 16 B valid words
    const unsigned xnring = ring + NB * SLOT + 256u + (unsigned)wave * 512u;  // [4] x 32 floats
    const int64_t tile0 = (s0 * 32) >> 8;
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.Xb + tile0 * TILE_B), (short)0, -1, 0x00020000);
    const uint32_t src_lane = (uint32_t)(16 * lane);
    // the next group to issue: block igb, part ih; ioff = its block's offset in the span's buffer
    int64_t igb = s0;
    int ih = 0;
    uint32_t ioff = (uint32_t)(((igb >> 3) - tile0) * TILE_B + (igb & 7) * 1024);
    // piece j of the next group into ring slot `slot`; the group's last piece advances it
    auto issue_piece = [&](int j, int slot, int pg) {
        if (j < P) {
            const int cc = wave + 4 * j;  // 16-column chunk of the part
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(size_t)(ring + (unsigned)(slot * SLOT + cc * 1024)),
                                                     16, src_lane, ioff + (uint32_t)((ih * 2 * NCP + cc) * 8192), 0, 0);
        } else if (j == P) {
            if (lane == 0)
                __builtin_amdgcn_global_load_lds(a.valid + igb, (lds_ptr_t)(size_t)(vring + (unsigned)((igb & 3) * 16)), 4,
                                                 0, 0);
        } else {
            if (lane < 8)
                __builtin_amdgcn_global_load_lds(a.xnorm2 + igb * 32 + 4 * lane,
                                                 (lds_ptr_t)(size_t)(xnring + (unsigned)((igb & 3) * 128)), 16, 0, 0);
        }
        if (j == pg - 1) {
            if (ih == NP - 1) {
                ih = 0;
                igb += 1;
                ioff += 1024;
                if ((igb & 7) == 0) ioff += (uint32_t)(TILE_B - 8192);
            } else {
                ih += 1;
            }
        }
    };
    auto issue_group = [&](int slot) {
        const int pg = P + (ih == 0 ? PX : 0);
        for (int j = 0; j < pg; j++) issue_piece(j, slot, pg);
    };
    // this wave's vector-memory ops issued after those of group g+1, once step
    // g has issued its own: the groups g+2 .. g+NB-1 and the key stores of the
    // steps from the one that issued group g+1 (store after pieces) to g
    auto ops_after = [&](int g) {
        int y = 0;
        for (int j = g + 2; j <= g + NB - 1 && j < G; j++) y += P + (j % NP == 0 ? PX : 0);
        for (int x = g + 2 - NB < 0 ? 0 : g + 2 - NB; x <= g; x++) y += (x % NP == 0 && x >= NP) ? 1 : 0;
        return y;
    };

    // lane (i = lane&15, kq = lane>>4) reads row 16m + i, columns 32c + 8kq .. +7
    const unsigned l16 = (unsigned)(((lane >> 5) & 1) * 1024 + (lane & 15) * 32 + 16 * ((lane >> 4) & 1));
    // the key row this lane stores: query q0 + lane (lanes < 16 QH)
    float* krow = a.key + (q0 + (lane < 16 * QH ? lane : 0)) * a.ldk;
    // A fragments of chunks c, c+1, c+2 in flight: with one wave per SIMD no
    // partner wave covers an LDS read's latency, 4 MFMAs per chunk do not
    bf16x8_t B2[AF][2];
    if (G > 0) {
        for (int j = 0; j < NB - 1 && j < G; j++) issue_group(j);
        qs_wait_vm(ops_after(0));  // group 0 landed, groups 1 .. NB-2 may stay in flight
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        B2[0][0] = lds_ld8bf_o<0>(ring + l16);
        B2[0][1] = lds_ld8bf_o<512>(ring + l16);
        B2[1][0] = lds_ld8bf_o<2048>(ring + l16);
        B2[1][1] = lds_ld8bf_o<2048 + 512>(ring + l16);
    }
    float mp[QH];
#pragma unroll
    for (int n = 0; n < QH; n++) mp[n] = 0.f;
    int64_t gbp = 0;
    auto finish = [&]() {  // previous block: cross-lane combine (the 4 row groups) + key store
        float m[QH];
#pragma unroll
        for (int n = 0; n < QH; n++) {
            float v = mp[n];
            const auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
            v = ISL2 ? fminf(v, __uint_as_float(x[1])) : fmaxf(v, __uint_as_float(x[1]));
            const auto y = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
            m[n] = ISL2 ? fminf(v, __uint_as_float(y[1])) : fmaxf(v, __uint_as_float(y[1]));
        }
        // only row 0 (lanes 0-15) of each m[n] holds all four row groups; gather
        // those rows: lane 16n + j of the store value = query 16n + j
        const auto c01 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m[0]), __float_as_uint(m[1]), false, false);
        const float v = __uint_as_float(c01[0]);  // rows: m0.r0, m1.r0, ..
        if (lane < 16 * QH) krow[gbp] = ISL2 ? v : -v;
    };
    int cur = 0;
    for (int tb = 0; tb < nblk; tb++) {
        f32x4_t acc[2][QH];
#pragma unroll
        for (int m = 0; m < 2; m++)
#pragma unroll
            for (int n = 0; n < QH; n++) acc[m][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        uint32_t vwv = 0;
        f32x4_t x0 = f32x4_t{0.f, 0.f, 0.f, 0.f}, x1 = x0;
        static_for<0, NP>([&](auto hh) {
            constexpr int H = decltype(hh)::value;
            const int g = NP * tb + H;
            const int nxt = cur == NB - 1 ? 0 : cur + 1;
            const int gslot = cur == 0 ? NB - 1 : cur - 1;  // slot of group g + NB - 1
            const unsigned sb = ring + (unsigned)(cur * SLOT) + l16;
            const bool dma = g + NB - 1 < G;
            constexpr int PG = P + ((H + NB - 1) % NP == 0 ? PX : 0);  // ops of group g + NB - 1
            static_for<0, NCP>([&](auto cc) {
                constexpr int c = decltype(cc)::value;
                if constexpr (c + 2 < NCP) {
                    B2[(c + 2) % AF][0] = lds_ld8bf_o<(2 * (c + 2)) * 1024>(sb);
                    B2[(c + 2) % AF][1] = lds_ld8bf_o<(2 * (c + 2)) * 1024 + 512>(sb);
                }
                // chunk c's reads done; those of c+1, c+2 (and the valid / norm reads
                // issued in chunk XC, behind c+2 = XC+2's) may stay in flight
                qs_wait_lgkm<2 * (NCP - 1 - c < 2 ? NCP - 1 - c : 2) +
                             (H == NP - 1 && (c == XC + 1 || c == XC + 2) ? XE : 0)>();
                asm volatile("" : "+v"(B2[c % AF][0]), "+v"(B2[c % AF][1]));
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int m = 0; m < 2; m++)
#pragma unroll
                    for (int n = 0; n < QH; n++)
                        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B2[c % AF][m], Qf[QH * (H * NCP + c) + n],
                                                                            acc[m][n], 0, 0, 0);
                if constexpr (c < PG) {
                    if (dma) issue_piece(c, gslot, PG);
                }
                if constexpr (H == 0 && c == PG + 1) {
                    if (tb > 0) finish();
                }
                if constexpr (H == NP - 1 && c == XC) {
                    asm volatile("ds_read_b32 %0, %1" : "=v"(vwv) : "v"(vring + (unsigned)(((s0 + tb) & 3) * 16)));
                    if constexpr (ISL2) {
                        // rows 4g..4g+3 and 16+4g..+3 of the block, g = lane>>4
                        const unsigned xb = xnring + (unsigned)(((s0 + tb) & 3) * 128) + (unsigned)(16 * ((lane >> 4) & 3));
                        x0 = lds_ld4f_o<0>(xb);
                        x1 = lds_ld4f_o<64>(xb);
                    }
                }
            });
            if constexpr (H == NP - 1) {
                if constexpr (ISL2) asm volatile("" : "+v"(vwv), "+v"(x0), "+v"(x1));
                else asm volatile("" : "+v"(vwv));
                const uint32_t vw = __builtin_amdgcn_readfirstlane(vwv);
                // acc[m][n][r] is row 16m + 4g + r (g = lane>>4) of query 16n + (lane&15)
                const uint32_t vl = vw >> (4 * ((lane >> 4) & 3));
#pragma unroll
                for (int n = 0; n < QH; n++) {
                    if constexpr (ISL2) {
                        float m = __builtin_inff();
#pragma unroll
                        for (int mm = 0; mm < 2; mm++)
#pragma unroll
                            for (int r = 0; r < 4; r++) {
                                const float v = fmaf(-2.f, acc[mm][n][r], mm ? x1[r] : x0[r]);
                                m = fminf(m, ((vl >> (16 * mm + r)) & 1u) ? v : __builtin_inff());
                            }
                        mp[n] = m;
                    } else if (vw == 0xFFFFFFFFu) {
                        float m = fmaxf(fmaxf(acc[0][n][0], acc[0][n][1]), fmaxf(acc[0][n][2], acc[0][n][3]));
                        m = fmaxf(m, fmaxf(fmaxf(acc[1][n][0], acc[1][n][1]), fmaxf(acc[1][n][2], acc[1][n][3])));
                        mp[n] = m;
                    } else {
                        float m = -__builtin_inff();
#pragma unroll
                        for (int mm = 0; mm < 2; mm++)
#pragma unroll
                            for (int r = 0; r < 4; r++)
                                m = fmaxf(m, ((vl >> (16 * mm + r)) & 1u) ? acc[mm][n][r] : -__builtin_inff());
                        mp[n] = m;
                    }
                }
                gbp = s0 + tb;
            }
            // ---- end of the step: group g + 1 must have landed (every wave) ----
            if (g + 1 < G) {
                qs_wait_vm(ops_after(g));
                __builtin_amdgcn_s_barrier();  // slot g is free; slot g+1 has landed for every wave
                __builtin_amdgcn_sched_barrier(0);
                const unsigned sbn = ring + (unsigned)(nxt * SLOT) + l16;
                B2[0][0] = lds_ld8bf_o<0>(sbn);
                B2[0][1] = lds_ld8bf_o<512>(sbn);
                B2[1][0] = lds_ld8bf_o<2048>(sbn);
                B2[1][1] = lds_ld8bf_o<2048 + 512>(sbn);
            }
            cur = nxt;
        });
    }
    if (nblk > 0) finish();
}

// ---------------------------------------------------------------------------
// bf16 hi planes + residual norms
// ---------------------------------------------------------------------------
// Corpus rows (listed slots or [0, n)): Xb[slot] = bf16(X[slot]) into the tiled
// plane; per row |x_h|^2 and |x - x_h|^2 update the index maxima (atomicMax on
// float bits), and a non-finite value or an overflowing norm sets nonfinite.
// One wave per row.
__global__ void k_rows_split(const float* __restrict__ X, int dpad, int dpb, int64_t n, const uint32_t* __restrict__ slots,
                             uint16_t* __restrict__ Xb, uint32_t* __restrict__ qsmax) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r >= n) return;
    const int64_t row = slots ? (int64_t)slots[r] : r;
    const float* x = X + row * dpad;
    float sh = 0.f, sr = 0.f, sx = 0.f;
    bool bad = false;
    for (int c = lane; c < dpb; c += 64) {
        const float v = c < dpad ? x[c] : 0.f;
        const __bf16 h = (__bf16)v;
        const float hf = (float)h;
        const float rv = v - hf;
        sh = fmaf(hf, hf, sh);
        sr = fmaf(rv, rv, sr);
        sx = fmaf(v, v, sx);
        bad |= !__builtin_isfinite(v);
        Xb[bf3_plane_index(row, c, dpb)] = __builtin_bit_cast(uint16_t, h);
    }
    for (int o = 32; o > 0; o >>= 1) {
        sh += __shfl_xor(sh, o);
        sr += __shfl_xor(sr, o);
        sx += __shfl_xor(sx, o);
    }
    bad = __any(bad);
    if (lane == 0) {
        atomicMax(&qsmax[0], __float_as_uint(sr));
        atomicMax(&qsmax[1], __float_as_uint(sh));
        if (bad || !(sx < 1e30f) || !(sh < 1e30f)) atomicOr(&qsmax[2], 1u);
    }
}

// Queries: Qb plane row q = bf16(Qn[q]) (rows [nq, nq_pad) are zero), and
// qinfo[q] = (|q|^2, |q_h|^2, |q - q_h|^2, non-finite ? 1 : 0).  Wave per row.
__global__ void k_query_split(const float* __restrict__ Qn, int dpad, int dpb, int64_t nq, int64_t nq_pad,
                              uint16_t* __restrict__ Qb, float4* __restrict__ qinfo) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (q >= nq_pad) return;
    float sh = 0.f, sr = 0.f, sx = 0.f;
    bool bad = false;
    for (int c = lane; c < dpb; c += 64) {
        const float v = (q < nq && c < dpad) ? Qn[q * dpad + c] : 0.f;
        const __bf16 h = (__bf16)v;
        const float hf = (float)h;
        const float rv = v - hf;
        sh = fmaf(hf, hf, sh);
        sr = fmaf(rv, rv, sr);
        sx = fmaf(v, v, sx);
        bad |= !__builtin_isfinite(v);
        Qb[bf3_plane_index(q, c, dpb)] = __builtin_bit_cast(uint16_t, h);
    }
    for (int o = 32; o > 0; o >>= 1) {
        sh += __shfl_xor(sh, o);
        sr += __shfl_xor(sr, o);
        sx += __shfl_xor(sx, o);
    }
    bad = __any(bad);
    if (lane == 0) qinfo[q] = make_float4(sx, sh, sr, (bad || !(sx < 1e30f)) ? 1.f : 0.f);
}

// ---------------------------------------------------------------------------
// per-query error bound eps(q) >= |A - E| for every stored row
//   dot_err = |q_h| R + |q_r| H + |q_r| R + g_acc |q_h| H + g_d |q| N
//   dot / cosine: eps = 1.05 (dot_err + 4u (1 + |q| N))
//   l2:           eps = 1.05 (2 dot_err + (2 g_d + 8u) (|q| + N)^2)
// N, H, R = max over stored rows of |x|, |x_h|, |x - x_h|; the fp32 sums of
// squares are inflated by 1e-4 (> gamma_d) before the square roots.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float qs_eps(int metric, float4 qi, const uint32_t* qsmax, const uint32_t* maxn2, float gd,
                                        float gacc) {
    const float infl = 1.0001f;
    const float nq = sqrtf(qi.x * infl), nh = sqrtf(qi.y * infl), nr = sqrtf(qi.z * infl);
    const float Nx = sqrtf(__uint_as_float(*maxn2) * infl);
    const float Rx = sqrtf(__uint_as_float(qsmax[0]) * infl);
    const float Hx = sqrtf(__uint_as_float(qsmax[1]) * infl);
    const float u = 5.9604645e-08f;
    const float dot_err = nh * Rx + nr * Hx + nr * Rx + gacc * nh * Hx + gd * nq * Nx;
    float e;
    if (metric == L2) { const float t = nq + Nx; e = 2.f * dot_err + (2.f * gd + 8.f * u) * t * t; }
    else e = dot_err + 4.f * u * (1.f + nq * Nx);
    return e * 1.05f + 1e-30f;
}

// monotone map from a block key to the block's smallest approximate distance A
__device__ __forceinline__ float qs_key_to_a(int metric, float key, float qn2) {
    if (metric == L2) return key + qn2;
    if (metric == DOT) return key;
    const float p = 1.f + key;
    return p < 0.f ? 0.f : p;
}

// the next float toward +inf (finite x)
__device__ __forceinline__ float qs_next_up(float x) {
    if (!(x < __builtin_inff())) return x;
    if (x == 0.f) return 1.4e-45f;
    const uint32_t b = __float_as_uint(x);
    return __uint_as_float(x > 0.f ? b + 1u : b - 1u);
}

// the next float below x (finite x): -qs_next_up(-x)
__device__ __forceinline__ float qs_next_down(float x) { return -qs_next_up(-x); }

// ---------------------------------------------------------------------------
// wave-level streaming selection of the L = 64 (R-1) smallest (key, id) pairs:
// list in rows 0..R-2 of the register arrays (sorted), row R-1 takes the LDS
// buffer of pending values at a merge.  thr = the L-th smallest so far.
// ---------------------------------------------------------------------------
template <int R>
struct WaveTopL {
    float key[R];
    uint32_t id[R];
    float thr;
    float cap;  // values >= cap are never kept (a known upper bound of the wanted prefix)
    int cnt;
    __device__ __forceinline__ void init(float cap_ = __builtin_inff()) {
#pragma unroll
        for (int r = 0; r < R; r++) { key[r] = __builtin_inff(); id[r] = NO_ID; }
        thr = cap = cap_;
        cnt = 0;
    }
    // rows 0..R-2 are sorted: only the pending row is sorted, then merged
    __device__ __forceinline__ void merge(const float* bk, const uint32_t* bi, int lane) {
        key[R - 1] = lane < cnt ? bk[lane] : __builtin_inff();
        id[R - 1] = lane < cnt ? bi[lane] : NO_ID;
        bitonic_merge_last<R>(key, id, lane);
        thr = fminf(__shfl(key[R - 2], 63), cap);
        cnt = 0;
    }
    // offer one value per lane; `c` = this lane's value passes (v < thr)
    __device__ __forceinline__ void offer(float v, uint32_t vid, float* bk, uint32_t* bi, int lane) {
        bool c = v < thr;
        uint64_t m = __ballot(c);
        if (m == 0) return;
        int n = __popcll(m);
        if (cnt + n > 64) {
            merge(bk, bi, lane);
            c = v < thr;
            m = __ballot(c);
            if (m == 0) return;
            n = __popcll(m);
        }
        const int pos = cnt + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        if (c) { bk[pos] = v; bi[pos] = vid; }
        cnt += n;
    }
    // element e (0-based) of the sorted list, broadcast
    __device__ __forceinline__ float key_at(int e) const {
        float v = 0.f;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const float t = __shfl(key[r], e & 63);
            if ((e >> 6) == r) v = t;
        }
        return v;
    }
};

// k_blk_select<R>: wave per query.  Candidate blocks (ids, ascending by key)
// -> cand[q][L], count -> ncand[q]; flags[q] = 2 when the list of L could not
// hold every block within 2 eps of M (the exact replay then resolves q).
template <int R>
__global__ __launch_bounds__(256) void k_blk_select(const float* __restrict__ key, int64_t ldk, int64_t nb, int nq, int k,
                                                    int metric, const float4* __restrict__ qinfo,
                                                    const uint32_t* __restrict__ qsmax, const uint32_t* __restrict__ maxn2,
                                                    float gd, float gacc, uint32_t* __restrict__ cand,
                                                    int32_t* __restrict__ ncand, int32_t* __restrict__ flags,
                                                    float* __restrict__ eps_out, const int32_t* __restrict__ qlist,
                                                    const uint32_t* __restrict__ qcount, float* __restrict__ topA,
                                                    float* __restrict__ cap_out = nullptr,
                                                    uint32_t* __restrict__ list_ctr = nullptr,
                                                    float* __restrict__ t_out = nullptr,
                                                    const uint32_t* __restrict__ pv = nullptr, int64_t pvq = 0,
                                                    const int32_t* __restrict__ mq = nullptr) {
    // the batch's flag-list cursors (k_flag_list counters[1] of the final and
    // the overflow lists), reset here instead of by two fills
    if (list_ctr && blockIdx.x == 0 && threadIdx.x == 0) {
        list_ctr[1] = 0u;
        list_ctr[3] = 0u;
    }
    constexpr int L = 64 * (R - 1);
    constexpr int U = 16;
    __shared__ float sbk[4][64];
    __shared__ uint32_t sbi[4][64];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    int q = blockIdx.x * 4 + w;
    if (qlist) {  // second pass over the listed queries (qcount[1] of them)
        if ((uint32_t)q >= qcount[1]) return;
        q = qlist[q];
    }
    if (q >= nq) return;
    const float4 qi = qinfo[q];
    const float eps = qs_eps(metric, qi, qsmax, maxn2, gd, gacc);
    const float* kr = key + (int64_t)q * ldk;
    // per-query allow bitmaps (pvq words each): a block without a row of the
    // query's own (its bitmap word, one per 32-row block) is not a candidate
    const uint32_t* vr = pvq ? pv + (int64_t)q * pvq : nullptr;
    WaveTopL<R> t;
    t.init();
    for (int64_t b0 = 0; b0 < nb; b0 += 64 * U) {
        float v[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const int64_t bb = b0 + j * 64 + lane;
            v[j] = bb < nb && (!vr || vr[bb]) ? kr[bb] : __builtin_inff();
        }
        bool any = false;
#pragma unroll
        for (int j = 0; j < U; j++) any |= v[j] < t.thr;
        if (!__any(any)) continue;
#pragma unroll
        for (int j = 0; j < U; j++) t.offer(v[j], (uint32_t)(b0 + j * 64 + lane), sbk[w], sbi[w], lane);
    }
    t.merge(sbk[w], sbi[w], lane);
    // M = A of the (k+1)-th smallest block key; T = M + 2 eps.  mq (per-query
    // allow lists): the mq[q]-th instead -- a block's key need not come from a
    // row of the query's own, so sparser lists take a deeper threshold (any T
    // keeps k_blk_exact's completeness proof; a deeper one passes it more often)
    const int me = mq ? (mq[q] < k + 1 ? k : mq[q] > L ? L - 1 : mq[q] - 1) : k;
    const float mk = t.key_at(me);
    const float M = qs_key_to_a(metric, mk, qi.x);
    float T = mk == __builtin_inff() ? __builtin_inff() : M + 2.0005f * eps;
    // a threshold the list can hold: below the L-th smallest A (rows 0..R-2
    // hold exactly the L smallest keys; row R-1 is not kept exact).  Always
    // for per-query lists (mq); else (t_out) instead of the overflow flag when
    // more than the list would qualify: k_blk_exact then proves the list
    // complete against T (its (k+1)-th exact distance <= T - eps) or flags it
    bool conv = false;
    if (mq || t_out) {
        const float kl = t.key_at(L - 1);
        const float al = qs_key_to_a(metric, kl, qi.x);
        if (kl < __builtin_inff() && (mq || al <= T)) {
            conv = !mq && qs_next_down(al) < T;
            T = fminf(T, qs_next_down(al));
        }
    }
    const bool proof = mq || conv;  // completeness against T in k_blk_exact
    int nc = 0;
#pragma unroll
    for (int r = 0; r < R - 1; r++) {
        const int e = r * 64 + lane;
        const bool in = t.key[r] < __builtin_inff() && qs_key_to_a(metric, t.key[r], qi.x) <= T;
        if (in) cand[(int64_t)q * L + e] = t.id[r];
        nc += __popcll(__ballot(in));
    }
    if (lane == 0) {
        ncand[q] = nc;
        eps_out[q] = eps;
        // the k+1 smallest blocks each hold a row with E <= A + eps <= M + eps, so
        // the (k+1)-th smallest exact distance over the candidates is below cap
        // (per-query lists: those blocks' rows need not be the query's; rows at
        // or above T - eps cannot pass k_blk_exact's completeness test anyway)
        if (cap_out)
            cap_out[q] = mk == __builtin_inff() ? __builtin_inff()
                         : proof ? T - eps : qs_next_up(M + 1.001f * eps);
        // k_blk_exact's completeness bound (+inf: the 2-eps argument holds)
        if (t_out) t_out[q] = proof ? T : __builtin_inff();
        // the L-th entry also qualifies: blocks beyond the list may too
        // (proof: T is below every block past the list)
        flags[q] = ((nc >= L && !proof) || qi.w != 0.f) ? 2 : 0;
    }
    if (topA) {  // sharded phase 1: this shard's k+1 smallest block-key A values
#pragma unroll
        for (int r = 0; r < R - 1; r++) {
            const int e = r * 64 + lane;
            if (e <= k) topA[(int64_t)q * (k + 1) + e] = qs_key_to_a(metric, t.key[r], qi.x);
        }
    }
}

// k_blk_select_f<R, RT>: k_blk_select's selection by filtering instead of a
// sorted L-list.  The wave keeps only the 64 (RT - 1) smallest keys (enough for
// M = the (k+1)-th; RT = qs_R(k)) and appends every block with A <= T_cur =
// A(M_cur) + 2 eps to an LDS buffer of L + 64 entries.  M_cur (the merged
// list's (k+1)-th) only falls, so T_cur bounds the final T from above: no
// qualifying block is missed; a full buffer is compacted with the current
// T_cur, and at the end with the final T.  The candidate list comes out in
// scan order, not sorted (k_blk_exact takes any order; k_blk_gthresh
// compacts).  flags[q] = 2 when more than L blocks qualify.  Same outputs
// (ncand, eps, cap, topA, flags) and the same candidate set as k_blk_select.
template <int R, int RT>
__global__ __launch_bounds__(256) void k_blk_select_f(const float* __restrict__ key, int64_t ldk, int64_t nb, int nq,
                                                      int k, int metric, const float4* __restrict__ qinfo,
                                                      const uint32_t* __restrict__ qsmax,
                                                      const uint32_t* __restrict__ maxn2, float gd, float gacc,
                                                      uint32_t* __restrict__ cand, int32_t* __restrict__ ncand,
                                                      int32_t* __restrict__ flags, float* __restrict__ eps_out,
                                                      const int32_t* __restrict__ qlist,
                                                      const uint32_t* __restrict__ qcount, float* __restrict__ topA,
                                                      float* __restrict__ cap_out, uint32_t* __restrict__ list_ctr,
                                                      float* __restrict__ t_out = nullptr) {
    if (list_ctr && blockIdx.x == 0 && threadIdx.x == 0) {
        list_ctr[1] = 0u;
        list_ctr[3] = 0u;
    }
    constexpr int L = 64 * (R - 1);
    constexpr int CB = L + 64;
    constexpr int U = 16;
    __shared__ float sbk[4][64];
    __shared__ uint32_t sbi[4][64];
    __shared__ float cbk[4][CB];
    __shared__ uint32_t cbi[4][CB];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    int q = blockIdx.x * 4 + w;
    if (qlist) {
        if ((uint32_t)q >= qcount[1]) return;
        q = qlist[q];
    }
    if (q >= nq) return;
    const float4 qi = qinfo[q];
    const float eps = qs_eps(metric, qi, qsmax, maxn2, gd, gacc);
    const float* kr = key + (int64_t)q * ldk;
    WaveTopL<RT> t;
    t.init();
    float T = __builtin_inff();
    float Kt = __builtin_inff();  // key-space prefilter: A(v) <= T implies v <= Kt
    int nc = 0;
    bool over = false;
    auto refresh = [&]() {
        t.merge(sbk[w], sbi[w], lane);
        const float mk = t.key_at(k);
        T = mk == __builtin_inff() ? __builtin_inff() : qs_key_to_a(metric, mk, qi.x) + 2.0005f * eps;
        // A = v (dot), fl(v + |q|^2) (L2), max(0, fl(1 + v)) (cosine): invert
        // with a few ulps of slack (the exact A <= T test follows the prefilter)
        if (!(T < __builtin_inff())) Kt = __builtin_inff();
        else if (metric == DOT) Kt = T;
        else if (metric == L2) Kt = (T - qi.x) + 4.8e-7f * fmaxf(fabsf(T), qi.x);
        else Kt = T < 0.f ? -__builtin_inff() : (T - 1.f) + 4.8e-7f * fmaxf(1.f, fabsf(T));
    };
    auto compact = [&]() {
        int n2 = 0;
        for (int e0 = 0; e0 < nc; e0 += 64) {
            const int e = e0 + lane;
            const float v = e < nc ? cbk[w][e] : __builtin_inff();
            const uint32_t id = e < nc ? cbi[w][e] : 0u;
            const bool in = e < nc && qs_key_to_a(metric, v, qi.x) <= T;
            const uint64_t m = __ballot(in);
            // in place: the wave's reads of this chunk precede its writes, and a
            // write goes to a position <= its read (LDS ops of a wave in order)
            const int pos = n2 + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            if (in) { cbk[w][pos] = v; cbi[w][pos] = id; }
            n2 += __popcll(m);
        }
        nc = n2;
    };
    for (int64_t b0 = 0; b0 < nb; b0 += 64 * U) {
        float v[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const int64_t bb = b0 + j * 64 + lane;
            v[j] = bb < nb ? kr[bb] : __builtin_inff();
        }
        bool any = false;
#pragma unroll
        for (int j = 0; j < U; j++) any |= v[j] < t.thr;
        if (__any(any)) {
#pragma unroll
            for (int j = 0; j < U; j++) t.offer(v[j], (uint32_t)(b0 + j * 64 + lane), sbk[w], sbi[w], lane);
        }
        if (over) continue;
        bool anyc = false;  // one wave vote per chunk: most chunks append nothing
#pragma unroll
        for (int j = 0; j < U; j++) anyc |= v[j] <= Kt;
        if (!__any(anyc)) continue;
#pragma unroll
        for (int j = 0; j < U; j++) {
            if (!__any(v[j] <= Kt)) continue;
            bool in = v[j] <= Kt && v[j] < __builtin_inff() && qs_key_to_a(metric, v[j], qi.x) <= T;
            uint64_t m = __ballot(in);
            if (m == 0) continue;
            int n = __popcll(m);
            if (nc + n > CB) {  // full: tighten T and drop what no longer qualifies
                refresh();
                compact();
                in = in && qs_key_to_a(metric, v[j], qi.x) <= T;
                m = __ballot(in);
                n = __popcll(m);
                if (nc + n > CB) { over = true; break; }
            }
            const int pos = nc + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            if (in) { cbk[w][pos] = v[j]; cbi[w][pos] = (uint32_t)(b0 + j * 64 + lane); }
            nc += n;
        }
    }
    refresh();
    const float mk = t.key_at(k);
    const float M = qs_key_to_a(metric, mk, qi.x);
    if (!over) compact();
    const bool full = over || nc > L;
    if (!full)
        for (int e = lane; e < nc; e += 64) cand[(int64_t)q * L + e] = cbi[w][e];
    if (lane == 0) {
        ncand[q] = full ? L : nc;
        eps_out[q] = eps;
        if (cap_out)
            cap_out[q] = mk == __builtin_inff() ? __builtin_inff() : qs_next_up(M + 1.001f * eps);
        if (t_out) t_out[q] = __builtin_inff();  // no lowered threshold: the 2-eps argument holds
        flags[q] = (full || qi.w != 0.f) ? 2 : 0;
    }
    if (topA) {  // sharded phase 1: this shard's k+1 smallest block-key A values
#pragma unroll
        for (int r = 0; r < RT - 1; r++) {
            const int e = r * 64 + lane;
            if (e <= k) topA[(int64_t)q * (k + 1) + e] = qs_key_to_a(metric, t.key[r], qi.x);
        }
    }
}

// ---------------------------------------------------------------------------
// Split selection for small batches (k_blk_select_f's outputs and candidate
// set).  One wave per query streams ldk keys with a serial latency chain
// (C3, B = 1: 312k keys, 0.73 ms -- a third of the batch); here a query's keys
// are cut into P chunks, one wave each, in three short kernels:
//   k_sel_part     the chunk's k+1 smallest keys (WaveTopL<RT>) -> part[q][p][k+1]
//   k_sel_mid      one wave per query: M = A of the (k+1)-th smallest of the P
//                  lists (= of all keys), eps, T = M + 2.0005 eps, the cap,
//                  topA, flags (non-finite query: 2), ncand = 0
//   k_sel_collect  every chunk again: blocks with A <= T appended through an
//                  atomic cursor (any order: k_blk_exact and the inversion
//                  take any order), more than L -> flag 2, ncand clamped to L
// ---------------------------------------------------------------------------
// a starting threshold for a wave's top-(k+1) list (k + 1 <= 64): `lm` = the
// lane's smallest value (+inf: none); with at least k + 1 lanes holding a
// value, their largest minimum bounds the (k+1)-th smallest from above (those
// minima are k + 1 distinct elements), so anything above it is never kept.
// Returns the offer threshold (values below it pass): next_up of that bound.
__device__ __forceinline__ float wave_kp1_cap(float lm, int k) {
    const bool has = lm < __builtin_inff();
    const int nl = __popcll(__ballot(has));
    float b = has ? lm : -__builtin_inff();
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) b = fmaxf(b, __shfl_xor(b, o));
    return (k + 1 <= 64 && nl >= k + 1) ? qs_next_up(b) : __builtin_inff();
}

template <int RT>
__global__ __launch_bounds__(64) void k_sel_part(const float* __restrict__ key, int64_t ldk, int64_t nb, int k, int P,
                                                 float* __restrict__ part) {
    __shared__ float sbk[64];
    __shared__ uint32_t sbi[64];
    constexpr int U = 16;
    const int p = blockIdx.x, lane = threadIdx.x;
    const int64_t q = blockIdx.y;
    const int64_t per = (nb + P - 1) / P;
    const int64_t b0 = (int64_t)p * per, b1 = b0 + per < nb ? b0 + per : nb;
    const float* kr = key + q * ldk;
    WaveTopL<RT> t;
    {   // a pre-pass over the part (cache-resident on the second read): without
        // a threshold every 64 keys offered forced a merge
        float lm = __builtin_inff();
        for (int64_t c0 = b0; c0 < b1; c0 += 64 * U) {
#pragma unroll
            for (int j = 0; j < U; j++) {
                const int64_t bb = c0 + j * 64 + lane;
                lm = fminf(lm, bb < b1 ? kr[bb] : __builtin_inff());
            }
        }
        t.init(wave_kp1_cap(lm, k));
    }
    for (int64_t c0 = b0; c0 < b1; c0 += 64 * U) {
        float v[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const int64_t bb = c0 + j * 64 + lane;
            v[j] = bb < b1 ? kr[bb] : __builtin_inff();
        }
        bool any = false;
#pragma unroll
        for (int j = 0; j < U; j++) any |= v[j] < t.thr;
        if (!__any(any)) continue;
#pragma unroll
        for (int j = 0; j < U; j++) t.offer(v[j], 0u, sbk, sbi, lane);
    }
    t.merge(sbk, sbi, lane);
#pragma unroll
    for (int r = 0; r < RT - 1; r++) {
        const int e = r * 64 + lane;
        if (e <= k) part[(q * P + p) * (k + 1) + e] = t.key[r];
    }
}

template <int RT>
__global__ __launch_bounds__(64) void k_sel_mid(const float* __restrict__ part, int P, int nq, int k, int metric,
                                                const float4* __restrict__ qinfo, const uint32_t* __restrict__ qsmax,
                                                const uint32_t* __restrict__ maxn2, float gd, float gacc,
                                                int32_t* __restrict__ ncand, int32_t* __restrict__ flags,
                                                float* __restrict__ eps_out, float* __restrict__ Tout,
                                                float* __restrict__ topA, float* __restrict__ cap_out,
                                                uint32_t* __restrict__ list_ctr) {
    __shared__ float sbk[64];
    __shared__ uint32_t sbi[64];
    const int lane = threadIdx.x;
    const int q = blockIdx.x;
    if (list_ctr && q == 0 && lane == 0) {
        list_ctr[1] = 0u;
        list_ctr[3] = 0u;
    }
    const float4 qi = qinfo[q];
    const float eps = qs_eps(metric, qi, qsmax, maxn2, gd, gacc);
    const int n = P * (k + 1);
    const float* pr = part + (int64_t)q * n;
    WaveTopL<RT> t;
    {
        float lm = __builtin_inff();
        for (int i0 = 0; i0 < n; i0 += 64) lm = fminf(lm, i0 + lane < n ? pr[i0 + lane] : __builtin_inff());
        t.init(wave_kp1_cap(lm, k));
    }
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        t.offer(i < n ? pr[i] : __builtin_inff(), 0u, sbk, sbi, lane);
    }
    t.merge(sbk, sbi, lane);
    const float mk = t.key_at(k);
    const float M = qs_key_to_a(metric, mk, qi.x);
    if (lane == 0) {
        ncand[q] = 0;
        eps_out[q] = eps;
        Tout[q] = mk == __builtin_inff() ? __builtin_inff() : M + 2.0005f * eps;
        if (cap_out) cap_out[q] = mk == __builtin_inff() ? __builtin_inff() : qs_next_up(M + 1.001f * eps);
        flags[q] = qi.w != 0.f ? 2 : 0;
    }
    if (topA) {
#pragma unroll
        for (int r = 0; r < RT - 1; r++) {
            const int e = r * 64 + lane;
            if (e <= k) topA[(int64_t)q * (k + 1) + e] = qs_key_to_a(metric, t.key[r], qi.x);
        }
    }
}

__global__ __launch_bounds__(64) void k_sel_collect(const float* __restrict__ key, int64_t ldk, int64_t nb, int P,
                                                    int metric, const float4* __restrict__ qinfo,
                                                    const float* __restrict__ Tq, uint32_t* __restrict__ cand, int L,
                                                    int32_t* __restrict__ ncand, int32_t* __restrict__ flags) {
    const int p = blockIdx.x, lane = threadIdx.x;
    const int64_t q = blockIdx.y;
    const int64_t per = (nb + P - 1) / P;
    const int64_t b0 = (int64_t)p * per, b1 = b0 + per < nb ? b0 + per : nb;
    const float T = Tq[q];
    const float qn2 = qinfo[q].x;
    const float* kr = key + q * ldk;
    for (int64_t bb = b0 + lane; bb - lane < b1; bb += 64) {
        const float v = bb < b1 ? kr[bb] : __builtin_inff();
        const bool in = v < __builtin_inff() && qs_key_to_a(metric, v, qn2) <= T;
        const uint64_t m = __ballot(in);
        if (m == 0) continue;
        int base = 0;
        if (lane == __builtin_ctzll(m)) base = atomicAdd(&ncand[q], __popcll(m));
        base = __shfl(base, __builtin_ctzll(m));
        const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        if (in && pos < L) cand[q * L + pos] = (uint32_t)bb;
        if (in && pos >= L) flags[q] = 2;  // more than L qualify (select_f: nc > L)
    }
}

__global__ void k_sel_clamp(int nq, int L, int32_t* __restrict__ ncand) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nq && ncand[q] > L) ncand[q] = L;
}

// k_blk_gthresh: sharded phase 2, wave per query.  M_g = the (k+1)-th smallest
// of the W shards' k+1 smallest block-key A values (= the (k+1)-th smallest
// key over the whole corpus), eps_max = the largest shard eps of the query.
// The k+1 blocks under M_g each hold a row with E <= M_g + eps_max, so a
// block of this shard with A > M_g + eps_max + eps cannot hold a global
// top-(k+1) row; the candidate list is compacted to the others (any order).
// Queries with flag 2 (their own second pass) or more than 1024 gathered
// values (W * (k+1) > 1024, e.g. k = 127 at 8 ranks) keep the local list:
// still exact, only without the global cut.  cap (phase 1's local cap, valid
// for the shard's own k+1 smallest) is lowered to the global one.
__global__ __launch_bounds__(256) void k_blk_gthresh(const float* __restrict__ topA_all, const float* __restrict__ eps_all,
                                                     int W, int nq, int k, int metric, const float4* __restrict__ qinfo,
                                                     const float* __restrict__ key, int64_t ldk,
                                                     uint32_t* __restrict__ cand, int L,
                                                     int32_t* __restrict__ ncand, const float* __restrict__ eps_own,
                                                     const int32_t* __restrict__ flags, float* __restrict__ cap) {
    __shared__ float sv[4][1024];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int q = blockIdx.x * 4 + w;
    if (q >= nq || flags[q] == 2) return;
    const int K1 = k + 1;
    const int n = W * K1;
    if (n > 1024) return;
    float emax = 0.f;
    for (int i = lane; i < n; i += 64) {
        const int r = i / K1, e = i % K1;
        sv[w][i] = topA_all[((int64_t)r * nq + q) * K1 + e];
    }
    for (int r = lane; r < W; r += 64) emax = fmaxf(emax, eps_all[(int64_t)r * nq + q]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) emax = fmaxf(emax, __shfl_xor(emax, o));
    wave_sync_lds();
    // M_g: a value v with #(< v) <= k < #(<= v)
    float M = __builtin_inff();
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        const float v = i < n ? sv[w][i] : __builtin_inff();
        int lt = 0, le = 0;
        for (int j = 0; j < n; j++) {
            const float u = sv[w][j];
            lt += u < v ? 1 : 0;
            le += u <= v ? 1 : 0;
        }
        const uint64_t hit = __ballot(i < n && lt <= k && k < le);
        if (hit) { M = __shfl(v, __builtin_ctzll(hit)); break; }
    }
    if (!(M < __builtin_inff())) return;
    const float T = M + 1.0005f * (emax + eps_own[q]);
    const int nc = ncand[q];
    const float qn2 = qinfo[q].x;
    int keep = 0;
    uint32_t* cq = cand + (int64_t)q * L;
    for (int e0 = 0; e0 < nc; e0 += 64) {  // compaction in place (any list order)
        const int e = e0 + lane;
        const uint32_t b = e < nc ? cq[e] : 0u;
        const bool in = e < nc && qs_key_to_a(metric, key[(int64_t)q * ldk + b], qn2) <= T;
        const uint64_t m = __ballot(in);
        const int pos = keep + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        if (in) cq[pos] = b;
        keep += __popcll(m);
    }
    if (lane == 0) {
        ncand[q] = keep;
        // the k+1 blocks under M_g each hold a row with E <= M_g + eps_max: the
        // global (k+1)-th smallest exact distance is below this cap, so the
        // capped exact pass (k_blk_exact) may skip every row at or above it
        if (cap) cap[q] = fminf(cap[q], qs_next_up(M + 1.001f * emax));
    }
}

// byte offset of int8 column c of row `row` in a tiled int8 plane of dpb8
// columns: 256-row tiles of 32-byte column chunks (the bf16 plane's tiling,
// two int8 columns per bf16 element)
__host__ __device__ __forceinline__ int64_t q8_plane_byte(int64_t row, int c, int dpb8) {
    return ((row >> 8) * (int64_t)(dpb8 >> 5) + (c >> 5)) * 8192 + ((row & 255) << 5) + (c & 31);
}

// ---------------------------------------------------------------------------
// row filter helpers (k_blk_exact, k_blk_replay)
// ---------------------------------------------------------------------------
constexpr int QS_FILT_DPB = 1536;  // the widest block-key plane (k_qs_blockkey_w4)
constexpr int Q8_FILT_DPB = 3072;  // the widest int8 plane (k_q8_blockkey_cp)

// S = sum_c bf16(q)_c * x_h,c of one stored row from the tiled bf16 plane
// (lane per row: the plane interleaves 256 rows per 16-column chunk, so the
// lanes' 32-byte reads are contiguous).  Two alternating fp32 accumulators:
// the error is within gamma_{dpb+2} sum|terms| (gacc_r of the callers).
__device__ __forceinline__ float plane_dot(const uint16_t* __restrict__ Xb, int64_t row, int dpb, const float* sqh) {
    float s0 = 0.f, s1 = 0.f;
#pragma unroll 8
    for (int c = 0; c < dpb; c += 16) {
        const uint4* xp = reinterpret_cast<const uint4*>(Xb + bf3_plane_index(row, c, dpb));
        const uint4 v0 = xp[0], v1 = xp[1];
        const float4* qp = reinterpret_cast<const float4*>(sqh + c);
        const float4 a0 = qp[0], a1 = qp[1], a2 = qp[2], a3 = qp[3];
        s0 = fmaf(__uint_as_float(v0.x << 16), a0.x, s0); s1 = fmaf(__uint_as_float(v0.x & 0xFFFF0000u), a0.y, s1);
        s0 = fmaf(__uint_as_float(v0.y << 16), a0.z, s0); s1 = fmaf(__uint_as_float(v0.y & 0xFFFF0000u), a0.w, s1);
        s0 = fmaf(__uint_as_float(v0.z << 16), a1.x, s0); s1 = fmaf(__uint_as_float(v0.z & 0xFFFF0000u), a1.y, s1);
        s0 = fmaf(__uint_as_float(v0.w << 16), a1.z, s0); s1 = fmaf(__uint_as_float(v0.w & 0xFFFF0000u), a1.w, s1);
        s0 = fmaf(__uint_as_float(v1.x << 16), a2.x, s0); s1 = fmaf(__uint_as_float(v1.x & 0xFFFF0000u), a2.y, s1);
        s0 = fmaf(__uint_as_float(v1.y << 16), a2.z, s0); s1 = fmaf(__uint_as_float(v1.y & 0xFFFF0000u), a2.w, s1);
        s0 = fmaf(__uint_as_float(v1.z << 16), a3.x, s0); s1 = fmaf(__uint_as_float(v1.z & 0xFFFF0000u), a3.y, s1);
        s0 = fmaf(__uint_as_float(v1.w << 16), a3.z, s0); s1 = fmaf(__uint_as_float(v1.w & 0xFFFF0000u), a3.w, s1);
    }
    return s0 + s1;
}

// A_row of one stored row: the block key's formula with plane_dot's S
template <int METRIC>
__device__ __forceinline__ float plane_a(const uint16_t* __restrict__ Xb, const float* __restrict__ xn2, int64_t row,
                                         int dpb, const float* sqh, float qn2) {
    const float S = plane_dot(Xb, row, dpb, sqh);
    const float kv = METRIC == L2 ? fmaf(-2.f, S, xn2[row]) : -S;
    return qs_key_to_a(METRIC == COSINE ? COSINE : METRIC == DOT ? DOT : L2, kv, qn2);
}

// The int8-plane form (q8_kernels.hip layout: 256-row tiles of 32-byte
// column chunks, lane per row reads contiguous 1 KiB per chunk): the exact
// int32 dot of the row's codes with the query's (sq8: dpb8 / 4 packed words
// in LDS), v_dot4_i32_i8.
__device__ __forceinline__ int plane_dot_q8(const unsigned char* __restrict__ X8, int64_t row, int dpb8,
                                            const uint32_t* sq8) {
    int acc = 0;
    const unsigned char* base = X8 + (row >> 8) * (int64_t)dpb8 * 256 + ((row & 255) << 5);
#pragma unroll 4
    for (int c = 0; c < dpb8; c += 32) {
        const uint4* xp = reinterpret_cast<const uint4*>(base + (int64_t)(c >> 5) * 8192);
        const uint4 v0 = xp[0], v1 = xp[1];
        const uint4* qp = reinterpret_cast<const uint4*>(sq8 + (c >> 2));
        const uint4 a0 = qp[0], a1 = qp[1];
        acc = __builtin_amdgcn_sdot4((int)v0.x, (int)a0.x, acc, false);
        acc = __builtin_amdgcn_sdot4((int)v0.y, (int)a0.y, acc, false);
        acc = __builtin_amdgcn_sdot4((int)v0.z, (int)a0.z, acc, false);
        acc = __builtin_amdgcn_sdot4((int)v0.w, (int)a0.w, acc, false);
        acc = __builtin_amdgcn_sdot4((int)v1.x, (int)a1.x, acc, false);
        acc = __builtin_amdgcn_sdot4((int)v1.y, (int)a1.y, acc, false);
        acc = __builtin_amdgcn_sdot4((int)v1.z, (int)a1.z, acc, false);
        acc = __builtin_amdgcn_sdot4((int)v1.w, (int)a1.w, acc, false);
    }
    return acc;
}

// A_row from the int8 plane: k_q8_blockkey's key formula for one row
// (S = fl(fl(sq sb) float(dot)); L2 fl(xnorm2 - 2 S) in one fma)
template <int METRIC>
__device__ __forceinline__ float plane_a_q8(const unsigned char* __restrict__ X8, const float* __restrict__ sb8,
                                            const float* __restrict__ xn2, int64_t row, int dpb8, const uint32_t* sq8,
                                            float sq, float qn2) {
    const float s = sq * sb8[row >> 5];
    const float Sf = (float)plane_dot_q8(X8, row, dpb8, sq8);
    const float kv = METRIC == L2 ? fmaf(-2.f * s, Sf, xn2[row]) : -(s * Sf);
    return qs_key_to_a(METRIC == COSINE ? COSINE : METRIC == DOT ? DOT : L2, kv, qn2);
}

// Reference-order distances of the rows of the lanes with `need` (row = the
// lane's stored row), 8 lanes per row (exact_dist8) in passes of 8 rows;
// slot[0..63] is this wave's LDS scratch.  Every lane of the wave must call.
template <int METRIC>
__device__ __forceinline__ float exact8_compact(const float* __restrict__ qv, const float* __restrict__ X, int dpad,
                                                int d, int64_t row, bool need, int lane, float* slot) {
    const uint64_t nm = __ballot(need);
    const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(nm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nm, 0));
    const int cnt = __popcll(nm);
    float dist = 0.f;
    if (cnt == 0) return dist;
    if (need) slot[rank] = __int_as_float((int)row);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int p0 = 0; p0 < cnt; p0 += 8) {
        const int gsel = p0 + (lane >> 3);
        const int64_t rw = (int64_t)__float_as_int(slot[gsel < cnt ? gsel : 0]);  // spare groups repeat the list's first row
        const float* xp1[1] = {X + rw * dpad};
        float dv[1];
        exact_dist8<METRIC, 1>(qv, xp1, d, lane & 7, dv);
        const float dg = __shfl(dv[0], ((rank - p0) & 7) * 8);
        if (need && rank >= p0 && rank < p0 + 8) dist = dg;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    return dist;
}

// k_blk_exact<R, METRIC, VARIANT, EB>: one workgroup (4 waves) per query over its
// candidate blocks (each wave two blocks per pass: lanes 0-31 and 32-63, lane
// = row); EB: the distances come from k_exact_bm (ebuf).  Reference-order SingleDist of every valid row, top-(k+1) by
// (distance, id) per wave, merged by wave 0; proof = the first min(k+1, n)
// are strictly increasing (the reference heap then holds exactly the k
// smallest and extractHeap returns them ascending).
template <int R, int METRIC, int VARIANT, bool EB>
__global__ __launch_bounds__(256) void k_blk_exact(const float* __restrict__ X, int dpad, const uint32_t* __restrict__ valid,
                                                   int64_t nrows, const float* __restrict__ Qn, int d,
                                                   const uint32_t* __restrict__ cand, const int32_t* __restrict__ ncand,
                                                   int nq, int k, int kout, uint64_t id_base, uint64_t* __restrict__ out_ids,
                                                   float* __restrict__ out_d, int32_t* __restrict__ out_n,
                                                   int32_t* __restrict__ flags, const int32_t* __restrict__ qlist,
                                                   const uint32_t* __restrict__ qcount,
                                                   const float* __restrict__ ebuf, int64_t ldE,
                                                   const float* __restrict__ cap, const float4* __restrict__ qinfo,
                                                   const uint16_t* __restrict__ Xb, int dpb, const float* __restrict__ xn2,
                                                   const uint32_t* __restrict__ qsmax, const uint32_t* __restrict__ maxn2,
                                                   float gd, float gacc_r, const Q8Filter q8f,
                                                   const uint32_t* __restrict__ fmask, int64_t vq = 0,
                                                   const float* __restrict__ tq = nullptr,
                                                   const float* __restrict__ qeps = nullptr) {
    constexpr int L = 64 * (R - 1);
    __shared__ float sbk[4][64];
    __shared__ uint32_t sbi[4][64];
    __shared__ float sslot[4][64];
    __shared__ __attribute__((aligned(16))) float sqh[EB ? 4 : QS_FILT_DPB];
    __shared__ __attribute__((aligned(16))) uint32_t sq8[EB ? 4 : Q8_FILT_DPB / 4];
    __shared__ float lk[3][L];
    __shared__ uint32_t lid[3][L];
    __shared__ int snv[4];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    int q = blockIdx.x;
    if (qlist) {
        if ((uint32_t)q >= qcount[1]) return;
        q = qlist[q];
    }
    if (q >= nq) return;
    const uint32_t* vrow = vq ? valid + (int64_t)q * vq : valid;  // per-query allow bitmaps (vq words each)
    if (flags[q]) return;  // overflowed selection: the replay resolves it
    const int nc = ncand[q];
    const float* qv = Qn + (int64_t)q * dpad;
    const int li = lane & 31, lh = lane >> 5;
    const bool coop = exact8_ok<METRIC, VARIANT>(d);
    // row filter (capped exact pass, finite query): a row whose plane bound
    // A_row - eps_r reaches the cap has an exact distance >= cap, which the
    // list never keeps; only the others get the reference-order distance
    const float4 qi = qinfo[q];
    // int8-plane row bound (the keys were int8): half the plane bytes per row;
    // above 1536 dims the only plane
    const bool f8 = !EB && q8f.X8 != nullptr && cap != nullptr && qi.w == 0.f && q8f.dpb8 <= Q8_FILT_DPB;
    const bool filt = f8 || (!EB && Xb != nullptr && cap != nullptr && qi.w == 0.f && dpb <= QS_FILT_DPB);
    float eps_r = 0.f, capq = __builtin_inff(), sqs = 0.f;
    // the block-major int8 filter (k_q8_filt_bm) already decided each row
    const bool fm = f8 && fmask != nullptr;
    if (fm) {
        capq = cap[q];
    } else if (f8) {
        for (int c4 = 4 * threadIdx.x; c4 < q8f.dpb8; c4 += 1024)
            sq8[c4 >> 2] = *reinterpret_cast<const uint32_t*>(q8f.Q8 + q8_plane_byte(q, c4, q8f.dpb8));
        eps_r = qs_eps(METRIC == COSINE ? COSINE : METRIC == DOT ? DOT : L2, q8f.qinfo8[q], q8f.qmax8, maxn2, gd,
                       q8f.gacc8);
        sqs = q8f.qscale[q];
        capq = cap[q];
        __syncthreads();
    } else if (filt) {
        for (int c = threadIdx.x; c < dpb; c += 256) sqh[c] = (float)(__bf16)(c < d ? qv[c] : 0.f);
        eps_r = qs_eps(METRIC == COSINE ? COSINE : METRIC == DOT ? DOT : L2, qi, qsmax, maxn2, gd, gacc_r);
        capq = cap[q];
        __syncthreads();
    }
    WaveTopL<R> t;
    t.init(cap ? cap[q] : __builtin_inff());  // only the k+1 smallest are used: nothing above cap
    int nvalid = 0;
    for (int j0 = 2 * w; j0 < nc; j0 += 8) {
        const int j = j0 + lh;
        bool ok = false;
        int64_t row = 0;
        if (j < nc) {
            row = (int64_t)cand[(int64_t)q * L + j] * 32 + li;
            ok = row < nrows && ((vrow[row >> 5] >> (row & 31)) & 1u);
        }
        float e = __builtin_inff();
        if (EB) {  // its own instantiation: the distance code's registers stay out of the read-back form
            if (ok) e = ebuf[(int64_t)q * ldE + j * 32 + li];
        } else if (filt) {
            const bool need = fm ? ok && ((fmask[(int64_t)q * L + (j < nc ? j : 0)] >> li) & 1u)
                                 : ok && (f8 ? plane_a_q8<METRIC>(q8f.X8, q8f.sb8, xn2, row, q8f.dpb8, sq8, sqs, qi.x)
                                             : plane_a<METRIC>(Xb, xn2, row, dpb, sqh, qi.x)) - eps_r < capq;
            const float dl = coop ? exact8_compact<METRIC>(qv, X, dpad, d, row, need, lane, sslot[w])
                                  : need ? exact_dist<METRIC, VARIANT>(qv, X + row * dpad, d) : 0.f;
            if (need) e = dl;
        } else if (coop) {  // 8 lanes per row, rows 8g + (lane >> 3) of the pass
            const float* xp[8];
#pragma unroll
            for (int g = 0; g < 8; g++) {
                const int r = 8 * g + (lane >> 3);
                const int jg = r >= 32 && j0 + 1 < nc ? j0 + 1 : j0;
                const int64_t rw = (int64_t)cand[(int64_t)q * L + jg] * 32 + (r & 31);
                xp[g] = X + (rw < nrows ? rw : 0) * dpad;
            }
            const float dl = exact8_rows64<METRIC>(qv, xp, d, lane);
            if (ok) e = dl;
        } else if (ok) {
            e = exact_dist<METRIC, VARIANT>(qv, X + row * dpad, d);
        }
        nvalid += __popcll(__ballot(ok));
        t.offer(ok ? e : __builtin_inff(), ok ? (uint32_t)row : NO_ID, sbk[w], sbi[w], lane);
    }
    t.merge(sbk[w], sbi[w], lane);
    if (w > 0) {
#pragma unroll
        for (int r = 0; r < R - 1; r++) {
            lk[w - 1][r * 64 + lane] = t.key[r];
            lid[w - 1][r * 64 + lane] = t.id[r];
        }
    }
    if (lane == 0) snv[w] = nvalid;
    __syncthreads();
    if (w > 0) return;
    // wave 0: merge the other waves' lists into its own
    for (int w2 = 0; w2 < 3; w2++)
        for (int r = 0; r < R - 1; r++) t.offer(lk[w2][r * 64 + lane], lid[w2][r * 64 + lane], sbk[0], sbi[0], lane);
    t.merge(sbk[0], sbi[0], lane);
    nvalid = snv[0] + snv[1] + snv[2] + snv[3];
    // with a finite cap the list holds exactly the rows below it (the others
    // were skipped or rejected): a shard's cap in the sharded phase 2 may leave
    // fewer than k+1 (the global top-(k+1) rows are all below it)
    if (cap && cap[q] < __builtin_inff()) {
        int nb = 0;
#pragma unroll
        for (int r = 0; r < R - 1; r++) nb += __popcll(__ballot(t.key[r] < __builtin_inff()));
        nvalid = nb < nvalid ? nb : nvalid;
    }
    const int m = (k + 1) < nvalid ? (k + 1) : nvalid;
    bool inc = true;
#pragma unroll
    for (int r = 0; r < R - 1; r++) {
        const float up = __shfl_up(t.key[r], 1);
        const float wrap = (r > 0) ? __shfl(t.key[r > 0 ? r - 1 : 0], 63) : 0.f;
        const float pv = lane == 0 ? wrap : up;
        const int e = r * 64 + lane;
        if (e >= 1 && e < m && !(t.key[r] > pv)) inc = false;
    }
    inc = __all(inc);
    // per-query allow bitmaps (vq): the keys came from their union, so the
    // k+1 blocks under M need not hold k+1 of this query's rows.  Rows of
    // unlisted blocks are > T - eps (A > T there, E >= A - eps): the list is
    // complete when it holds k+1 rows and its (k+1)-th is <= T - eps (the
    // rounded difference one ulp down: below the exact one); else the replay
    // decides.  T = inf: every block with a union row is listed.
    // The same test for a list whose threshold was lowered below the L-th key
    // (k_blk_select: more blocks than the list qualified).
    if (tq && inc && tq[q] < __builtin_inff())
        inc = nvalid >= k + 1 && t.key_at(k) <= qs_next_down(tq[q] - qeps[q]);
    if (!inc) {
        if (lane == 0) flags[q] = 1;
        return;
    }
    const int nout = kout < nvalid ? kout : nvalid;
#pragma unroll
    for (int r = 0; r < R - 1; r++) {
        const int e = r * 64 + lane;
        if (e < nout) {
            out_ids[(int64_t)q * kout + e] = id_base + t.id[r];
            out_d[(int64_t)q * kout + e] = t.key[r];
        }
    }
    if (lane == 0) out_n[q] = nout;
}

// ---------------------------------------------------------------------------
// Block-major exact distances (rows of up to 508 floats).  Many queries list
// the same candidate block (C2: ~60 per block); reading the block once per
// listing query makes k_blk_exact bandwidth-bound on re-reads.  The candidate
// lists are inverted per 32-row block (k_inv_count / k_inv_scan /
// k_inv_scatter: pairs (query << 9 | list position)), k_exact_bm stages each
// listed block's rows in LDS once and writes the reference-order exact
// distance of every row for every listing query to ebuf[q][j*32 + row];
// k_blk_exact then reads them instead of recomputing (same values, same
// selection and proof).  Order of pairs within a block does not matter: every
// pair writes its own slot.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_inv_count(const uint32_t* __restrict__ cand, const int32_t* __restrict__ ncand,
                                                   const int32_t* __restrict__ flags, int nq, int L,
                                                   uint32_t* __restrict__ cnt) {
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq || flags[q]) return;
    const int nc = ncand[q];
    for (int j = lane; j < nc; j += 64) atomicAdd(&cnt[cand[(int64_t)q * L + j]], 1u);
}

// exclusive prefix of cnt[0..nb) -> off[0..nb]; cnt stays (the scatter counts
// it back down to 0, so the next batch starts from a zeroed array without a
// fill).  Two passes over chunks of 4096 counts: k_inv_part sums each chunk
// (coalesced), k_inv_scan adds the sums of the chunks before its own and
// scans the chunk (4 contiguous counts per thread + a workgroup scan).
constexpr int INV_CHUNK = 4096;
__global__ __launch_bounds__(1024) void k_inv_part(const uint32_t* __restrict__ cnt, int64_t nb,
                                                   uint32_t* __restrict__ part) {
    __shared__ uint32_t ws[16];
    const int64_t base = (int64_t)blockIdx.x * INV_CHUNK;
    uint32_t s = 0;
    for (int i = threadIdx.x; i < INV_CHUNK; i += 1024) s += base + i < nb ? cnt[base + i] : 0u;
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < 16; w++) t += ws[w];
        part[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(1024) void k_inv_scan(const uint32_t* __restrict__ cnt, int64_t nb,
                                                   const uint32_t* __restrict__ part, uint32_t* __restrict__ off) {
    __shared__ uint32_t sc[1024];
    __shared__ uint32_t ws[16];
    const int t = threadIdx.x;
    // the chunks before this one
    uint32_t pre = 0;
    for (int c = t; c < (int)blockIdx.x; c += 1024) pre += part[c];
    for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o);
    if ((t & 63) == 0) ws[t >> 6] = pre;
    const int64_t base = (int64_t)blockIdx.x * INV_CHUNK + 4 * t;
    uint32_t v[4], s = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        v[i] = base + i < nb ? cnt[base + i] : 0u;
        s += v[i];
    }
    sc[t] = s;
    __syncthreads();
    uint32_t run = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) run += ws[w];
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
        const uint32_t x = t >= o ? sc[t - o] : 0u;
        __syncthreads();
        sc[t] += x;
        __syncthreads();
    }
    run += sc[t] - s;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (base + i < nb) off[base + i] = run;
        run += v[i];
    }
    if (base < nb && base + 4 >= nb) off[nb] = run;  // the thread holding the last count
}

__global__ __launch_bounds__(256) void k_inv_scatter(const uint32_t* __restrict__ cand, const int32_t* __restrict__ ncand,
                                                     const int32_t* __restrict__ flags, int nq, int L,
                                                     const uint32_t* __restrict__ off, uint32_t* __restrict__ cur,
                                                     uint32_t* __restrict__ pairs) {
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq || flags[q]) return;
    const int nc = ncand[q];
    for (int j = lane; j < nc; j += 64) {
        const uint32_t b = cand[(int64_t)q * L + j];
        pairs[off[b] + atomicSub(&cur[b], 1u) - 1u] = ((uint32_t)q << 9) | (uint32_t)j;
    }
}

// one workgroup per 32-row block; LDS rows at stride dpad + 4 floats (16-byte
// aligned; lane = row reads conflict-free in 16-lane groups)
template <int METRIC, int VARIANT>
__global__ __launch_bounds__(256) void k_exact_bm(const float* __restrict__ X, int dpad, int64_t nrows,
                                                  const float* __restrict__ Qn, int d, const uint32_t* __restrict__ off,
                                                  const uint32_t* __restrict__ pairs, int64_t ldE,
                                                  float* __restrict__ ebuf) {
    extern __shared__ float4 rows4[];
    const int64_t b = blockIdx.x;
    const uint32_t p0 = off[b], p1 = off[b + 1];
    if (p0 == p1) return;
    const int t = threadIdx.x;
    const int d4 = dpad / 4, s4 = d4 + 1;  // float4s per row in global / in LDS
    const float4* X4 = reinterpret_cast<const float4*>(X);
    for (int i = t; i < 32 * d4; i += 256) {
        const int r = i / d4, c = i - r * d4;
        const int64_t row = b * 32 + r;
        rows4[r * s4 + c] = row < nrows ? X4[row * d4 + c] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    const int lane = t & 63, w = t >> 6;
    const int li = lane & 31, lh = lane >> 5;
    const float* xr = reinterpret_cast<const float*>(rows4 + li * s4);
    for (uint32_t p = p0 + 2 * w + lh; p < p1; p += 8) {
        const uint32_t pr = pairs[p];
        const int64_t q = pr >> 9;
        const int j = (int)(pr & 511u);
        ebuf[q * ldE + j * 32 + li] = exact_dist<METRIC, VARIANT>(Qn + q * dpad, xr, d);
    }
}

// Block-major int8 row filter of the capped exact pass (int8 block keys,
// int8 rows of up to 1536 columns).  Candidate-major, every listing query
// re-reads its candidate block's codes from HBM (C3: ~920k listings over
// ~312k distinct blocks per 8192-query batch, 22.6 GB); here one workgroup per
// listed 32-row block (the k_inv_* inversion) stages the block's codes in LDS
// once and gives every listing (query, list position) the 32 rows' survivor
// mask: bit r = row r is valid and A_row - eps_r < cap(q), with A_row the
// same float arithmetic as plane_a_q8 (so the same rows survive).  LDS:
// [chunk][32 rows][32 B] block codes, then per wave two listings' query codes.
template <int METRIC>
__global__ __launch_bounds__(256) void k_q8_filt_bm(const Q8Filter f, const float* __restrict__ xn2,
                                                    const uint32_t* __restrict__ valid, int64_t nrows,
                                                    const uint32_t* __restrict__ off, const uint32_t* __restrict__ pairs,
                                                    int L, const float* __restrict__ cap,
                                                    const float4* __restrict__ qinfo,
                                                    const uint32_t* __restrict__ maxn2, float gd,
                                                    uint32_t* __restrict__ fmask) {
    extern __shared__ uint4 fsm4[];
    const int64_t b = blockIdx.x;
    const uint32_t p0 = off[b], p1 = off[b + 1];
    if (p0 == p1) return;
    const int t = threadIdx.x;
    const int nch = f.dpb8 >> 5;  // 32-byte column chunks
    // the block's rows are 1 KiB contiguous per chunk in the tiled plane
    const uint4* src = reinterpret_cast<const uint4*>(f.X8 + (b >> 3) * (int64_t)f.dpb8 * 256 + (b & 7) * 1024);
    for (int i = t; i < nch * 64; i += 256) fsm4[i] = src[(int64_t)(i >> 6) * 512 + (i & 63)];
    const int lane = t & 63, w = t >> 6, li = lane & 31, lh = lane >> 5;
    uint4* qs = fsm4 + nch * 64 + (w * 2 + lh) * nch * 2;
    const int64_t row = b * 32 + li;
    const bool okr = row < nrows && ((valid[row >> 5] >> li) & 1u);
    const float sbk = f.sb8[b];
    const float x2 = METRIC == L2 ? xn2[row] : 0.f;
    __syncthreads();
    for (uint32_t pb = p0 + 2 * w; pb < p1; pb += 8) {
        const uint32_t p = pb + lh;
        const bool has = p < p1;
        const uint32_t pr = pairs[has ? p : pb];
        const int64_t q = pr >> 9;
        const int j = (int)(pr & 511u);
        for (int i = li; i < nch * 2; i += 32)
            qs[i] = *reinterpret_cast<const uint4*>(f.Q8 + ((q >> 8) * nch + (i >> 1)) * 8192 + (q & 255) * 32 +
                                                    (i & 1) * 16);
        wave_sync_lds();
        int acc = 0;
        for (int c = 0; c < nch; c++) {
            const uint4 v0 = fsm4[c * 64 + li * 2], v1 = fsm4[c * 64 + li * 2 + 1];
            const uint4 a0 = qs[2 * c], a1 = qs[2 * c + 1];
            acc = __builtin_amdgcn_sdot4((int)v0.x, (int)a0.x, acc, false);
            acc = __builtin_amdgcn_sdot4((int)v0.y, (int)a0.y, acc, false);
            acc = __builtin_amdgcn_sdot4((int)v0.z, (int)a0.z, acc, false);
            acc = __builtin_amdgcn_sdot4((int)v0.w, (int)a0.w, acc, false);
            acc = __builtin_amdgcn_sdot4((int)v1.x, (int)a1.x, acc, false);
            acc = __builtin_amdgcn_sdot4((int)v1.y, (int)a1.y, acc, false);
            acc = __builtin_amdgcn_sdot4((int)v1.z, (int)a1.z, acc, false);
            acc = __builtin_amdgcn_sdot4((int)v1.w, (int)a1.w, acc, false);
        }
        const float eps_r = qs_eps(METRIC == COSINE ? COSINE : METRIC == DOT ? DOT : L2, f.qinfo8[q], f.qmax8, maxn2,
                                   gd, f.gacc8);
        const float s = f.qscale[q] * sbk;
        const float Sf = (float)acc;
        const float kv = METRIC == L2 ? fmaf(-2.f * s, Sf, x2) : -(s * Sf);
        const float A = qs_key_to_a(METRIC == COSINE ? COSINE : METRIC == DOT ? DOT : L2, kv, qinfo[q].x);
        const uint64_t m = __ballot(okr && A - eps_r < cap[q]);
        if (has && li == 0) fmask[q * L + j] = (uint32_t)(m >> (32 * lh));
        wave_sync_lds();  // the next listings' codes overwrite qs
    }
}

// flagged queries -> list (order irrelevant: every listed query is handled
// independently); want = 0: every nonzero flag, else flags == want.
// counters[0] += count, counters[1] = count (this batch)
__global__ void k_flag_list(const int32_t* __restrict__ flags, int nq, int32_t* __restrict__ qlist,
                            uint32_t* __restrict__ counters, int want) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const bool f = q < nq && (want ? flags[q] == want : flags[q] != 0);
    const uint64_t m = __ballot(f);
    if (m == 0) return;
    const int lane = threadIdx.x & 63;
    uint32_t base = 0;
    if (lane == __builtin_ctzll(m)) {
        base = atomicAdd(&counters[1], (uint32_t)__popcll(m));
        atomicAdd(&counters[0], (uint32_t)__popcll(m));
    }
    base = __shfl(base, __builtin_ctzll(m));
    if (f) qlist[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0))] = q;
}

// k_blk_replay<METRIC, VARIANT>: the reference heap over the id-ordered scan
// (flat/index.go:578-688, priorityqueue/queue.go:58-198) for listed queries,
// one wave each.  A 32-row block is visited while the heap is short or
// top > A_block - eps (a lower bound of every row's exact distance); a
// skipped block cannot pass insertToHeap's `top.Dist > distance` for any row.
// Queries with non-finite values visit every block.  Blocks are taken two at
// a time (lanes 0-31, 32-63), inserted by lane 0 in row order.
// Row filter (Xb != null, finite query): a visited row's approximate distance
// A_row from the bf16 planes (the block key's formula with S summed per lane,
// error bound eps_row = qs_eps with gacc_r for that summation) is a lower
// bound A_row - eps_row of its exact distance; only rows with
// top > A_row - eps_row (or a short heap) get the reference-order distance.
// A rejected row cannot pass insertToHeap's test, so the heap sees the same
// insertions; the planes are half the fp32 bytes (C2: most visited rows are
// rejected).
// DBG = 1 (option replay_dbg, diagnostics only): per-wave clock totals of the key
// scan, the exact distances and the heap, printed for the first listed queries
template <int METRIC, int VARIANT, int DBG = 0>
__global__ __launch_bounds__(64) void k_blk_replay(const float* __restrict__ key, int64_t ldk, int64_t nb,
                                                   const float* __restrict__ eps_q, const float4* __restrict__ qinfo,
                                                   const float* __restrict__ X, int dpad, const uint32_t* __restrict__ valid,
                                                   int64_t nrows, const float* __restrict__ Qn, int d,
                                                   const int32_t* __restrict__ qlist, const uint32_t* __restrict__ counters,
                                                   int nlist, int k, int kout, uint64_t id_base,
                                                   uint64_t* __restrict__ out_ids, float* __restrict__ out_d,
                                                   int32_t* __restrict__ out_n, const uint64_t* __restrict__ in_ids,
                                                   const float* __restrict__ in_d, const int32_t* __restrict__ in_len,
                                                   int extract, int by_list, const uint16_t* __restrict__ Xb, int dpb,
                                                   const float* __restrict__ xn2, const uint32_t* __restrict__ qsmax,
                                                   const uint32_t* __restrict__ maxn2, float gd, float gacc_r, int64_t vq = 0) {
    // dynamic LDS: [k] heap records (PHeap) | [64] f32 | len (16 B) | [RU * 64] keys | [dpb] bf16(q) as f32
    extern __shared__ __attribute__((aligned(16))) unsigned char rsm[];
    HeapRec* hr = reinterpret_cast<HeapRec*>(rsm);
    float* s_d = reinterpret_cast<float*>(hr + k);
    int* s_len = reinterpret_cast<int*>(s_d + 64);
    const int lane = threadIdx.x;
    const int li_ = blockIdx.x;  // list position
    if (counters ? (uint32_t)li_ >= counters[1] : li_ >= nlist) return;
    const int q = qlist[li_];
    const uint32_t* vrow = vq ? valid + (int64_t)q * vq : valid;  // per-query allow bitmaps (vq words each)
    const int metric = METRIC == COSINE ? COSINE : METRIC == DOT ? DOT : L2;
    const float4 qi = qinfo[q];
    const bool noskip = qi.w != 0.f;
    const float eps = eps_q[q];
    const float* kr = key + (int64_t)q * ldk;
    const float* qv = Qn + (int64_t)q * dpad;
    const int li = lane & 31, lh = lane >> 5;
    const bool coop = exact8_ok<METRIC, VARIANT>(d);
    // the heap handed over by the previous shard (layout order), or empty
    int len_in = in_len ? in_len[by_list ? li_ : q] : 0;
    len_in = len_in < 0 ? 0 : len_in > k ? k : len_in;
    for (int i = lane; i < len_in; i += 64)
        hr[i] = hr_make(in_ids[(int64_t)(by_list ? li_ : q) * k + i], in_d[(int64_t)(by_list ? li_ : q) * k + i]);
    if (lane == 0) *s_len = len_in;
    __syncthreads();
    // block keys in rounds of 64 * RU: all loads of a round in flight at once,
    // parked in LDS; a round with no visitable block is skipped whole
    constexpr int RU = 16;
    float* skey = s_d + 64 + 4;  // [RU * 64]
    const bool filt = Xb != nullptr && !noskip;
    float* sqh = skey + RU * 64;  // [dpb]: bf16(q) (k_query_split's rounding), widened
    float eps_r = 0.f;
    if (filt) {
        for (int c = lane; c < dpb; c += 64) sqh[c] = (float)(__bf16)(c < d ? qv[c] : 0.f);
        eps_r = qs_eps(metric, qi, qsmax, maxn2, gd, gacc_r);
        __syncthreads();
    }
    long long t_dist = 0, t_heap = 0, t_all = DBG ? clock64() : 0;
    int n_vis = 0, n_ins = 0;
    for (int64_t r0 = 0; r0 < nb; r0 += 64 * RU) {
        float kvr[RU];
#pragma unroll
        for (int u = 0; u < RU; u++) {
            const int64_t bb = r0 + u * 64 + lane;
            kvr[u] = bb < nb ? kr[bb] : __builtin_inff();
        }
        {
            const int len0 = *s_len;
            const float top0 = len0 > 0 ? hr[0].d : 0.f;
            bool any = false;
#pragma unroll
            for (int u = 0; u < RU; u++) {
                const int64_t bb = r0 + u * 64 + lane;
                const bool has = bb < nb && (noskip || kvr[u] < __builtin_inff());
                const float lb = noskip ? -__builtin_inff() : qs_key_to_a(metric, kvr[u], qi.x) - eps;
                any |= has && (len0 < k || top0 > lb);
                skey[u * 64 + lane] = kvr[u];
            }
            if (!__any(any)) continue;
        }
    for (int64_t b0 = r0; b0 < r0 + 64 * RU && b0 < nb; b0 += 64) {
        const int64_t bb = b0 + lane;
        float lb = __builtin_inff();
        bool has = false;
        const uint32_t vwb = bb < nb && bb * 32 < nrows ? vrow[bb] : 0u;  // the group's valid words (nb may pass the bitmap)
        if (bb < nb) {
            const float kv = skey[(b0 - r0) + lane];
            has = noskip || kv < __builtin_inff();
            lb = noskip ? -__builtin_inff() : qs_key_to_a(metric, kv, qi.x) - eps;
        }
        int len = *s_len;
        float top = len > 0 ? hr[0].d : 0.f;
        uint64_t bmask = __ballot(has && (len < k || top > lb));
        while (bmask) {
            // next one or two blocks still able to insert under the current top
            len = *s_len;
            top = len > 0 ? hr[0].d : 0.f;
            int j1 = -1, j2 = -1;
            while (bmask && j2 < 0) {
                const int j = __builtin_ctzll(bmask);
                bmask &= bmask - 1;
                const float lbj = __shfl(lb, j);
                if (!(len < k || top > lbj)) continue;
                if (j1 < 0) j1 = j; else j2 = j;
            }
            if (j1 < 0) break;
            const int jj = lh ? j2 : j1;
            const int64_t row = (b0 + jj) * 32 + li;
            const uint32_t vword = __shfl(vwb, jj < 0 ? 0 : jj);
            const bool ok = jj >= 0 && row < nrows && ((vword >> li) & 1u);
            long long tc = DBG ? clock64() : 0;
            float dist = 0.f;
            bool cand = ok;  // an exact distance was computed for this lane's row
            if (filt) {
                bool need = ok;
                if (ok && len >= k) need = top > plane_a<METRIC>(Xb, xn2, row, dpb, sqh, qi.x) - eps_r;
                if (coop) dist = exact8_compact<METRIC>(qv, X, dpad, d, row, need, lane, s_d);
                else if (need) dist = exact_dist<METRIC, VARIANT>(qv, X + row * dpad, d);
                cand = need;
            } else if (coop) {  // 8 lanes per row, rows 8g + (lane >> 3) of the pair
                const float* xp[8];
#pragma unroll
                for (int g = 0; g < 8; g++) {
                    const int r = 8 * g + (lane >> 3);
                    const int jg = r >= 32 && j2 >= 0 ? j2 : j1;
                    const int64_t rw = (b0 + jg) * 32 + (r & 31);
                    xp[g] = X + (rw < nrows ? rw : 0) * dpad;
                }
                const float dl = exact8_rows64<METRIC>(qv, xp, d, lane);
                dist = ok ? dl : 0.f;
            } else if (ok) {
                dist = exact_dist<METRIC, VARIANT>(qv, X + row * dpad, d);
            }
            uint64_t mask = __ballot(cand && (len < k || top > dist));
            if (DBG) { t_dist += clock64() - tc; n_vis += j2 >= 0 ? 2 : 1; }
            if (mask == 0) continue;
            if (DBG) { tc = clock64(); n_ins += __popcll(mask); }
            s_d[lane] = dist;
            __syncthreads();
            if (lane == 0) {
                PHeap h{hr, *s_len};
                while (mask) {
                    const int l = __builtin_ctzll(mask);
                    mask &= mask - 1;
                    const float dj = s_d[l];
                    const int jb = l >= 32 ? j2 : j1;
                    ph_offer(h, k, id_base + (uint64_t)((b0 + jb) * 32 + (l & 31)), dj);
                }
                *s_len = h.len;
            }
            __syncthreads();
            if (DBG) t_heap += clock64() - tc;
        }
    }
    }
    if (DBG && lane == 0 && li_ < 24)
        printf("k_blk_replay dbg: list %d query %d visits %d offered %d heap_len %d cycles: all %lld dist %lld heap %lld\n",
               li_, q, n_vis, n_ins, *s_len, clock64() - t_all, t_dist, t_heap);
    const int64_t orow = by_list ? li_ : q;
    if (!extract) {  // hand the heap on in layout order (kout == k)
        const int n = *s_len;
        for (int i = lane; i < n; i += 64) {
            out_ids[orow * kout + i] = hr_id(hr[i]);
            out_d[orow * kout + i] = hr[i].d;
        }
        if (lane == 0) out_n[orow] = n;
        return;
    }
    if (lane == 0) {  // extractHeap (flat/index.go:676-688): pops max-first into the tail
        PHeap h{hr, *s_len};
        const int n = h.len;
        for (int i = n - 1; i >= 0; i--) {
            uint64_t x; float y;
            ph_pop(h, &x, &y);
            if (i < kout) { out_ids[orow * kout + i] = x; out_d[orow * kout + i] = y; }
        }
        out_n[orow] = n < kout ? n : kout;
    }
}

// ---------------------------------------------------------------------------
// k_blk_replay_par<METRIC, VARIANT>: the exact heap replay of k_blk_replay for
// k < 64 with the block-key scan spread over 8 waves (latency: a lone flagged
// query no longer walks every block key in one wave).
//   1. every wave: per chunk of 1024 blocks, the lane minima of U = A + eps
//      (16 blocks per lane) -> scratch; each is the exact-distance upper bound
//      of one distinct row;
//   2. wave 0: Uc[c] = k-th smallest of the minima of chunks < c and of the
//      handed-over heap -- an upper bound of the heap top at chunk c (the heap
//      holds the k smallest distances seen, flat/index.go:665-674);
//   3. every wave: candidate blocks A - eps < Uc[c] (a superset of the blocks
//      the reference scan can insert from), compacted in block order in LDS;
//   4. wave 0: the heap replay over the candidates only, visiting a block iff
//      the heap is short or top > A - eps (exactly k_blk_replay's rule).
// Non-finite queries and lists beyond RP_CAP fall back to every block in 4.
// ---------------------------------------------------------------------------
constexpr int RP_NW = 8, RP_CH = 1024, RP_CAP = 6144, RP_MAXCH = 4096;


template <int METRIC, int VARIANT>
__global__ __launch_bounds__(512) void k_blk_replay_par(const float* __restrict__ key, int64_t ldk, int64_t nb,
                                                        const float* __restrict__ eps_q, const float4* __restrict__ qinfo,
                                                        const float* __restrict__ X, int dpad,
                                                        const uint32_t* __restrict__ valid, int64_t nrows,
                                                        const float* __restrict__ Qn, int d,
                                                        const int32_t* __restrict__ qlist,
                                                        const uint32_t* __restrict__ counters, int nlist, int k, int kout,
                                                        uint64_t id_base, uint64_t* __restrict__ out_ids,
                                                        float* __restrict__ out_d, int32_t* __restrict__ out_n,
                                                        const uint64_t* __restrict__ in_ids,
                                                        const float* __restrict__ in_d,
                                                        const int32_t* __restrict__ in_len, int extract, int by_list,
                                                        float* __restrict__ scratch, int64_t vq = 0) {
    __shared__ uint64_t hid[64];
    __shared__ float hd[64];
    __shared__ float s_d[64];
    __shared__ int s_len, s_total;
    __shared__ uint32_t scand[RP_CAP];
    __shared__ float slb[RP_CAP];
    __shared__ float suc[RP_MAXCH];
    __shared__ int scc[RP_MAXCH];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int metric = METRIC == COSINE ? COSINE : METRIC == DOT ? DOT : L2;
    const int count = counters ? (int)counters[1] : nlist;
    const int nch = (int)((nb + RP_CH - 1) / RP_CH);
    float* sc = scratch + (int64_t)blockIdx.x * nch * 64;
    const int li = lane & 31, lh = lane >> 5;
    for (int li_ = blockIdx.x; li_ < count; li_ += gridDim.x) {
        const int q = qlist[li_];
        const uint32_t* vrow = vq ? valid + (int64_t)q * vq : valid;  // per-query allow bitmaps (vq words each)
        const float4 qi = qinfo[q];
        const bool noskip = qi.w != 0.f;
        const float eps = eps_q[q];
        const float* kr = key + (int64_t)q * ldk;
        const float* qv = Qn + (int64_t)q * dpad;
        int len_in = in_len ? in_len[by_list ? li_ : q] : 0;
        len_in = len_in < 0 ? 0 : len_in > k ? k : len_in;
        if (w == 0) {
            if (lane < len_in) {
                hid[lane] = in_ids[(int64_t)(by_list ? li_ : q) * k + lane];
                hd[lane] = in_d[(int64_t)(by_list ? li_ : q) * k + lane];
            }
            if (lane == 0) s_len = len_in;
        }
        // 1. lane minima of the upper bounds per chunk
        if (!noskip) {
            for (int c = w; c < nch; c += RP_NW) {
                float kv[16];
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const int64_t bb = (int64_t)c * RP_CH + u * 64 + lane;
                    kv[u] = bb < nb ? kr[bb] : __builtin_inff();
                }
                float m = __builtin_inff();
#pragma unroll
                for (int u = 0; u < 16; u++)
                    if (kv[u] < __builtin_inff()) m = fminf(m, qs_key_to_a(metric, kv[u], qi.x) + eps);
                sc[(int64_t)c * 64 + lane] = m;
            }
        }
        __syncthreads();
        // 2. prefix k-th smallest -> Uc
        if (w == 0 && !noskip) {
            float sk[2];
            uint32_t sid[2];
            sk[0] = lane < len_in ? hd[lane] : __builtin_inff();
            sid[0] = sid[1] = 0;
            {
                float t1[1] = {sk[0]};
                uint32_t i1[1] = {0};
                bitonic_sort<1>(t1, i1, lane);
                sk[0] = t1[0];
            }
            float thr = __shfl(sk[0], k - 1);
            for (int c0 = 0; c0 < nch; c0 += 16) {
                float v[16];
#pragma unroll
                for (int u = 0; u < 16; u++) v[u] = c0 + u < nch ? sc[(int64_t)(c0 + u) * 64 + lane] : __builtin_inff();
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    if (c0 + u >= nch) break;
                    if (lane == 0) suc[c0 + u] = thr;
                    if (__any(v[u] < thr)) {
                        sk[1] = v[u];
                        bitonic_sort<2>(sk, sid, lane);
                        thr = __shfl(sk[0], k - 1);
                    }
                }
            }
        }
        __syncthreads();
        // 3a. candidate counts per chunk
        if (!noskip) {
            for (int c = w; c < nch; c += RP_NW) {
                const float U = suc[c];
                int cnt = 0;
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const int64_t bb = (int64_t)c * RP_CH + u * 64 + lane;
                    const float kv = bb < nb ? kr[bb] : __builtin_inff();
                    const bool in = kv < __builtin_inff() && qs_key_to_a(metric, kv, qi.x) - eps < U;
                    cnt += __popcll(__ballot(in));
                }
                if (lane == 0) scc[c] = cnt;
            }
        }
        __syncthreads();
        // 3b. exclusive scan (wave 0)
        if (w == 0) {
            if (noskip) {
                if (lane == 0) s_total = RP_CAP + 1;
            } else {
                const int per = (nch + 63) / 64;
                const int c0 = lane * per, c1 = c0 + per < nch ? c0 + per : nch;
                int sum = 0;
                for (int c = c0; c < c1; c++) sum += scc[c];
                int incl = sum;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int t = __shfl_up(incl, o);
                    if (lane >= o) incl += t;
                }
                int run = incl - sum;
                for (int c = c0; c < c1; c++) { const int t = scc[c]; scc[c] = run; run += t; }
                if (lane == 63) s_total = incl;
            }
        }
        __syncthreads();
        const int total = s_total;
        // 3c. compaction in block order
        if (total <= RP_CAP) {
            for (int c = w; c < nch; c += RP_NW) {
                const float U = suc[c];
                int pos = scc[c];
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const int64_t bb = (int64_t)c * RP_CH + u * 64 + lane;
                    const float kv = bb < nb ? kr[bb] : __builtin_inff();
                    const float lb = qs_key_to_a(metric, kv, qi.x) - eps;
                    const bool in = kv < __builtin_inff() && lb < U;
                    const uint64_t m = __ballot(in);
                    if (in) {
                        const int o = pos + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                        scand[o] = (uint32_t)bb;
                        slb[o] = lb;
                    }
                    pos += __popcll(m);
                }
            }
        }
        __syncthreads();
        // 4. the heap replay over the candidates (wave 0)
        if (w == 0) {
            const bool use_list = total <= RP_CAP;
            const int64_t ncand = use_list ? total : nb;
            for (int64_t base = 0; base < ncand; base += 64) {
                const int64_t e = base + lane;
                int64_t blk = 0;
                float lb = __builtin_inff();
                bool has = false;
                if (e < ncand) {
                    if (use_list) {
                        blk = scand[e];
                        lb = slb[e];
                        has = true;
                    } else {
                        blk = e;
                        const float kv = kr[e];
                        has = noskip || kv < __builtin_inff();
                        lb = noskip ? -__builtin_inff() : qs_key_to_a(metric, kv, qi.x) - eps;
                    }
                }
                int len = s_len;
                float top = len > 0 ? hd[0] : 0.f;
                uint64_t bmask = __ballot(has && (len < k || top > lb));
                while (bmask) {
                    len = s_len;
                    top = len > 0 ? hd[0] : 0.f;
                    int j1 = -1, j2 = -1;
                    while (bmask && j2 < 0) {
                        const int j = __builtin_ctzll(bmask);
                        bmask &= bmask - 1;
                        const float lbj = __shfl(lb, j);
                        if (!(len < k || top > lbj)) continue;
                        if (j1 < 0) j1 = j; else j2 = j;
                    }
                    if (j1 < 0) break;
                    const int64_t b1 = __shfl(blk, j1);
                    const int64_t b2 = __shfl(blk, j2 < 0 ? j1 : j2);
                    const bool okb = lh ? j2 >= 0 : true;
                    const int64_t row = (lh ? b2 : b1) * 32 + li;
                    const bool ok = okb && row < nrows && ((vrow[row >> 5] >> (row & 31)) & 1u);
                    const float dist = ok ? exact_dist<METRIC, VARIANT>(qv, X + row * dpad, d) : 0.f;
                    uint64_t mask = __ballot(ok && (len < k || top > dist));
                    if (mask == 0) continue;
                    s_d[lane] = dist;
                    wave_sync_lds();
                    if (lane == 0) {
                        ReplayHeap h{hid, hd, s_len};
                        while (mask) {
                            const int l = __builtin_ctzll(mask);
                            mask &= mask - 1;
                            const float dj = s_d[l];
                            const int64_t bj = l >= 32 ? b2 : b1;
                            const uint64_t idj = id_base + (uint64_t)(bj * 32 + (l & 31));
                            if (h.len < k) rh_insert(h, idj, dj);
                            else if (h.dist[0] > dj) { uint64_t x; float y; rh_pop(h, &x, &y); rh_insert(h, idj, dj); }
                        }
                        s_len = h.len;
                    }
                    wave_sync_lds();
                }
            }
            const int64_t orow = by_list ? li_ : q;
            if (!extract) {
                const int n = s_len;
                if (lane < n) {
                    out_ids[orow * kout + lane] = hid[lane];
                    out_d[orow * kout + lane] = hd[lane];
                }
                if (lane == 0) out_n[orow] = n;
            } else if (lane == 0) {
                ReplayHeap h{hid, hd, s_len};
                const int n = h.len;
                for (int i = n - 1; i >= 0; i--) {
                    uint64_t x; float y;
                    rh_pop(h, &x, &y);
                    if (i < kout) { out_ids[orow * kout + i] = x; out_d[orow * kout + i] = y; }
                }
                out_n[orow] = n < kout ? n : kout;
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Three-kernel form of the block-key replay (default):
//   k_rp_bounds  8 waves per listed query: heap-top upper bounds per chunk of
//                1024 blocks (k-th smallest of the earlier chunks' row upper
//                bounds A + eps, and of the handed-over heap), refined inside
//                chunk 0 per 64-block group; candidate blocks (A - eps below
//                the bound) compacted in block order into a shared pool;
//   k_rp_exact   the whole grid: reference-order exact distances of every
//                row of every pooled block (no serial dependency left);
//   k_rp_heap    one wave per listed query: insertToHeap over the pooled
//                blocks in order, visiting a block iff the heap is short or
//                top > A - eps (k_blk_replay's rule), distances read back
//                from the pool in windows of 16 blocks.
// A query whose candidates do not fit the pool, or with non-finite values,
// replays every block with on-the-fly distances in k_rp_heap.
// ---------------------------------------------------------------------------
constexpr int RPW = 64;  // k_rp_heap window (blocks)

// element e of a wave-sorted list of RS rows (broadcast)
template <int RS>
__device__ __forceinline__ float rp_key_at(const float (&key)[RS], int e) {
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < RS; r++) {
        const float t = __shfl(key[r], e & 63);
        if ((e >> 6) == r) v = t;
    }
    return v;
}

// merge 64 new values (one per lane) into the sorted list rows 0..RS-2 when any
// is below thr; returns the new k-th smallest
template <int RS>
__device__ __forceinline__ float rp_offer(float (&sk)[RS], uint32_t (&sid)[RS], float v, float thr, int k, int lane) {
    uint64_t bm = __ballot(v < thr);
    if (!bm) return thr;
    if (__popcll(bm) <= 8) {
        // a few values under the threshold (the common case after the first
        // chunks): insert them one by one into rows 0..RS-2 (element e = 64 r +
        // lane, ascending; the last one drops out), new[e] = old[e] < x ? old[e]
        // : max(x, old[e - 1]) -- a few shuffles each instead of a 64-value sort
        // (the list's ids stay 0: k_rp_bounds keeps values only)
        while (bm) {
            const int l = __builtin_ctzll(bm);
            bm &= bm - 1;
            const float x = __shfl(v, l);
            if (!(x < thr)) continue;
            float prev_last = -__builtin_inff();
#pragma unroll
            for (int r = 0; r < RS - 1; r++) {
                const float o = sk[r];
                const float up = __shfl_up(o, 1);
                const float last = __shfl(o, 63);
                const float pe = lane == 0 ? prev_last : up;
                sk[r] = o < x ? o : fmaxf(x, pe);
                prev_last = last;
            }
            thr = rp_key_at<RS>(sk, k - 1);
        }
        return thr;
    }
    sk[RS - 1] = v;
    sid[RS - 1] = 0;
    bitonic_merge_last<RS>(sk, sid, lane);
    return rp_key_at<RS>(sk, k - 1);
}

// k_rp_bounds: 16 waves per listed query, two chunks per wave and step (64
// loads in flight per lane): a lone flagged query of a 10M-row corpus (306
// chunks) is latency-bound in one workgroup
// (8 waves for RS = 4 / 8: their sorted lists need the registers)
constexpr int rp_bounds_nw(int RS) { return RS == 2 ? 16 : 8; }

template <int RS, int METRIC>
__global__ __launch_bounds__(64 * rp_bounds_nw(RS)) void k_rp_bounds(const float* __restrict__ key, int64_t ldk, int64_t nb,
                                                   const float* __restrict__ eps_q, const float4* __restrict__ qinfo,
                                                   const int32_t* __restrict__ qlist, const uint32_t* __restrict__ counters,
                                                   int nlist, int k, const float* __restrict__ in_d,
                                                   const int32_t* __restrict__ in_len, float* __restrict__ scratch,
                                                   uint32_t* __restrict__ pool_blk, float* __restrict__ pool_lb,
                                                   int32_t* __restrict__ pool_q, uint32_t* __restrict__ pool_ctr,
                                                   int64_t pool_cap, int32_t* __restrict__ rp_off,
                                                   int32_t* __restrict__ rp_tot, int by_list) {
    __shared__ float suc[RP_MAXCH];
    __shared__ int scc[RP_MAXCH];
    __shared__ float sg0[16];
    __shared__ int s_total, s_off;
    constexpr int NW = rp_bounds_nw(RS);
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int metric = METRIC == COSINE ? COSINE : METRIC == DOT ? DOT : L2;
    const int count = counters ? (int)counters[1] : nlist;
    const int nch = (int)((nb + RP_CH - 1) / RP_CH);
    float* sc = scratch + (int64_t)blockIdx.x * nch * 64;
    for (int li_ = blockIdx.x; li_ < count; li_ += gridDim.x) {
        const int q = qlist[li_];
        const float4 qi = qinfo[q];
        const bool noskip = qi.w != 0.f;
        const float eps = eps_q[q];
        const float* kr = key + (int64_t)q * ldk;
        int len_in = in_len ? in_len[by_list ? li_ : q] : 0;
        len_in = len_in < 0 ? 0 : len_in > k ? k : len_in;
        if (noskip) {  // every block, distances on the fly (k_rp_heap)
            if (threadIdx.x == 0) { rp_off[li_] = -1; rp_tot[li_] = 0; }
            continue;
        }
        // 1. per chunk, per lane: the smallest row upper bound A + eps of 16 blocks
        for (int c = w; c < nch; c += 2 * NW) {
            float kv[2][16];
#pragma unroll
            for (int h = 0; h < 2; h++) {  // one base address per chunk, immediate offsets
                const float* kc = kr + (int64_t)(c + h * NW) * RP_CH;
                const int64_t rem = nb - (int64_t)(c + h * NW) * RP_CH;
#pragma unroll
                for (int u = 0; u < 16; u++) kv[h][u] = u * 64 + lane < rem ? kc[u * 64 + lane] : __builtin_inff();
            }
#pragma unroll
            for (int h = 0; h < 2; h++) {
                float m = __builtin_inff();
#pragma unroll
                for (int u = 0; u < 16; u++)
                    if (kv[h][u] < __builtin_inff()) m = fminf(m, qs_key_to_a(metric, kv[h][u], qi.x) + eps);
                if (c + h * NW < nch) sc[(int64_t)(c + h * NW) * 64 + lane] = m;
            }
        }
        __syncthreads();
        // 2. wave 0: suc[c] = k-th smallest of the handed-over heap and of the
        //    lane minima of chunks < c (an upper bound of the heap top at chunk c)
        if (w == 0) {
            float sk[RS];
            uint32_t sid[RS];
#pragma unroll
            for (int r = 0; r < RS; r++) {
                const int e = r * 64 + lane;
                sk[r] = (r < RS - 1 && e < len_in) ? in_d[(int64_t)(by_list ? li_ : q) * k + e] : __builtin_inff();
                sid[r] = 0;
            }
            bitonic_sort<RS>(sk, sid, lane);
            float thr = rp_key_at<RS>(sk, k - 1);
            float v[16];  // the next 16 chunks' lane minima are read while these merge
#pragma unroll
            for (int u = 0; u < 16; u++) v[u] = u < nch ? sc[(int64_t)u * 64 + lane] : __builtin_inff();
            for (int c0 = 0; c0 < nch; c0 += 16) {
                float vn[16];
#pragma unroll
                for (int u = 0; u < 16; u++)
                    vn[u] = c0 + 16 + u < nch ? sc[(int64_t)(c0 + 16 + u) * 64 + lane] : __builtin_inff();
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    if (c0 + u >= nch) break;
                    if (lane == 0) suc[c0 + u] = thr;
                    thr = rp_offer<RS>(sk, sid, v[u], thr, k, lane);
                }
#pragma unroll
                for (int u = 0; u < 16; u++) v[u] = vn[u];
            }
            // chunk 0 per 64-block group: also bounded by the k-th smallest A + eps
            // of its own earlier groups (the chunk-level bound is weakest there)
            float kv[16];
#pragma unroll
            for (int u = 0; u < 16; u++) kv[u] = u * 64 + lane < nb ? kr[u * 64 + lane] : __builtin_inff();
#pragma unroll
            for (int r = 0; r < RS; r++) { sk[r] = __builtin_inff(); sid[r] = 0; }
            float tin = __builtin_inff();
            const float U0 = suc[0];
#pragma unroll
            for (int u = 0; u < 16; u++) {
                if (lane == 0) sg0[u] = fminf(U0, tin);
                tin = rp_offer<RS>(sk, sid, kv[u] < __builtin_inff() ? qs_key_to_a(metric, kv[u], qi.x) + eps
                                                                    : __builtin_inff(), tin, k, lane);
            }
        }
        __syncthreads();
        // 3. candidate blocks of chunk c: A - eps < bound (suc[c]; inside chunk 0
        //    the per-group bound sg0[u]).  pass 0: counts, pass 1: compaction.
        for (int pass = 0; pass < 2; pass++) {
            const int off = pass ? s_off : 0;
            if (pass == 0 || off >= 0) {
                for (int c2 = w; c2 < nch; c2 += 2 * NW) {
                    float ka[16], kb[16];  // both chunks' keys in flight, one body (ballot SGPRs)
                    {
                        const float* kc = kr + (int64_t)c2 * RP_CH;
                        const int64_t rem = nb - (int64_t)c2 * RP_CH;
#pragma unroll
                        for (int u = 0; u < 16; u++) ka[u] = u * 64 + lane < rem ? kc[u * 64 + lane] : __builtin_inff();
                        const int64_t remb = rem - (int64_t)NW * RP_CH;
#pragma unroll
                        for (int u = 0; u < 16; u++)
                            kb[u] = u * 64 + lane < remb ? kc[(int64_t)NW * RP_CH + u * 64 + lane] : __builtin_inff();
                    }
#pragma unroll 1
                    for (int h = 0; h < 2; h++) {
                        const int c = c2 + h * NW;
                        if (c >= nch) break;
                        const float U = suc[c];
                        int pos = pass ? off + scc[c] : 0;
#pragma unroll
                        for (int u = 0; u < 16; u++) {
                            const uint32_t bb = (uint32_t)(c * RP_CH + u * 64 + lane);
                            const float lb = qs_key_to_a(metric, ka[u], qi.x) - eps;
                            const bool in = ka[u] < __builtin_inff() && lb < (c == 0 ? sg0[u] : U);
                            const uint64_t m = __ballot(in);
                            if (pass && in) {
                                const int o = pos + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                                pool_blk[o] = (uint32_t)bb;
                                pool_lb[o] = c == 0 ? sg0[u] : U;  // the heap top's bound at this block
                                pool_q[o] = li_;
                            }
                            pos += __popcll(m);
                        }
#pragma unroll
                        for (int u = 0; u < 16; u++) ka[u] = kb[u];
                        if (!pass && lane == 0) scc[c] = pos;
                    }
                }
            }
            __syncthreads();
            if (pass == 0 && w == 0) {  // exclusive scan of the chunk counts, pool allocation
                const int per = (nch + 63) / 64;
                const int c0 = lane * per, c1 = c0 + per < nch ? c0 + per : nch;
                int sum = 0;
                for (int c = c0; c < c1; c++) sum += scc[c];
                int incl = sum;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int t = __shfl_up(incl, o);
                    if (lane >= o) incl += t;
                }
                int run = incl - sum;
                for (int c = c0; c < c1; c++) { const int t = scc[c]; scc[c] = run; run += t; }
                if (lane == 63) {
                    s_total = incl;
                    int64_t o = incl > 0 ? (int64_t)atomicAdd(pool_ctr, (uint32_t)incl) : 0;
                    if (o + incl > pool_cap) {  // pool exhausted: mark the claimed tail dead
                        for (int64_t e = o; e < pool_cap; e++) pool_q[e] = -1;
                        o = -1;
                    }
                    s_off = (int)o;
                    rp_off[li_] = (int)o;
                    rp_tot[li_] = incl;
                }
            }
            __syncthreads();
        }
    }
}

// exact distances of the pooled blocks' rows: pool_E[e][32], and in pool_vm[e]
// the rows that can enter the heap: valid and E < pool_ub[e], the bound of the
// heap top at that block (k_rp_bounds; +inf: the heap may still be short, every
// valid row)
template <int METRIC, int VARIANT>
__global__ __launch_bounds__(256) void k_rp_exact(const float* __restrict__ X, int dpad, const uint32_t* __restrict__ valid,
                                                  int64_t nrows, const float* __restrict__ Qn, int d,
                                                  const int32_t* __restrict__ qlist, const uint32_t* __restrict__ pool_blk,
                                                  const float* __restrict__ pool_ub,
                                                  const int32_t* __restrict__ pool_q, const uint32_t* __restrict__ pool_ctr,
                                                  int64_t pool_cap, float* __restrict__ pool_E,
                                                  uint32_t* __restrict__ pool_vm, int64_t vq = 0) {
    const int lane = threadIdx.x & 63;
    const int li = lane & 31, lh = lane >> 5;
    int64_t used = (int64_t)pool_ctr[0];
    used = used < pool_cap ? used : pool_cap;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t p = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); 2 * p < used; p += nw) {
        const int64_t e = 2 * p + lh;
        bool ok = false;
        float dist = 0.f;
        if (e < used) {
            const int lq = pool_q[e];
            if (lq >= 0) {
                const int q = qlist[lq];
                const uint32_t* vrow = vq ? valid + (int64_t)q * vq : valid;  // per-query allow bitmaps (vq words each)
                const int64_t row = (int64_t)pool_blk[e] * 32 + li;
                ok = row < nrows && ((vrow[row >> 5] >> (row & 31)) & 1u);
                if (ok) dist = exact_dist<METRIC, VARIANT>(Qn + (int64_t)q * dpad, X + row * dpad, d);
                pool_E[e * 32 + li] = dist;
                const float ub = pool_ub[e];
                ok = ok && (dist < ub || !(ub < __builtin_inff()));
            }
        }
        const uint64_t m = __ballot(ok);
        if (e < used && li == 0) pool_vm[e] = (uint32_t)(m >> (32 * lh));
    }
}

// one wave per listed query: the reference heap over the pooled blocks
template <int METRIC, int VARIANT>
__global__ __launch_bounds__(64) void k_rp_heap(const float* __restrict__ key, int64_t ldk, int64_t nb,
                                                const float* __restrict__ eps_q, const float4* __restrict__ qinfo,
                                                const float* __restrict__ X, int dpad, const uint32_t* __restrict__ valid,
                                                int64_t nrows, const float* __restrict__ Qn, int d,
                                                const int32_t* __restrict__ qlist, const uint32_t* __restrict__ counters,
                                                int nlist, int k, int kout, uint64_t id_base, uint64_t* __restrict__ out_ids,
                                                float* __restrict__ out_d, int32_t* __restrict__ out_n,
                                                const uint64_t* __restrict__ in_ids, const float* __restrict__ in_d,
                                                const int32_t* __restrict__ in_len, int extract, int by_list,
                                                const uint32_t* __restrict__ pool_blk, const float* __restrict__ pool_lb,
                                                const float* __restrict__ pool_E, const uint32_t* __restrict__ pool_vm,
                                                const int32_t* __restrict__ rp_off, const int32_t* __restrict__ rp_tot,
                                                uint64_t* __restrict__ rec_ids, float* __restrict__ rec_d,
                                                int32_t* __restrict__ rec_n, int rec_cap, int64_t vq = 0) {
    extern __shared__ __attribute__((aligned(16))) unsigned char rsm[];
    uint64_t* hid = reinterpret_cast<uint64_t*>(rsm);
    float* hd = reinterpret_cast<float*>(hid + k);
    float* s_d = hd + k;                 // [64]
    float* sE = s_d + 64;                // [RPW][32]
    uint64_t* sM = reinterpret_cast<uint64_t*>(((uintptr_t)(sE + RPW * 32) + 7) & ~(uintptr_t)7);  // [RPW / 2]
    int* s_len = reinterpret_cast<int*>(sM + RPW / 2);
    const int lane = threadIdx.x;
    const int metric = METRIC == COSINE ? COSINE : METRIC == DOT ? DOT : L2;
    const int count = counters ? (int)counters[1] : nlist;
    const int li = lane & 31, lh = lane >> 5;
    for (int li_ = blockIdx.x; li_ < count; li_ += gridDim.x) {
        const int q = qlist[li_];
        const uint32_t* vrow = vq ? valid + (int64_t)q * vq : valid;  // per-query allow bitmaps (vq words each)
        const float* qv = Qn + (int64_t)q * dpad;
        const int64_t orow = by_list ? li_ : q;
        int nrec = 0;  // recorded insertions (lane 0): the parallel cross-shard replay
        // insertToHeap (flat/index.go:665-674) by lane 0, recording what entered
        auto ins = [&](ReplayHeap& h, uint64_t idj, float dj) {
            bool did = false;
            if (h.len < k) { rh_insert(h, idj, dj); did = true; }
            else if (h.dist[0] > dj) { uint64_t x; float y; rh_pop(h, &x, &y); rh_insert(h, idj, dj); did = true; }
            if (did && rec_ids) {
                if (nrec < rec_cap) { rec_ids[orow * rec_cap + nrec] = idj; rec_d[orow * rec_cap + nrec] = dj; }
                nrec++;
            }
        };
        int len_in = in_len ? in_len[by_list ? li_ : q] : 0;
        len_in = len_in < 0 ? 0 : len_in > k ? k : len_in;
        for (int i = lane; i < len_in; i += 64) {
            hid[i] = in_ids[(int64_t)(by_list ? li_ : q) * k + i];
            hd[i] = in_d[(int64_t)(by_list ? li_ : q) * k + i];
        }
        if (lane == 0) *s_len = len_in;
        wave_sync_lds();
        const int off = rp_off[li_];
        if (off >= 0) {
            const int tot = rp_tot[li_];
            // a window of RPW = 64 pooled blocks = 2048 rows, row e = lane + 64 u
            // of block e >> 5 held in registers; the next window's rows are read
            // while this one is tested.  pool_vm holds only the rows under the
            // bound of the heap top at their block (k_rp_exact), and the top only
            // falls: a window with no such row under the top at its start (heap
            // full) is skipped whole, otherwise lane 0 runs insertToHeap over its
            // candidate rows in id order.
            uint32_t* sBlk = reinterpret_cast<uint32_t*>(s_d);  // [RPW] block ids of the window
            float cur[RPW / 2], nxt[RPW / 2];
            auto load_win = [&](int w0, float (&v)[RPW / 2]) {
                const int nwin = tot - w0 < RPW ? tot - w0 : RPW;
#pragma unroll
                for (int u = 0; u < RPW / 2; u++) {
                    const int e = lane + 64 * u;
                    v[u] = (e >> 5) < nwin ? pool_E[(int64_t)(off + w0) * 32 + e] : 0.f;
                }
            };
            if (tot > 0) load_win(0, cur);
            for (int w0 = 0; w0 < tot; w0 += RPW) {
                const int nwin = tot - w0 < RPW ? tot - w0 : RPW;
                const bool more = w0 + RPW < tot;
                if (more) load_win(w0 + RPW, nxt);
                const uint32_t blk = lane < nwin ? pool_blk[off + w0 + lane] : 0u;
                const uint32_t vm = lane < nwin ? pool_vm[off + w0 + lane] : 0u;
                if (__any(vm != 0u)) {
                    const int len = *s_len;
                    const bool open = len < k;
                    const float top = len > 0 ? hd[0] : 0.f;
                    uint32_t cb = 0;
#pragma unroll
                    for (int u = 0; u < RPW / 2; u++) {
                        const uint32_t vmb = (uint32_t)__shfl((int)vm, 2 * u + lh);
                        if (((vmb >> li) & 1u) && (open || top > cur[u])) cb |= 1u << u;
                    }
                    if (open && __any(cb != 0)) {
                        // the heap is still short: block by block with the top
                        // re-read (as it fills, a window-wide test admits every row)
#pragma unroll
                        for (int u = 0; u < RPW / 2; u++) sE[lane + 64 * u] = cur[u];
                        sBlk[lane] = blk;
                        wave_sync_lds();
                        for (int j = 0; j < nwin; j++) {
                            const int lj = *s_len;
                            const float tj = lj > 0 ? hd[0] : 0.f;
                            const uint32_t vmj = (uint32_t)__shfl((int)vm, j);
                            const float dist = lane < 32 ? sE[j * 32 + lane] : 0.f;
                            uint64_t mask = __ballot(lane < 32 && ((vmj >> lane) & 1u) && (lj < k || tj > dist));
                            if (mask == 0) continue;
                            if (lane == 0) {
                                ReplayHeap h{hid, hd, lj};
                                while (mask) {
                                    const int l = __builtin_ctzll(mask);
                                    mask &= mask - 1;
                                    ins(h, id_base + (uint64_t)sBlk[j] * 32 + (uint64_t)l, sE[j * 32 + l]);
                                }
                                *s_len = h.len;
                            }
                            wave_sync_lds();
                        }
                        wave_sync_lds();
                    } else if (__any(cb != 0)) {
#pragma unroll
                        for (int u = 0; u < RPW / 2; u++) sE[lane + 64 * u] = cur[u];
                        sBlk[lane] = blk;
#pragma unroll
                        for (int u = 0; u < RPW / 2; u++) {
                            const uint64_t m = __ballot((cb >> u) & 1u);
                            if (lane == 0) sM[u] = m;
                        }
                        wave_sync_lds();
                        if (lane == 0) {
                            ReplayHeap h{hid, hd, len};
                            for (int u = 0; u < RPW / 2; u++) {
                                uint64_t mask = sM[u];
                                while (mask) {
                                    const int e = 64 * u + __builtin_ctzll(mask);
                                    mask &= mask - 1;
                                    const uint64_t idj = id_base + (uint64_t)sBlk[e >> 5] * 32 + (uint64_t)(e & 31);
                                    ins(h, idj, sE[e]);
                                }
                            }
                            *s_len = h.len;
                        }
                        wave_sync_lds();  // heap state for the next window; sE / sBlk / sM are rewritten there
                    }
                }
                if (more) {
#pragma unroll
                    for (int u = 0; u < RPW / 2; u++) cur[u] = nxt[u];
                }
            }
        } else {
            // every block (non-finite values or pool exhausted), distances on the fly
            const float4 qi = qinfo[q];
            const bool noskip = qi.w != 0.f;
            const float eps = eps_q[q];
            const float* kr = key + (int64_t)q * ldk;
            for (int64_t b0 = 0; b0 < nb; b0 += 64) {
                const int64_t bb = b0 + lane;
                float lb = __builtin_inff();
                bool has = false;
                if (bb < nb) {
                    const float kv = kr[bb];
                    has = noskip || kv < __builtin_inff();
                    lb = noskip ? -__builtin_inff() : qs_key_to_a(metric, kv, qi.x) - eps;
                }
                int len = *s_len;
                float top = len > 0 ? hd[0] : 0.f;
                uint64_t bmask = __ballot(has && (len < k || top > lb));
                while (bmask) {
                    len = *s_len;
                    top = len > 0 ? hd[0] : 0.f;
                    int j1 = -1, j2 = -1;
                    while (bmask && j2 < 0) {
                        const int j = __builtin_ctzll(bmask);
                        bmask &= bmask - 1;
                        const float lbj = __shfl(lb, j);
                        if (!(len < k || top > lbj)) continue;
                        if (j1 < 0) j1 = j; else j2 = j;
                    }
                    if (j1 < 0) break;
                    const int jj = lh ? j2 : j1;
                    const int64_t row = (b0 + jj) * 32 + li;
                    const bool ok = jj >= 0 && row < nrows && ((vrow[row >> 5] >> (row & 31)) & 1u);
                    const float dist = ok ? exact_dist<METRIC, VARIANT>(qv, X + row * dpad, d) : 0.f;
                    uint64_t mask = __ballot(ok && (len < k || top > dist));
                    if (mask == 0) continue;
                    s_d[lane] = dist;
                    wave_sync_lds();
                    if (lane == 0) {
                        ReplayHeap h{hid, hd, *s_len};
                        while (mask) {
                            const int l = __builtin_ctzll(mask);
                            mask &= mask - 1;
                            const int jb = l >= 32 ? j2 : j1;
                            const uint64_t idj = id_base + (uint64_t)((b0 + jb) * 32 + (l & 31));
                            const float dj = s_d[l];
                            ins(h, idj, dj);
                        }
                        *s_len = h.len;
                    }
                    wave_sync_lds();
                }
            }
        }
        if (rec_ids && lane == 0) rec_n[orow] = nrec > rec_cap ? rec_cap + 1 : nrec;
        if (!extract) {  // hand the heap on in layout order (kout == k)
            const int n = *s_len;
            for (int i = lane; i < n; i += 64) {
                out_ids[orow * kout + i] = hid[i];
                out_d[orow * kout + i] = hd[i];
            }
            if (lane == 0) out_n[orow] = n;
        } else if (lane == 0) {  // extractHeap (flat/index.go:676-688)
            ReplayHeap h{hid, hd, *s_len};
            const int n = h.len;
            for (int i = n - 1; i >= 0; i--) {
                uint64_t x; float y;
                rh_pop(h, &x, &y);
                if (i < kout) { out_ids[orow * kout + i] = x; out_d[orow * kout + i] = y; }
            }
            out_n[orow] = n < kout ? n : kout;
        }
        wave_sync_lds();
    }
}

// Parallel cross-shard replay, final step (weaviate_amd/sharded.py): one wave
// per listed query.  Start from shard 0's heap state (layout order), then apply
// insertToHeap over every later shard's recorded insertions in shard (= id)
// order, then extractHeap.  A shard's record holds every row that entered its
// replay from a full heap of k copies of T_r (>= the real heap top at that
// shard's start), a superset of the rows that enter the real heap there, so
// this equals the serial chain.  rec_n > cap: overflowed -> unresolved[li] = 1.
__global__ __launch_bounds__(64) void k_heap_merge_records(int nlist, int k, int W, int cap,
                                                           const uint64_t* __restrict__ st_ids,
                                                           const float* __restrict__ st_d,
                                                           const int32_t* __restrict__ st_n,
                                                           const uint64_t* __restrict__ rec_ids,
                                                           const float* __restrict__ rec_d,
                                                           const int32_t* __restrict__ rec_n,
                                                           uint64_t* __restrict__ out_ids, float* __restrict__ out_d,
                                                           int32_t* __restrict__ out_n, int32_t* __restrict__ unresolved) {
    extern __shared__ __attribute__((aligned(16))) unsigned char msm[];
    uint64_t* hid = reinterpret_cast<uint64_t*>(msm);
    float* hd = reinterpret_cast<float*>(hid + k);
    const int li = blockIdx.x;
    if (li >= nlist || threadIdx.x != 0) return;
    int n0 = st_n[li];
    n0 = n0 < 0 ? 0 : n0 > k ? k : n0;
    for (int i = 0; i < n0; i++) { hid[i] = st_ids[(int64_t)li * k + i]; hd[i] = st_d[(int64_t)li * k + i]; }
    ReplayHeap h{hid, hd, n0};
    int bad = 0;
    for (int r = 1; r < W; r++) {
        const int64_t base = (int64_t)r * nlist + li;
        const int m = rec_n[base];
        if (m > cap) { bad = 1; continue; }
        for (int j = 0; j < m; j++) {
            const float dj = rec_d[base * cap + j];
            const uint64_t idj = rec_ids[base * cap + j];
            if (h.len < k) rh_insert(h, idj, dj);
            else if (h.dist[0] > dj) { uint64_t x; float y; rh_pop(h, &x, &y); rh_insert(h, idj, dj); }
        }
    }
    unresolved[li] = bad;
    const int n = h.len;
    for (int i = n - 1; i >= 0; i--) {
        uint64_t x; float y;
        rh_pop(h, &x, &y);
        out_ids[(int64_t)li * k + i] = x;
        out_d[(int64_t)li * k + i] = y;
    }
    out_n[li] = n;
}

}  // namespace
}  // namespace wv
