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
};

__device__ __forceinline__ uint32_t sload_u32(const void* p) {
    const uint64_t pi = (uint64_t)p;
    const uint64_t up = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(pi >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)pi);
    uint32_t v;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(up) : "memory");
    return v;
}

// s_waitcnt vmcnt(y) for a run-time wave-uniform y (0..23)
__device__ __forceinline__ void qs_wait_vm(int y) {
#define QS_VM(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    switch (y) {
        QS_VM(0) QS_VM(1) QS_VM(2) QS_VM(3) QS_VM(4) QS_VM(5) QS_VM(6) QS_VM(7) QS_VM(8) QS_VM(9) QS_VM(10)
        QS_VM(11) QS_VM(12) QS_VM(13) QS_VM(14) QS_VM(15) QS_VM(16) QS_VM(17) QS_VM(18) QS_VM(19) QS_VM(20)
        QS_VM(21) QS_VM(22) QS_VM(23)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
#undef QS_VM
}

template <int N>
__device__ __forceinline__ void qs_wait_lgkm() {
    if constexpr (N == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else if constexpr (N == 1) asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
}

typedef float f32x4_t __attribute__((ext_vector_type(4)));
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
template <int NK, bool ISL2>
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

    // this wave's 32 queries as MFMA B fragments for all of d: lane (li, lh)
    // holds query wave*32+li, columns 16c + 8lh .. +7 of chunk c
    bf16x8_t Qf[NK];
    {
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
    const int prow = lane >> 1;
    const uint32_t src_lane = (uint32_t)(prow * 32 + 16 * ((lane & 1) ^ ((prow >> 3) & 1)));
    const unsigned ring = lds_addr(qsm);
    const unsigned xnring = ring + QS_NBUF * SLOT;  // L2: [NBUF][RB*32] floats
    const int P0 = P + ((ISL2 && wave == 0) ? 1 : 0);
    // the span's rows through one buffer resource (the host keeps a span's
    // plane bytes below 4 GiB): per piece an SGPR offset + the lane's VGPR
    const int64_t tile0 = (s0 * RB * 32) >> 8;
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.Xb + tile0 * TILE_B), (short)0, -1, 0x00020000);
    auto issue = [&](int64_t gs, int slot) {
        const unsigned sb = ring + (unsigned)(slot * SLOT);
#pragma unroll
        for (int i = 0; i < P; i++) {
            const int p = wave + 8 * i;
            const int rb = p / NK, c = p % NK;
            const int64_t gb = gs * RB + rb;
            const uint32_t so = (uint32_t)(((gb >> 3) - tile0) * TILE_B + (int64_t)c * 8192 + (gb & 7) * 1024);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(size_t)(sb + (unsigned)((rb * NK + c) * 1024)), 16,
                                                     src_lane, so, 0, 0);
        }
        if (ISL2 && wave == 0) {
            if (lane < RB * 8)
                __builtin_amdgcn_global_load_lds(a.xnorm2 + gs * RB * 32 + 4 * lane,
                                                 (lds_ptr_t)(size_t)(xnring + (unsigned)(slot * RB * 128)), 16, 0, 0);
        }
    };

    if (nsteps > 0) issue(s0, 0);
    if (nsteps > 1) issue(s0 + 1, 1);

    const unsigned lane_off = (unsigned)(li * 32 + 16 * (lh ^ ((li >> 3) & 1)));
    const int64_t qrow = (int64_t)grp * QS_QPB + wave * 32 + li;
    float* krow = a.key + qrow * a.ldk;
    int slot = 0;
    for (int step = 0; step < nsteps; step++) {
        // ops issued after slot `step`'s pieces: the stores of the two
        // previous steps and slot step+1's pieces (issue order, vmcnt counts both)
        const int y = (step >= 1 ? RB : 0) + (step >= 2 ? RB : 0) + (step + 1 < nsteps ? P0 : 0);
        qs_wait_vm(y);
        __builtin_amdgcn_s_barrier();  // every wave's pieces of this slot landed; slot step+2 is free
        __builtin_amdgcn_sched_barrier(0);
        if (step + 2 < nsteps) issue(s0 + step + 2, slot == 0 ? 2 : slot - 1);
        const unsigned sb = ring + (unsigned)(slot * SLOT) + lane_off;
        static_for<0, RB>([&](auto rbc) {
            constexpr int rb = decltype(rbc)::value;
            f32x16 acc;
#pragma unroll
            for (int r = 0; r < 16; r++) acc[r] = 0.f;
            bf16x8_t A[4];
            A[0] = lds_ld8bf_o<(rb * NK + 0) * 1024>(sb);
            A[1] = lds_ld8bf_o<(rb * NK + 1) * 1024>(sb);
            A[2] = lds_ld8bf_o<(rb * NK + 2) * 1024>(sb);
            A[3] = lds_ld8bf_o<(rb * NK + 3) * 1024>(sb);
            static_for<0, NK>([&](auto cc) {
                constexpr int c = decltype(cc)::value;
                qs_wait_lgkm<(NK - 1 - c) < 3 ? (NK - 1 - c) : 3>();
                asm volatile("" : "+v"(A[c & 3]));
                __builtin_amdgcn_sched_barrier(0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[c & 3], Qf[c], acc, 0, 0, 0);
                if constexpr (c + 4 < NK) A[c & 3] = lds_ld8bf_o<(rb * NK + c + 4) * 1024>(sb);
            });
            // ---- epilogue: the block's key for this lane's query ----
            const int64_t gb = (s0 + step) * RB + rb;
            const uint32_t vw = sload_u32(a.valid + gb);
            // rows of acc[r]: (r&3) + 8(r>>2) + 4lh; the valid word shifted by 4lh
            // leaves a compile-time bit position per r
            const uint32_t vl = vw >> (4 * lh);
            float m;
            if constexpr (ISL2) {
                const unsigned xb = xnring + (unsigned)(slot * RB * 128 + rb * 128 + 16 * lh);
                m = __builtin_inff();
                static_for<0, 4>([&](auto gg) {
                    constexpr int g = decltype(gg)::value;
                    f32x4_t x = lds_ld4f_o<32 * g>(xb);
                    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(x));
#pragma unroll
                    for (int t = 0; t < 4; t++) {
                        const float v = fmaf(-2.f, acc[4 * g + t], x[t]);
                        m = fminf(m, v);
                        if (vw != 0xFFFFFFFFu) acc[4 * g + t] = ((vl >> (8 * g + t)) & 1u) ? v : __builtin_inff();
                    }
                });
                if (vw != 0xFFFFFFFFu) {  // partial block: min over the valid rows only
                    m = __builtin_inff();
#pragma unroll
                    for (int r = 0; r < 16; r++) m = fminf(m, acc[r]);
                }
                const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
                m = fminf(m, __uint_as_float(sw[1]));
            } else {
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
        slot = slot == QS_NBUF - 1 ? 0 : slot + 1;
    }
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
    int cnt;
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int r = 0; r < R; r++) { key[r] = __builtin_inff(); id[r] = NO_ID; }
        thr = __builtin_inff();
        cnt = 0;
    }
    __device__ __forceinline__ void merge(const float* bk, const uint32_t* bi, int lane) {
        key[R - 1] = lane < cnt ? bk[lane] : __builtin_inff();
        id[R - 1] = lane < cnt ? bi[lane] : NO_ID;
        bitonic_sort<R>(key, id, lane);
        thr = __shfl(key[R - 2], 63);
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
                                                    float* __restrict__ eps_out) {
    constexpr int L = 64 * (R - 1);
    constexpr int U = 16;
    __shared__ float sbk[4][64];
    __shared__ uint32_t sbi[4][64];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int q = blockIdx.x * 4 + w;
    if (q >= nq) return;
    const float4 qi = qinfo[q];
    const float eps = qs_eps(metric, qi, qsmax, maxn2, gd, gacc);
    const float* kr = key + (int64_t)q * ldk;
    WaveTopL<R> t;
    t.init();
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
        if (!__any(any)) continue;
#pragma unroll
        for (int j = 0; j < U; j++) t.offer(v[j], (uint32_t)(b0 + j * 64 + lane), sbk[w], sbi[w], lane);
    }
    t.merge(sbk[w], sbi[w], lane);
    // M = A of the (k+1)-th smallest block key; T = M + 2 eps
    const float mk = t.key_at(k);
    const float M = qs_key_to_a(metric, mk, qi.x);
    const float T = mk == __builtin_inff() ? __builtin_inff() : M + 2.0005f * eps;
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
        // the L-th entry also qualifies: blocks beyond the list may too
        flags[q] = (nc >= L || qi.w != 0.f) ? 2 : 0;
    }
}

// k_blk_exact<R, METRIC, VARIANT>: wave per query over its candidate blocks
// (two blocks per pass: lanes 0-31 and 32-63, lane = row).  Reference-order
// SingleDist of every valid row, top-(k+1) by (distance, id); proof = the
// first min(k+1, n) are strictly increasing (the reference heap then holds
// exactly the k smallest and extractHeap returns them ascending).
template <int R, int METRIC, int VARIANT>
__global__ __launch_bounds__(256) void k_blk_exact(const float* __restrict__ X, int dpad, const uint32_t* __restrict__ valid,
                                                   int64_t nrows, const float* __restrict__ Qn, int d,
                                                   const uint32_t* __restrict__ cand, const int32_t* __restrict__ ncand,
                                                   int nq, int k, int kout, uint64_t id_base, uint64_t* __restrict__ out_ids,
                                                   float* __restrict__ out_d, int32_t* __restrict__ out_n,
                                                   int32_t* __restrict__ flags) {
    constexpr int L = 64 * (R - 1);
    __shared__ float sbk[4][64];
    __shared__ uint32_t sbi[4][64];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int q = blockIdx.x * 4 + w;
    if (q >= nq) return;
    if (flags[q]) return;  // overflowed selection: the replay resolves it
    const int nc = ncand[q];
    const float* qv = Qn + (int64_t)q * dpad;
    const int li = lane & 31, lh = lane >> 5;
    WaveTopL<R> t;
    t.init();
    int nvalid = 0;
    for (int j0 = 0; j0 < nc; j0 += 2) {
        const int j = j0 + lh;
        bool ok = false;
        int64_t row = 0;
        if (j < nc) {
            row = (int64_t)cand[(int64_t)q * L + j] * 32 + li;
            ok = row < nrows && ((valid[row >> 5] >> (row & 31)) & 1u);
        }
        float e = __builtin_inff();
        if (ok) e = exact_dist<METRIC, VARIANT>(qv, X + row * dpad, d);
        nvalid += __popcll(__ballot(ok));
        t.offer(ok ? e : __builtin_inff(), ok ? (uint32_t)row : NO_ID, sbk[w], sbi[w], lane);
    }
    t.merge(sbk[w], sbi[w], lane);
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

// flagged queries -> list (order irrelevant: every listed query is replayed
// independently); counters[0] += count, counters[1] = count (this batch)
__global__ void k_flag_list(const int32_t* __restrict__ flags, int nq, int32_t* __restrict__ qlist,
                            uint32_t* __restrict__ counters) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const bool f = q < nq && flags[q] != 0;
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
template <int METRIC, int VARIANT>
__global__ __launch_bounds__(64) void k_blk_replay(const float* __restrict__ key, int64_t ldk, int64_t nb,
                                                   const float* __restrict__ eps_q, const float4* __restrict__ qinfo,
                                                   const float* __restrict__ X, int dpad, const uint32_t* __restrict__ valid,
                                                   int64_t nrows, const float* __restrict__ Qn, int d,
                                                   const int32_t* __restrict__ qlist, const uint32_t* __restrict__ counters,
                                                   int k, int kout, uint64_t id_base, uint64_t* __restrict__ out_ids,
                                                   float* __restrict__ out_d, int32_t* __restrict__ out_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char rsm[];
    uint64_t* hid = reinterpret_cast<uint64_t*>(rsm);
    float* s_d = reinterpret_cast<float*>(hid + k);
    float* hd = s_d + 64;
    int* s_len = reinterpret_cast<int*>(hd + k);
    const int lane = threadIdx.x;
    if ((uint32_t)blockIdx.x >= counters[1]) return;
    const int q = qlist[blockIdx.x];
    const int metric = METRIC == COSINE ? COSINE : METRIC == DOT ? DOT : L2;
    const float4 qi = qinfo[q];
    const bool noskip = qi.w != 0.f;
    const float eps = eps_q[q];
    const float* kr = key + (int64_t)q * ldk;
    const float* qv = Qn + (int64_t)q * dpad;
    const int li = lane & 31, lh = lane >> 5;
    if (lane == 0) *s_len = 0;
    __syncthreads();
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
            // next one or two blocks still able to insert under the current top
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
            const bool ok = jj >= 0 && row < nrows && ((valid[row >> 5] >> (row & 31)) & 1u);
            const float dist = ok ? exact_dist<METRIC, VARIANT>(qv, X + row * dpad, d) : 0.f;
            uint64_t mask = __ballot(ok && (len < k || top > dist));
            if (mask == 0) continue;
            s_d[lane] = dist;
            __syncthreads();
            if (lane == 0) {
                ReplayHeap h{hid, hd, *s_len};
                while (mask) {
                    const int l = __builtin_ctzll(mask);
                    mask &= mask - 1;
                    const float dj = s_d[l];
                    const int jb = l >= 32 ? j2 : j1;
                    const uint64_t idj = id_base + (uint64_t)((b0 + jb) * 32 + (l & 31));
                    if (h.len < k) rh_insert(h, idj, dj);
                    else if (h.dist[0] > dj) { uint64_t x; float y; rh_pop(h, &x, &y); rh_insert(h, idj, dj); }
                }
                *s_len = h.len;
            }
            __syncthreads();
        }
    }
    if (lane == 0) {
        ReplayHeap h{hid, hd, *s_len};
        const int n = h.len;
        for (int i = n - 1; i >= 0; i--) {
            uint64_t x; float y;
            rh_pop(h, &x, &y);
            if (i < kout) { out_ids[(int64_t)q * kout + i] = x; out_d[(int64_t)q * kout + i] = y; }
        }
        out_n[q] = n < kout ? n : kout;
    }
}

}  // namespace wv
