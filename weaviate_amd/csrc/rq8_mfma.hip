// rq8_mfma.hip -- flat "rq-8" search on the integer matrix cores (DESIGN.md
// §3.7b), without the B x N distance matrix.
//
// The reference's rq-8 distance (DistanceBetweenCompressedVectors,
// compressionhelpers/rotational_quantization.go:294-306) is a float expression
// of per-vector metadata and one exact integer, dotByteImpl(x, y) = sum x_i y_i
// over the code bytes (:294).  The data codes are stored offset by 128
// (x' = x - 128 as int8, k_rq_encode); with y' = y - 128 for the query,
//     sum x y = sum x'y' + 128 (Sx + Sy) - 16384 D
// exactly in int32 (|terms| < 2^31 for D <= 4096), so one
// v_mfma_i32_16x16x64_i8 chain plus the two code sums is the reference's
// integer bit for bit, and the epilogue is the reference's float expression
// in its order, unfused (-ffp-contract=off).  Three kernels:
//   k_rq8_keys  the exact rq-8 distance of every (query, row) of a 32-row
//               block, reduced in registers to the block minimum (a NaN
//               distance -> -inf: its block is always a candidate and the
//               query is replayed)
//   k_rq8_sel   wave per query: M = the (R+1)-th smallest block minimum;
//               candidates = every block with minimum <= M -- they hold every
//               row with distance < M and at least R+1 rows <= M
//   k_rq8_cand  wave per query: exact distances of the candidates' rows
//               (v_dot4_u32_u8, as k_rq8_dist), the R+1 smallest.  With no tie
//               among them and no NaN, the reference heap's survivors
//               (flat/index.go:470-487: the R smallest) and its pop order
//               (descending) follow from the distances alone: the ascending
//               list goes to ascI / ascD / ascN.  Otherwise the query is
//               flagged and replayed exactly (k_rq8_dist + k_replay_scan).
#pragma once

namespace wv {

// k_rq8_keys operands (external linkage: quant_runtime.hip launches it)
struct RQ8Args {
    const unsigned char* codes;  // data codes x' (32-row tiles of 16-byte chunks, rq_tile_u4)
    const float4* meta;          // [cap] {lower, step, step * codeSum, norm2}
    const uint32_t* csum;        // [cap] code sums Sx
    const uint32_t* valid;       // [cap / 32] slots to scan
    const unsigned char* Qp;     // [nq_pad][D] query codes y' (int8), rows past nq zero
    const float4* qmeta;         // [nq_pad]
    const uint32_t* qcsum;       // [nq_pad] Sy
    float* key;                  // [nq_pad][ldk] block minima
    int64_t ldk;
    int64_t nblk;                // 32-row blocks to scan
    int blocks_per_span;
    int nspans;
    int nqg;                     // query groups of 256
    float fl2, fcos;             // L2: 1, 0; cosine: 0, 1; dot: 0, 0 (rq_dist's)
    int dbg_serial;              // debug option rq_serial: one block in flight, drained before each barrier
};

namespace {

// query codes of the group-tiled rq-8 layout -> Qp row q (y ^ 0x80 = y - 128
// as int8) and the code sum; wave per query, rows [nq, nq_pad) zero
__global__ __launch_bounds__(256) void k_rq8_qprep(const uint4* __restrict__ qcodes, int D, int64_t nq,
                                                   int64_t nq_pad, unsigned char* __restrict__ Qp,
                                                   uint32_t* __restrict__ qcsum) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq_pad) return;
    const int nch = D >> 4;
    uint32_t s = 0;
    for (int c = lane; c < nch; c += 64) {
        uint4 y = make_uint4(0u, 0u, 0u, 0u);
        if (q < nq) y = qcodes[((q / RQ_QPB) * nch + c) * RQ_QPB + (q % RQ_QPB)];
        s = __builtin_amdgcn_udot4(y.x, 0x01010101u, s, false);
        s = __builtin_amdgcn_udot4(y.y, 0x01010101u, s, false);
        s = __builtin_amdgcn_udot4(y.z, 0x01010101u, s, false);
        s = __builtin_amdgcn_udot4(y.w, 0x01010101u, s, false);
        const uint32_t X = q < nq ? 0x80808080u : 0u;
        *reinterpret_cast<uint4*>(Qp + q * D + 16 * c) = make_uint4(y.x ^ X, y.y ^ X, y.z ^ X, y.w ^ X);
    }
    s = wave_sum_u32(s);
    if (lane == 0) qcsum[q] = s;
}

// rq-1 query planes (group-tiled, 5 per 64-bit word) -> Qp row q: per dim
// w_i = sum_p 2^p (1 - 2 bit_pi) = 31 - 2 c_i (c_i the 5-bit code), or 0 for a
// query encoded as zero (qmeta.z == 0: the reference's dot is 0 then); thread
// per (query, 16 dims)
__global__ void k_rq1_qprep(const uint64_t* __restrict__ planes, const float4* __restrict__ qmeta, int D,
                            int64_t nq, int64_t nq_pad, unsigned char* __restrict__ Qp) {
    const int nch = D >> 4, W = D >> 6;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq_pad * nch) return;
    const int64_t q = i / nch;
    const int c = (int)(i % nch);
    uint32_t wd[4] = {0u, 0u, 0u, 0u};
    if (q < nq && qmeta[q].z != 0.f) {
        const int w = c >> 2, sh = 16 * (c & 3);
        uint32_t pl[5];
#pragma unroll
        for (int p = 0; p < 5; p++)
            pl[p] = (uint32_t)(planes[(((q / RQ_QPB) * W + w) * 5 + p) * RQ_QPB + (q % RQ_QPB)] >> sh) & 0xFFFFu;
#pragma unroll
        for (int b = 0; b < 16; b++) {
            int cc = 0;
#pragma unroll
            for (int p = 0; p < 5; p++) cc |= (int)((pl[p] >> b) & 1u) << p;
            wd[b >> 2] |= (uint32_t)(unsigned char)(signed char)(31 - 2 * cc) << (8 * (b & 3));
        }
    }
    *reinterpret_cast<uint4*>(Qp + q * D + 16 * c) = make_uint4(wd[0], wd[1], wd[2], wd[3]);
}

__device__ __forceinline__ uint32_t rq8_lds_ld4(unsigned addr) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(addr));
    return v;
}

// ring slots of k_rq8_keys: as many as 150 KiB of LDS holds, 4..8
__host__ __device__ constexpr int rq8_nbuf(int NC) {
    return (150 * 1024) / (32 * 64 * NC + 656) > 8 ? 8 : (150 * 1024) / (32 * 64 * NC + 656) < 4 ? 4
                                                                                              : (150 * 1024) / (32 * 64 * NC + 656);
}

// ---------------------------------------------------------------------------
// k_rq8_keys<NC>: block minima of 256 queries (8 waves x 32, their codes in
// VGPRs as B fragments) x one span of 32-row blocks, D = 64 NC.  A block's
// codes (32 D bytes: 2 NC 1-KiB pieces, [16-byte chunk][row]), meta, code sums
// and valid word land in an LDS ring of rq8_nbuf(NC) slots by LDS-DMA
// NBUF - 2 blocks ahead (as much in flight as 150 KiB of LDS holds);
// one barrier per block.  Per 64-column chunk: 2 A-fragment reads (row halves,
// the next chunk's issued before this chunk's MFMAs), 4 MFMAs.  acc[m][n][r]
// is row 16m + 4g + r (g = lane >> 4) of query 16n + (lane & 15); the C input
// of the first chunk is 128 Sy, the epilogue adds 128 Sx - 16384 D.
// ---------------------------------------------------------------------------
template <int NC, int BITS>
__global__ __launch_bounds__(512, 2) void k_rq8_keys(RQ8Args a) {
    constexpr int D = 64 * NC;
    constexpr int NCH = 4 * NC;         // 16-byte chunks per row
    constexpr int CB = 32 * D;          // code bytes per block
    constexpr int MB = CB;              // meta: 32 x 16 B
    constexpr int SB = CB + 512;        // code sums: 32 x 4 B
    constexpr int VB = CB + 640;        // valid word
    constexpr int SLOT = CB + 656;
    constexpr int NP = 2 * NC + 3;      // wave-wide loads per block
    constexpr int PW = (NP + 7) / 8;    // per wave (padded: every wave issues PW)
    // a late wave reads block t-1's meta while block t + AHEAD lands
    constexpr int NBUF = rq8_nbuf(NC);
    constexpr int AHEAD = NBUF - 2;
    static_assert(SLOT % 16 == 0, "slot alignment");
    static_assert((NC - 1) * 2048 + 256 < 65536, "ds_read offsets");
    extern __shared__ __attribute__((aligned(16))) unsigned char rsm[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int total = a.nqg * a.nspans;
    const int b = blockIdx.x;
    // XCD-aware order: the query groups of one span share an XCD (its L2)
    const int logical = (total % 8 == 0) ? (b % 8) * (total / 8) + (b / 8) : b;
    const int span = logical / a.nqg, grp = logical % a.nqg;
    const int j = lane & 15, g = lane >> 4;
    const int64_t q0 = (int64_t)grp * 256 + wave * 32;
    static_assert(BITS == 8 || BITS == 1, "rq-8 or rq-1");

    // Qf[2c + n]: query q0 + 16n + j, columns 64c + 16g .. +15
    i32x4_t Qf[2 * NC];
    {
        const unsigned char* qp = a.Qp + (q0 + j) * D + 16 * g;
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int n = 0; n < 2; n++)
                Qf[2 * c + n] = *reinterpret_cast<const i32x4_t*>(qp + (int64_t)n * 16 * D + 64 * c);
    }
    float4 ym[2];
    i32x4_t C0[2];
#pragma unroll
    for (int n = 0; n < 2; n++) {
        ym[n] = a.qmeta[q0 + 16 * n + j];
        const int ky = BITS == 8 ? (int)(128u * a.qcsum[q0 + 16 * n + j]) : 0;
        C0[n] = i32x4_t{ky, ky, ky, ky};
    }
    // the fast epilogue: every product of the reference's expression stays far
    // from overflow when both squared norms are <= 1e16 (|components| <= 1e8),
    // so no NaN can arise, and 0 (n2x + n2y) + fcos == fcos for cosine / dot
    constexpr float FINE = 1e16f;
    const bool qfine = BITS == 8 ? (ym[0].w <= FINE && ym[1].w <= FINE) : (ym[0].y <= FINE && ym[1].y <= FINE);
    const bool l2 = a.fl2 != 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the query loads retire before the DMA ring

    const int64_t b0 = (int64_t)span * a.blocks_per_span;
    int64_t b1 = b0 + a.blocks_per_span;
    if (b1 > a.nblk) b1 = a.nblk;
    const int nsteps = b1 > b0 ? (int)(b1 - b0) : 0;
    const unsigned ring = lds_addr(rsm);
    auto issue = [&](int t, int slot) {
        const int64_t blk = b0 + t;
        const unsigned char* gb = a.codes + blk * CB;  // the block's contiguous run (rq_tile_u4)
        const unsigned sb = ring + (unsigned)(slot * SLOT);
        static_for<0, PW>([&](auto jc) {
            constexpr int jj = decltype(jc)::value;
            int p = wave + 8 * jj;
            if (p >= NP) p -= NP;  // padding: a copy of a piece another wave loads (same bytes, same place)
            if (p < 2 * NC) {
                __builtin_amdgcn_global_load_lds(gb + p * 1024 + 16 * lane, (lds_ptr_t)(size_t)(sb + (unsigned)(p * 1024)),
                                                 16, 0, 0);
            } else if (p == 2 * NC) {
                if (lane < 32)
                    __builtin_amdgcn_global_load_lds(a.meta + blk * 32 + lane, (lds_ptr_t)(size_t)(sb + MB), 16, 0, 0);
            } else if (p == 2 * NC + 1) {
                if (lane < 8)
                    __builtin_amdgcn_global_load_lds(a.csum + blk * 32 + 4 * lane, (lds_ptr_t)(size_t)(sb + SB), 16, 0,
                                                     0);
            } else {
                if (lane == 0)
                    __builtin_amdgcn_global_load_lds(a.valid + blk, (lds_ptr_t)(size_t)(sb + VB), 4, 0, 0);
            }
        });
    };
    const int ahead = (a.dbg_serial & 1) ? 1 : AHEAD;
    for (int t = 0; t < ahead && t < nsteps; t++) issue(t, t);

    const unsigned l16 = (unsigned)(g * 512 + j * 16);
    float* krow = a.key + (q0 + (lane & 31)) * a.ldk;
    const float fD = (float)D;
    const float s_ = 1.0f + a.fl2;
    // Waves 4-7 (each the SIMD partner of wave w - 4) run block t-1's
    // epilogue before block t's MFMAs instead of after them, so the two
    // waves of a SIMD alternate MFMA and VALU phases (MI355X_MICROARCH.md, two
    // waves per SIMD: a stagger) instead of issuing both at once.
    const bool late = wave >= 4 && !(a.dbg_serial & 2);
    i32x4_t acc[2][2];
    float pend = 0.f;  // an early wave's key of the previous block, stored after the next barrier
    auto mfma_block = [&](unsigned sb) {
        const unsigned ab = sb + l16;
        i32x4_t A[2][2];
        A[0][0] = lds_ld16_o<0>(ab);
        A[0][1] = lds_ld16_o<256>(ab);
        static_for<0, NC>([&](auto cc) {
            constexpr int c = decltype(cc)::value;
            if constexpr (c + 1 < NC) {
                A[(c + 1) & 1][0] = lds_ld16_o<(c + 1) * 2048>(ab);
                A[(c + 1) & 1][1] = lds_ld16_o<(c + 1) * 2048 + 256>(ab);
                qs_wait_lgkm<2>();
            } else {
                qs_wait_lgkm<0>();
            }
            asm volatile("" : "+v"(A[c & 1][0]), "+v"(A[c & 1][1]));
            __builtin_amdgcn_sched_barrier(0);
            if (a.dbg_serial & 16) {  // timing experiment: no MFMAs (wrong keys)
                acc[0][0] = A[c & 1][0];
                acc[1][1] = A[c & 1][1];
                return;
            }
#pragma unroll
            for (int m = 0; m < 2; m++)
#pragma unroll
                for (int n = 0; n < 2; n++)
                    acc[m][n] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[c & 1][m], Qf[2 * c + n],
                                                                      c == 0 ? C0[n] : acc[m][n], 0, 0, 0);
        });
    };
    // a block's epilogue (its meta in slot sb, its sums in acc) -> the lane's
    // key of it (lanes 0-31)
    auto epilogue = [&](unsigned sb) -> float {
        // the lane's rows 16m + 4g + r: meta, code sums; the block's valid word
        i32x4_t mt[2][4], cs[2];
        const unsigned mb = sb + MB + (unsigned)(g * 64);
        mt[0][0] = lds_ld16_o<0>(mb);
        mt[0][1] = lds_ld16_o<16>(mb);
        mt[0][2] = lds_ld16_o<32>(mb);
        mt[0][3] = lds_ld16_o<48>(mb);
        mt[1][0] = lds_ld16_o<256>(mb);
        mt[1][1] = lds_ld16_o<272>(mb);
        mt[1][2] = lds_ld16_o<288>(mb);
        mt[1][3] = lds_ld16_o<304>(mb);
        const unsigned cb = sb + SB + (unsigned)(g * 16);
        cs[0] = lds_ld16_o<0>(cb);
        cs[1] = lds_ld16_o<64>(cb);
        uint32_t vw0 = rq8_lds_ld4(sb + VB);
        qs_wait_lgkm<0>();
        // the loaded registers are defined only after the wait: tie them to it,
        // or the compiler may schedule their uses above it
        asm volatile("" : "+v"(mt[0][0]), "+v"(mt[0][1]), "+v"(mt[0][2]), "+v"(mt[0][3]), "+v"(vw0));
        asm volatile("" : "+v"(mt[1][0]), "+v"(mt[1][1]), "+v"(mt[1][2]), "+v"(mt[1][3]));
        asm volatile("" : "+v"(cs[0]), "+v"(cs[1]));
        const uint32_t vw = __builtin_amdgcn_readfirstlane(vw0);
        if (a.dbg_serial & 8) return __int_as_float(acc[0][0][0] ^ acc[1][1][3] ^ mt[0][0][0] ^ cs[1][0]);  // timing: no epilogue math
        float p[2] = {__builtin_inff(), __builtin_inff()};
        bool bad[2] = {false, false};
        // the fast forms: every row valid, every norm <= FINE (wave-uniform);
        // l2: (1 (n2x + n2y) + 0) - 2 est, cosine / dot: (0 (..) + fcos) - 1 est
        bool fine = qfine;
    #pragma unroll
        for (int m = 0; m < 2; m++)
    #pragma unroll
            for (int r = 0; r < 4; r++) fine = fine && __int_as_float(mt[m][r][BITS == 8 ? 3 : 1]) <= FINE;
        const int mode = (vw == 0xFFFFFFFFu && __all(fine) && !(a.dbg_serial & 4)) ? (l2 ? 0 : 1) : 2;
        if (mode != 2 && !(a.dbg_serial & 32)) {
            // the fast forms on packed fp32 (v_pk_mul_f32 / v_pk_add_f32: the
            // two query halves n = 0, 1 of a row in one instruction, each
            // element rounded as the scalar op would).  cosine / dot: fl(fcos -
            // est) falls as est grows, so the block's minimum is fcos - (the
            // maximum est) and the subtraction moves out of the row loop.
            const f32x2_t yx = {ym[0].x, ym[1].x}, yz = {ym[0].z, ym[1].z};
            const f32x2_t yyv = {BITS == 8 ? ym[0].y : ym[0].x, BITS == 8 ? ym[1].y : ym[1].x};
            const f32x2_t ynv = {BITS == 8 ? ym[0].w : ym[0].y, BITS == 8 ? ym[1].w : ym[1].y};
            f32x2_t best = {mode == 0 ? __builtin_inff() : -__builtin_inff(), mode == 0 ? __builtin_inff() : -__builtin_inff()};
    #pragma unroll
            for (int m = 0; m < 2; m++)
    #pragma unroll
                for (int r = 0; r < 4; r++) {
                    f32x2_t est;
                    float xnorm;
                    if constexpr (BITS == 8) {
                        const float xl = __int_as_float(mt[m][r][0]);
                        const float xs = __int_as_float(mt[m][r][1]);
                        const float xz = __int_as_float(mt[m][r][2]);
                        xnorm = __int_as_float(mt[m][r][3]);
                        const float a1 = fD * xl;
                        const int kx = (int)(128u * (uint32_t)cs[m][r]) - 16384 * D;
                        const f32x2_t dotv = {(float)(uint32_t)(acc[m][0][r] + kx), (float)(uint32_t)(acc[m][1][r] + kx)};
                        const f32x2_t e1 = f32x2_t{a1, a1} * yx;
                        const f32x2_t e2 = f32x2_t{xl, xl} * yz;
                        const f32x2_t e3 = yx * f32x2_t{xz, xz};
                        f32x2_t e4 = f32x2_t{xs, xs} * yyv;
                        e4 = e4 * dotv;
                        est = ((e1 + e2) + e3) + e4;
                    } else {
                        const float xs = __int_as_float(mt[m][r][0]);
                        xnorm = __int_as_float(mt[m][r][1]);
                        const f32x2_t accv = {(float)acc[m][0][r], (float)acc[m][1][r]};
                        est = (yyv * f32x2_t{xs, xs}) * accv;
                    }
                    if (mode == 0) {
                        const f32x2_t v = (f32x2_t{xnorm, xnorm} + ynv) - f32x2_t{2.0f, 2.0f} * est;
                        best[0] = fminf(best[0], v[0]);
                        best[1] = fminf(best[1], v[1]);
                    } else {
                        best[0] = fmaxf(best[0], est[0]);
                        best[1] = fmaxf(best[1], est[1]);
                    }
                }
            if (mode == 1) {
                p[0] = a.fcos - best[0];
                p[1] = a.fcos - best[1];
            } else {
                p[0] = best[0];
                p[1] = best[1];
            }
        } else
    #pragma unroll
        for (int m = 0; m < 2; m++)
    #pragma unroll
            for (int r = 0; r < 4; r++) {
                const bool ok = (vw >> (16 * m + 4 * g + r)) & 1u;
                float est[2], xnorm;
                if constexpr (BITS == 8) {
                    // est = ((D lx ly + lx cy) + ly cx) + sx sy dot (the reference's order)
                    const float xl = __int_as_float(mt[m][r][0]);
                    const float xs = __int_as_float(mt[m][r][1]);
                    const float xz = __int_as_float(mt[m][r][2]);
                    xnorm = __int_as_float(mt[m][r][3]);
                    const float a1 = fD * xl;
                    const int kx = (int)(128u * (uint32_t)cs[m][r]) - 16384 * D;
    #pragma unroll
                    for (int n = 0; n < 2; n++) {
                        const uint32_t dot = (uint32_t)(acc[m][n][r] + kx);
                        float e1 = a1 * ym[n].x;
                        const float e2 = xl * ym[n].z;
                        const float e3 = ym[n].x * xz;
                        float e4 = xs * ym[n].y;
                        e4 = e4 * (float)dot;
                        float e = e1 + e2;
                        e = e + e3;
                        est[n] = e + e4;
                    }
                } else {
                    // rq-1 (BinaryRQDistancer.Distance, binary_rotational_quantization.go:364-385):
                    // acc = sum s_x w_q = 31 qdim - sum_p 2^(p+1) popcount(x ^ plane_p) exactly
                    const float xs = __int_as_float(mt[m][r][0]);
                    xnorm = __int_as_float(mt[m][r][1]);
    #pragma unroll
                    for (int n = 0; n < 2; n++) {
                        const float e = ym[n].x * xs;
                        est[n] = e * (float)acc[m][n][r];
                    }
                }
    #pragma unroll
                for (int n = 0; n < 2; n++) {
                    const float yn = BITS == 8 ? ym[n].w : ym[n].y;
                    if (mode == 0) {
                        p[n] = fminf(p[n], (xnorm + yn) - 2.0f * est[n]);
                    } else if (mode == 1) {
                        p[n] = fminf(p[n], a.fcos - est[n]);
                    } else {
                        float tt = a.fl2 * (xnorm + yn);
                        tt = tt + a.fcos;
                        const float dist = tt - s_ * est[n];
                        bad[n] = bad[n] || (ok && dist != dist);
                        p[n] = fminf(p[n], ok ? dist : __builtin_inff());
                    }
                }
                __builtin_amdgcn_sched_barrier(0);  // one row at a time: bounds the live temporaries
            }
    #pragma unroll
        for (int n = 0; n < 2; n++)
            if (bad[n]) p[n] = -__builtin_inff();
        // minimum over the 4 row groups: lanes j, j + 16, j + 32, j + 48
        // (ds_bpermute, which the compiler's hazard and wait tracking covers)
        float m0 = p[0], m1 = p[1];
        m0 = fminf(m0, __shfl_xor(m0, 32));
        m1 = fminf(m1, __shfl_xor(m1, 32));
        m0 = fminf(m0, __shfl_xor(m0, 16));
        m1 = fminf(m1, __shfl_xor(m1, 16));
        // lanes 0-15: queries j (m0); lanes 16-31: queries 16 + j (m1)
        return (lane & 16) ? m1 : m0;
    };
    for (int t = 0; t <= nsteps; t++) {
        const int cur = t % NBUF;
        if (t < nsteps) {
            // block t's pieces landed: vector-memory ops retire in issue order
            // (loads, stores and LDS-DMA alike), so the wait leaves in flight
            // exactly the ops issued after them: the pieces of the blocks up to
            // t + ahead - 1 and the key stores of the steps since (an early
            // wave stores before its step's pieces, a late wave after them).
            // Counting the stores keeps the scattered key writes out of the
            // critical path.
            const int later = nsteps - 1 - t < ahead - 1 ? nsteps - 1 - t : ahead - 1;  // blocks issued after t
            const int fs = t < ahead ? 1 : (late ? (t - ahead > 1 ? t - ahead : 1) : (t - ahead + 1 > 1 ? t - ahead + 1 : 1));
            const int nst = t > fs ? t - fs : 0;  // the stores of steps fs .. t-1
            qs_wait_vm(PW * later + nst);
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if (!late && t > 0 && lane < 32) krow[b0 + t - 1] = pend;
            if (t + ahead < nsteps) issue(t + ahead, (t + ahead) % NBUF);
        }
        if (!late) {
            if (t < nsteps) {
                mfma_block(ring + (unsigned)(cur * SLOT));
                pend = epilogue(ring + (unsigned)(cur * SLOT));
            }
        } else {
            if (t > 0) {
                const float kv = epilogue(ring + (unsigned)(((t - 1) % NBUF) * SLOT));
                if (lane < 32) krow[b0 + t - 1] = kv;
            }
            if (t < nsteps) mfma_block(ring + (unsigned)(cur * SLOT));
        }
    }
    if (!late && nsteps > 0 && lane < 32) krow[b0 + nsteps - 1] = pend;
}

// ---------------------------------------------------------------------------
// k_rq8_sel<RT>: wave per query (4 per block).  The 64 (RT - 1) >= R + 2
// smallest block minima (WaveTopL), M = the (R+1)-th; cand[q] = the blocks with
// minimum <= M (a sorted prefix of the list).  oflag[q] = 1 when the list's
// last entry is still <= M (ties at M may run past it): the query is replayed.
// ---------------------------------------------------------------------------
template <int RT>
__global__ __launch_bounds__(256) void k_rq8_sel(const float* __restrict__ key, int64_t ldk, int64_t nb, int nq, int R,
                                                 uint32_t* __restrict__ cand, int Lc, int32_t* __restrict__ ncand,
                                                 int32_t* __restrict__ oflag) {
    constexpr int U = 16;
    __shared__ float sbk[4][64];
    __shared__ uint32_t sbi[4][64];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int q = blockIdx.x * 4 + w;
    if (q >= nq) return;
    const float* kr = key + (int64_t)q * ldk;
    WaveTopL<RT> t;
    t.init();
    for (int64_t c0 = 0; c0 < nb; c0 += 64 * U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t bb = c0 + u * 64 + lane;
            v[u] = bb < nb ? kr[bb] : __builtin_inff();
        }
        bool any = false;
#pragma unroll
        for (int u = 0; u < U; u++) any |= v[u] < t.thr;
        if (!__any(any)) continue;
#pragma unroll
        for (int u = 0; u < U; u++) t.offer(v[u], (uint32_t)(c0 + u * 64 + lane), sbk[w], sbi[w], lane);
    }
    t.merge(sbk[w], sbi[w], lane);
    const float M = t.key_at(R);
    int cnt = 0;
    bool last_in = false;
#pragma unroll
    for (int r = 0; r < RT - 1; r++) {
        const bool in = t.key[r] <= M && t.key[r] < __builtin_inff();
        const uint64_t bm = __ballot(in);
        const int pos = cnt + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0));
        if (in && pos < Lc) cand[(int64_t)q * Lc + pos] = t.id[r];
        cnt += __popcll(bm);
        if (r == RT - 2) last_in = (bm >> 63) & 1ull;
    }
    if (lane == 0) {
        ncand[q] = cnt < Lc ? cnt : Lc;
        oflag[q] = last_in ? 1 : 0;
    }
}

// the exact rq-8 / rq-1 distance of stored row `slot` to one query, as
// k_rq8_dist / k_rq1_dist compute it: rq-8 v_dot4_u32_u8 over the code bytes
// (stored offset by 128) against the query's bytes (qs, LDS), rq-1 xor +
// popcount of the word-major bits against the 5 query planes (qs as u64)
template <int BITS>
__device__ __forceinline__ float rq_row_dist(const void* __restrict__ codes_, int64_t cap,
                                             const float4* __restrict__ meta, int64_t slot, const uint4* qs,
                                             const float4& ym, int D, float fl2, float fcos) {
    const float s_ = 1.0f + fl2;
    if constexpr (BITS == 1) {
        const uint64_t* codes = reinterpret_cast<const uint64_t*>(codes_);
        const uint64_t* qpl = reinterpret_cast<const uint64_t*>(qs);
        const int W = D >> 6;
        uint32_t acc = 0;
#pragma unroll 8
        for (int wd = 0; wd < W; wd++) {
            const uint64_t x = codes[(int64_t)wd * cap + slot];
            const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
#pragma unroll
            for (int p = 0; p < 5; p++) {
                const uint64_t y = qpl[5 * wd + p];
                uint32_t h = __builtin_popcount(xl ^ (uint32_t)y);
                h += __builtin_popcount(xh ^ (uint32_t)(y >> 32));
                acc += h << (p + 1);
            }
        }
        const int qdim = (int)ym.z;
        const int dot = qdim > 0 ? 31 * qdim - (int)acc : 0;
        const float4 xm = meta[slot];
        float est = ym.x * xm.x;
        est = est * (float)dot;
        float tt = fl2 * (xm.y + ym.y);
        tt = tt + fcos;
        return tt - s_ * est;
    } else {
        const int nch = D >> 4;
        const uint4* xr = reinterpret_cast<const uint4*>(codes_) + rq_tile_u4(slot, 0, nch);
        uint32_t acc = 0;
        // 16 chunk loads in flight at a time (nch is a multiple of 4): the row's
        // bytes are 16 scattered 16-byte pieces per group, latency-bound otherwise
#pragma unroll 16
        for (int c = 0; c < nch; c++) {
            const uint4 x = xr[(int64_t)c * 32];
            const uint4 y = qs[c];
            acc = __builtin_amdgcn_udot4(x.x ^ 0x80808080u, y.x, acc, false);
            acc = __builtin_amdgcn_udot4(x.y ^ 0x80808080u, y.y, acc, false);
            acc = __builtin_amdgcn_udot4(x.z ^ 0x80808080u, y.z, acc, false);
            acc = __builtin_amdgcn_udot4(x.w ^ 0x80808080u, y.w, acc, false);
        }
        const float4 xm = meta[slot];
        float e1 = (float)D * xm.x;
        e1 = e1 * ym.x;
        const float e2 = xm.x * ym.z;
        const float e3 = ym.x * xm.z;
        float e4 = xm.y * ym.y;
        e4 = e4 * (float)acc;
        float est = e1 + e2;
        est = est + e3;
        est = est + e4;
        float tt = fl2 * (xm.w + ym.w);
        tt = tt + fcos;
        return tt - s_ * est;
    }
}

// a query's codes into LDS for rq_row_dist (wave-cooperative): rq-8 bytes
// y (Qp holds y ^ 0x80), rq-1 the 5 W planes of query gq (group-tiled)
template <int BITS>
__device__ __forceinline__ void rq_query_to_lds(uint4* qs, const void* __restrict__ qsrc, int64_t q, int64_t gq, int D,
                                                int lane) {
    if constexpr (BITS == 8) {
        const unsigned char* Qp = reinterpret_cast<const unsigned char*>(qsrc);
        for (int c = lane; c < (D >> 4); c += 64) {
            const uint4 y = *reinterpret_cast<const uint4*>(Qp + q * D + 16 * c);
            qs[c] = make_uint4(y.x ^ 0x80808080u, y.y ^ 0x80808080u, y.z ^ 0x80808080u, y.w ^ 0x80808080u);
        }
    } else {
        const uint64_t* planes = reinterpret_cast<const uint64_t*>(qsrc);
        uint64_t* qpl = reinterpret_cast<uint64_t*>(qs);
        const int W = D >> 6;
        for (int e = lane; e < 5 * W; e += 64)  // e = 5 w + p
            qpl[e] = planes[((gq / RQ_QPB) * W * 5 + e) * RQ_QPB + gq % RQ_QPB];
    }
}
__host__ __device__ constexpr int rq_query_lds_u4(int bits, int D) { return bits == 8 ? D / 16 : (5 * (D / 64) + 1) / 2; }

// ---------------------------------------------------------------------------
// k_rq8_cand<RT>: wave per query (4 per block), skipped when k_rq8_sel flagged
// it.  Lanes 0-31 / 32-63 take the rows of two candidate blocks at a time:
// the exact rq-8 distance as k_rq8_dist computes it (v_dot4_u32_u8 over the
// code bytes, the query's from LDS), offered to the wave's sorted
// 64 (RT - 1) >= R + 1 list.  No tie among the R + 1 smallest and no NaN: the
// R smallest ascending -> asc; else oflag[q] = 1.
// ---------------------------------------------------------------------------
// BITS = 1: rq-1's exact distance as k_rq1_dist computes it (xor + popcount of
// the word-major bit codes against the 5 query planes, copied to LDS from
// the group-tiled layout; query q of this launch is q_base + q there).
template <int RT, int BITS>
__global__ __launch_bounds__(256) void k_rq8_cand(const void* __restrict__ codes_, int64_t cap,
                                                  const float4* __restrict__ meta, const uint32_t* __restrict__ valid,
                                                  int64_t nslots, const void* __restrict__ qsrc, int64_t q_base,
                                                  const float4* __restrict__ qmeta, int D, float fl2, float fcos,
                                                  const uint32_t* __restrict__ cand, int Lc,
                                                  const int32_t* __restrict__ ncand, int nq, int R, uint64_t id_base,
                                                  uint64_t* __restrict__ ascI, float* __restrict__ ascD,
                                                  int32_t* __restrict__ ascN, int32_t* __restrict__ oflag) {
    // [4][D / 16] query code bytes (rq-8) or [4][5 W] planes (rq-1)
    extern __shared__ __attribute__((aligned(16))) uint4 cqs[];
    __shared__ float sbk[4][64];
    __shared__ uint32_t sbi[4][64];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int q = blockIdx.x * 4 + w;
    if (q >= nq) return;
    if (oflag[q]) {  // k_rq8_sel's overflow: replayed; no rescoring of this row before that
        if (lane == 0) ascN[q] = 0;
        return;
    }
    uint4* qs = cqs + w * rq_query_lds_u4(BITS, D);
    rq_query_to_lds<BITS>(qs, qsrc, q, q_base + q, D, lane);
    wave_sync_lds();
    const float4 ym = qmeta[q];
    const int nc = ncand[q];
    WaveTopL<RT> t;
    t.init();
    int nvalid = 0;
    bool nan = false;
    for (int i = 0; i < nc; i += 2) {
        const int bi = i + (lane >> 5);
        const bool has = bi < nc;
        const uint32_t blk = has ? cand[(int64_t)q * Lc + bi] : 0u;
        const int64_t slot = (int64_t)blk * 32 + (lane & 31);
        const bool ok = has && slot < nslots && ((valid[blk] >> (lane & 31)) & 1u);
        float dist = __builtin_inff();
        if (ok) {
            dist = rq_row_dist<BITS>(codes_, cap, meta, slot, qs, ym, D, fl2, fcos);
            nan = nan || dist != dist;
        }
        nvalid += __popcll(__ballot(ok));
        t.offer(dist, (uint32_t)slot, sbk[w], sbi[w], lane);
    }
    t.merge(sbk[w], sbi[w], lane);
    // a tie at the boundary (the R-th and (R+1)-th smallest) leaves the heap's
    // survivors to its insertion order: replayed (1).  A tie inside the R
    // leaves only their pop order open, which matters to the k-heap of the
    // rescored distances only if those tie as well: checked after the
    // rescoring (2, k_rq_tiecheck).
    const int nk = nvalid < R + 1 ? nvalid : R + 1;  // sorted entries that matter
    bool tie_b = false, tie_i = false;
#pragma unroll
    for (int r = 0; r < RT - 1; r++) {
        const float nx0 = __shfl(t.key[r], (lane + 1) & 63);
        const float nx1 = r + 1 < RT - 1 ? __shfl(t.key[r + 1 < RT - 1 ? r + 1 : r], 0) : __builtin_inff();
        const float nx = lane < 63 ? nx0 : nx1;
        const int e = r * 64 + lane;
        const bool eq = e + 1 < nk && t.key[r] == nx;
        tie_b = tie_b || (eq && e + 1 == R);
        tie_i = tie_i || (eq && e + 1 < R);
    }
    if (__any(tie_b) || __any(nan)) {
        if (lane == 0) {
            oflag[q] = 1;
            ascN[q] = 0;
        }
        return;
    }
    const bool tie_in = __any(tie_i);
    const int nout = nvalid < R ? nvalid : R;
#pragma unroll
    for (int r = 0; r < RT - 1; r++) {
        const int e = r * 64 + lane;
        if (e < nout) {
            ascI[(int64_t)q * R + e] = id_base + (uint64_t)t.id[r];
            ascD[(int64_t)q * R + e] = t.key[r];
        }
    }
    if (lane == 0) {
        ascN[q] = nout;
        if (tie_in) oflag[q] = 2;
    }
}

// queries k_rq8_cand left at 2 (equal quantized distances inside the R): the
// k-heap over the rescored distances (k_bq_final) depends on the feeding
// (pop) order only through equal rescored distances among its survivors: a
// value equal to another one and not above the k-th smallest (or a NaN) ->
// 3 (replayed), else 0.  Wave per query; lists longer than 2048 are replayed
// without the check.
__global__ __launch_bounds__(256) void k_rq_tiecheck(const float* __restrict__ candE, const int32_t* __restrict__ cnt,
                                                     int nq, int R, int k, int32_t* __restrict__ oflag) {
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq || oflag[q] != 2) return;
    const int n = cnt[q];
    const float* e = candE + (int64_t)q * R;
    bool dup = n > 2048;
    for (int i = lane; i < n && !dup; i += 64) {
        const float v = e[i];
        if (v != v) { dup = true; break; }
        int below = 0;
        bool eq = false;
        for (int j = 0; j < n; j++) {
            const float u = e[j];
            below += u < v ? 1 : 0;
            eq = eq || (j != i && u == v);
        }
        if (eq && below < k) dup = true;  // v is among the k smallest (with its equals)
    }
    const bool any = __any(dup);
    if (lane == 0) oflag[q] = any ? 3 : 0;
}

// ---------------------------------------------------------------------------
// k_rq8_replay<BITS>: the reference R-heap (searchByVectorQuantized,
// flat/index.go:470-487: insertToHeap in id order) of one listed query per
// 512-thread workgroup, without a distance matrix.  Windows of 512 32-row
// blocks in id order: a block is a candidate unless the heap is full and
// !(top > its exact minimum from k_rq8_keys) -- no row of it could pass
// `top.Dist > distance`, and the top never rises.  The candidates' rows get
// their exact distances (rq_row_dist) 16 blocks at a time, 2 per wave; lane 0
// then offers, in id order, the rows that pass against the top at that point
// (ph_offer: k_replay_scan's packed heap; computing a row that then fails is
// only wasted work).  Extracted ascending into asc row `q`.
// First every wave takes windows w = wave mod 8 and writes each window's
// smallest block minimum to LDS (up to RQ_RP_WMAX windows); the scan then
// passes a window whose minimum cannot beat a full heap's top without
// touching its keys (the test is the per-block one applied to the window's
// smallest key: no block of it would be a candidate).
// ---------------------------------------------------------------------------
constexpr int RQ_RP_WMAX = 4096;  // windows with an LDS minimum (2M blocks, 67M rows)
__host__ __device__ constexpr size_t rq8_replay_lds(int R, int qu4) {
    return (size_t)R * 16 + 16 + (size_t)qu4 * 16 + 512 * 4 + 16 * 32 * 4 + 16 * 4 + 8 * 4 + RQ_RP_WMAX * 4;
}
template <int BITS>
__global__ __launch_bounds__(512) void k_rq8_replay(const float* __restrict__ key, int64_t ldk, int64_t nblk,
                                                    const void* __restrict__ codes, int64_t cap,
                                                    const float4* __restrict__ meta, const uint32_t* __restrict__ valid,
                                                    int64_t nslots, const void* __restrict__ qsrc, int64_t q_base,
                                                    const float4* __restrict__ qmeta, int D, float fl2, float fcos,
                                                    const int32_t* __restrict__ list, int nlist, int R,
                                                    uint64_t id_base, uint64_t* __restrict__ ascI,
                                                    float* __restrict__ ascD, int32_t* __restrict__ ascN) {
    extern __shared__ __attribute__((aligned(16))) unsigned char rsm[];
    HeapRec* hr = reinterpret_cast<HeapRec*>(rsm);
    int* s_len = reinterpret_cast<int*>(hr + R);
    uint4* qs = reinterpret_cast<uint4*>(rsm + (size_t)R * 16 + 16);
    uint32_t* clist = reinterpret_cast<uint32_t*>(qs + rq_query_lds_u4(BITS, D));  // [512] window candidates
    float* cd = reinterpret_cast<float*>(clist + 512);                              // [16][32] row distances
    uint32_t* cm = reinterpret_cast<uint32_t*>(cd + 16 * 32);                        // [16] rows that pass
    int* wcnt = reinterpret_cast<int*>(cm + 16);                                     // [8] per-wave counts
    float* wmin = reinterpret_cast<float*>(wcnt + 8);                                // [RQ_RP_WMAX] window minima
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = blockIdx.x;
    if (li >= nlist) return;
    const int q = list[li];
    if (wave == 0) rq_query_to_lds<BITS>(qs, qsrc, q, q_base + q, D, lane);
    if (tid == 0) *s_len = 0;
    const float4 ym = qmeta[q];
    const float* kq = key + (int64_t)q * ldk;
    const int64_t nwin = (nblk + 511) / 512;
    const int64_t nwm = nwin < RQ_RP_WMAX ? nwin : RQ_RP_WMAX;
    for (int64_t w = wave; w < nwm; w += 8) {
        float m = __builtin_inff();
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int64_t bb = w * 512 + i * 64 + lane;
            m = fminf(m, bb < nblk ? kq[bb] : __builtin_inff());
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fminf(m, __shfl_xor(m, o));
        if (lane == 0) wmin[w] = m;
    }
    __syncthreads();
    for (int64_t w0 = 0; w0 < nblk; w0 += 512) {
        int len = *s_len;
        float top = len > 0 ? hr[0].d : 0.f;
        // (uniform: every thread reads the same heap state and window minimum)
        if (w0 / 512 < nwm && len >= R && !(top > wmin[w0 / 512])) continue;
        const float kcur = w0 + tid < nblk ? kq[w0 + tid] : __builtin_inff();
        const bool cand = w0 + tid < nblk && (len < R || top > kcur);
        const uint64_t mb = __ballot(cand);
        if (lane == 0) wcnt[wave] = __popcll(mb);
        __syncthreads();
        int off = 0, nc = 0;
#pragma unroll
        for (int w = 0; w < 8; w++) {
            const int c = wcnt[w];
            off += w < wave ? c : 0;
            nc += c;
        }
        if (cand) clist[off + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0))] =
            (uint32_t)(w0 + tid);
        __syncthreads();
        for (int c0 = 0; c0 < nc; c0 += 16) {
            const int bi = c0 + 2 * wave + (lane >> 5);
            const int64_t blk = bi < nc ? (int64_t)clist[bi] : 0;
            const int64_t s = blk * 32 + (lane & 31);
            const bool ok = bi < nc && s < nslots && ((valid[blk] >> (lane & 31)) & 1u);
            const float dist = ok ? rq_row_dist<BITS>(codes, cap, meta, s, qs, ym, D, fl2, fcos) : 0.f;
            len = *s_len;
            top = len > 0 ? hr[0].d : 0.f;
            const uint64_t pm = __ballot(ok && (len < R || top > dist));
            cd[(2 * wave + (lane >> 5)) * 32 + (lane & 31)] = dist;
            if (lane == 0) cm[2 * wave] = (uint32_t)pm;
            if (lane == 32) cm[2 * wave + 1] = (uint32_t)(pm >> 32);
            __syncthreads();
            if (tid == 0) {
                PHeap ph{hr, *s_len};
                const int nb = nc - c0 < 16 ? nc - c0 : 16;
                for (int b = 0; b < nb; b++) {
                    uint32_t m = cm[b];
                    const uint64_t base = id_base + (uint64_t)clist[c0 + b] * 32;
                    while (m) {
                        const int r = __builtin_ctz(m);
                        m &= m - 1;
                        ph_offer(ph, R, base + (uint64_t)r, cd[b * 32 + r]);
                    }
                }
                *s_len = ph.len;
            }
            __syncthreads();
        }
    }
    if (tid == 0) {  // extractHeap: pop max-first, fill from the back
        PHeap ph{hr, *s_len};
        const int n = *s_len;
        for (int i = n - 1; i >= 0; i--) {
            uint64_t a;
            float b;
            ph_pop(ph, &a, &b);
            ascI[(int64_t)q * R + i] = a;
            ascD[(int64_t)q * R + i] = b;
        }
        ascN[q] = n;
    }
}

// SingleDist of the replayed queries' candidates (k_rescore_ids with rows by
// query: ids / counts / distances of query list[li] at row list[li])
template <int METRIC, int VARIANT>
__global__ __launch_bounds__(64) void k_rescore_list(const float* __restrict__ X, int dpad, const float* __restrict__ Q,
                                                     int d, const uint64_t* __restrict__ ids,
                                                     const int32_t* __restrict__ cnt, const int32_t* __restrict__ list,
                                                     int nlist, int R, uint64_t id_base, int64_t nslots,
                                                     float* __restrict__ outE) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)nlist * R) return;
    const int q = list[p / R], i = (int)(p % R);
    if (i >= cnt[q]) return;
    const int64_t e = (int64_t)q * R + i;
    const uint64_t id = ids[e];
    if (id < id_base || id - id_base >= (uint64_t)nslots) return;
    outE[e] = exact_dist<METRIC, VARIANT>(Q + (int64_t)q * dpad, X + (int64_t)(id - id_base) * dpad, d);
}

// flagged queries' codes and meta (group-tiled rq-8 query layout) -> a
// compact copy: entry f = query list[f]; thread per (entry, 16-byte chunk)
__global__ void k_rq8_gather_q(const uint4* __restrict__ qcodes, const float4* __restrict__ qmeta, int nch,
                               const int32_t* __restrict__ list, int nf, uint4* __restrict__ ocodes,
                               float4* __restrict__ ometa) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)nf * nch) return;
    const int f = (int)(i / nch), c = (int)(i % nch);
    const int64_t q = list[f];
    ocodes[((int64_t)(f / RQ_QPB) * nch + c) * RQ_QPB + f % RQ_QPB] = qcodes[((q / RQ_QPB) * nch + c) * RQ_QPB + q % RQ_QPB];
    if (c == 0) ometa[f] = qmeta[q];
}

// as k_rq8_gather_q for rq-1's planes: ne = 5 W u64 per query, group-tiled
// ((g * ne + e) * RQ_QPB + q % RQ_QPB); thread per (entry, word)
__global__ void k_rq1_gather_q(const uint64_t* __restrict__ planes, const float4* __restrict__ qmeta, int ne,
                               const int32_t* __restrict__ list, int nf, uint64_t* __restrict__ oplanes,
                               float4* __restrict__ ometa) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)nf * ne) return;
    const int f = (int)(i / ne), e = (int)(i % ne);
    const int64_t q = list[f];
    oplanes[((int64_t)(f / RQ_QPB) * ne + e) * RQ_QPB + f % RQ_QPB] = planes[((q / RQ_QPB) * ne + e) * RQ_QPB + q % RQ_QPB];
    if (e == 0) ometa[f] = qmeta[q];
}

}  // namespace
}  // namespace wv
