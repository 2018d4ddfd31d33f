// ---------------------------------------------------------------------------
// k_gemv_select: small query batches (nq <= gemv_max, default 8) as an
// HBM-streaming GEMV.  One fp32 query alone makes the scan a matrix-vector
// product: the MFMA tile kernels then compute 128 query columns of which one
// is real (SURVEY.md §8d C3, B=1: HBM-bound, 30.72 GB per pass -> 3.84 ms).
//
// Workgroup = QG queries (staged in LDS) x one span of rows.  A 16-lane group
// owns 2 rows at a time and reads each as 16 contiguous float4 per step
// (256 B per row per load instruction, 4 row groups per wave), FMAs against
// the LDS query rows (conflict-free: 16 consecutive float4), then a 4-step
// xor-shuffle reduction.  The distance form and candidate protocol are those
// of the MFMA kernels (k_mfma_select: A = (|x|^2 - 2 x.q) + |q|^2 / -x.q /
// max(0, 1 - x.q); per (query, span) KP-list of the smallest A, ascending,
// +inf / NO_ID padded), so k_merge_spans, k_rescore and k_finalize's
// exactness proof apply unchanged: each dot product is an fp32 FMA chain of
// dpad/64 steps plus 4 tree levels, inside the gamma_{dpad+4} bound the f32
// MFMA kernel is proved with.
// Per chunk of 32 rows a query gains at most 32 candidates (C = 64 - KP >= 32
// since KP <= 32), so the candidate buffer never overflows; a merge pass runs
// only after chunks that produced candidates.
// ---------------------------------------------------------------------------
#pragma once
namespace wv {
namespace {  // internal linkage: each runtime unit compiles the kernels it launches

template <int METRIC, int QG>
__global__ __launch_bounds__(256) void k_gemv_select(SelectArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int KP = a.KP, C = a.C, dpad = a.dpad;
    float* Qs = smem;                                        // QG*dpad
    float* listA = Qs + QG * dpad;                           // QG*KP
    uint32_t* listI = reinterpret_cast<uint32_t*>(listA + QG * KP);
    float* cbA = reinterpret_cast<float*>(listI + QG * KP);  // QG*C
    uint32_t* cbI = reinterpret_cast<uint32_t*>(cbA + QG * C);
    float* thr = reinterpret_cast<float*>(cbI + QG * C);     // QG
    int* cnt = reinterpret_cast<int*>(thr + QG);             // QG
    int* flag = cnt + QG;                                    // 3 (rotating, see below)

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int sub = lane & 15, rg = lane >> 4;
    const int group = blockIdx.x / a.nspans;
    const int span = blockIdx.x % a.nspans;
    const int q0 = group * QG;

    for (int i = tid; i < QG * dpad; i += 256) {
        const int q = i / dpad;
        Qs[i] = (q0 + q < a.nq) ? a.Q[(int64_t)(q0 + q) * dpad + (i - q * dpad)] : 0.f;
    }
    for (int i = tid; i < QG * KP; i += 256) { listA[i] = __builtin_inff(); listI[i] = NO_ID; }
    if (tid < QG) { thr[tid] = __builtin_inff(); cnt[tid] = 0; }
    if (tid < 3) flag[tid] = 0;
    float qn[QG];
#pragma unroll
    for (int q = 0; q < QG; q++) qn[q] = (METRIC == L2 && q0 + q < a.nq) ? a.qnorm2[q0 + q] : 0.f;
    __syncthreads();

    const int64_t t0 = (int64_t)span * a.tiles_per_span;
    int64_t t1 = t0 + a.tiles_per_span;
    if (t1 > a.ntiles) t1 = a.ntiles;
    const int64_t r_begin = t0 * BN3, r_end = t1 > t0 ? t1 * BN3 : r_begin;
    const int nc4 = dpad >> 2;

    int it = 0;
    for (int64_t base = r_begin; base < r_end; base += 32, it++) {
        // flag[it % 3] collects "some candidate this chunk"; flag[(it + 1) % 3]
        // was last read before the previous chunk's barrier, so it is reset here
        if (tid == 0) flag[(it + 1) % 3] = 0;
        const int64_t row0 = base + wave * 8 + rg * 2;
        const float* x0p = a.X + row0 * (int64_t)dpad;
        const float* x1p = x0p + dpad;
        float acc0[QG], acc1[QG];
#pragma unroll
        for (int q = 0; q < QG; q++) { acc0[q] = 0.f; acc1[q] = 0.f; }
#pragma unroll 4
        for (int c = sub; c < nc4; c += 16) {
            const float4 x0 = ld4(x0p + 4 * c);
            const float4 x1 = ld4(x1p + 4 * c);
#pragma unroll
            for (int q = 0; q < QG; q++) {
                const float4 y = *reinterpret_cast<const float4*>(Qs + q * dpad + 4 * c);
                acc0[q] = __builtin_fmaf(x0.x, y.x, acc0[q]);
                acc0[q] = __builtin_fmaf(x0.y, y.y, acc0[q]);
                acc0[q] = __builtin_fmaf(x0.z, y.z, acc0[q]);
                acc0[q] = __builtin_fmaf(x0.w, y.w, acc0[q]);
                acc1[q] = __builtin_fmaf(x1.x, y.x, acc1[q]);
                acc1[q] = __builtin_fmaf(x1.y, y.y, acc1[q]);
                acc1[q] = __builtin_fmaf(x1.z, y.z, acc1[q]);
                acc1[q] = __builtin_fmaf(x1.w, y.w, acc1[q]);
            }
        }
#pragma unroll
        for (int off = 8; off >= 1; off >>= 1) {
#pragma unroll
            for (int q = 0; q < QG; q++) {
                acc0[q] += __shfl_xor(acc0[q], off);
                acc1[q] += __shfl_xor(acc1[q], off);
            }
        }
        // lane sub = u * QG + q of the group tests (row0 + u, query q)
        if (sub < 2 * QG) {
            const int u = sub / QG, q = sub % QG;
            float dot = 0.f;
#pragma unroll
            for (int uu = 0; uu < 2; uu++)
#pragma unroll
                for (int qq = 0; qq < QG; qq++)
                    if (uu * QG + qq == sub) dot = uu ? acc1[qq] : acc0[qq];
            float qnq = 0.f;
#pragma unroll
            for (int qq = 0; qq < QG; qq++)
                if (qq == q) qnq = qn[qq];
            const int64_t row = row0 + u;
            const bool ok = ((a.valid[row >> 5] >> (row & 31)) & 1u) && (q0 + q < a.nq);
            float v;
            if (METRIC == L2) v = (a.xnorm2[row] - 2.f * dot) + qnq;
            else if (METRIC == DOT) v = -dot;
            else { v = 1.f - dot; v = v < 0.f ? 0.f : v; }
            if (ok && v < thr[q]) {
                const int slot = atomicAdd(&cnt[q], 1);
                cbA[q * C + slot] = v;
                cbI[q * C + slot] = (uint32_t)row;
                flag[it % 3] = 1;
            }
        }
        __syncthreads();
        if (flag[it % 3]) {
            for (int q = wave; q < QG; q += 4) {
                const int c = cnt[q];
                if (c == 0) continue;
                merge_query_list<1>(listA + q * KP, listI + q * KP, cbA + q * C, cbI + q * C, KP, C, c, lane, &thr[q]);
                if (lane == 0) cnt[q] = 0;
            }
            __syncthreads();
        }
    }

    for (int q = wave; q < QG; q += 4) {
        if (q0 + q >= a.nq) continue;
        const int64_t base = ((int64_t)(q0 + q) * a.nspans + span) * KP;
        for (int e = lane; e < KP; e += 64) {
            a.outA[base + e] = listA[q * KP + e];
            a.outI[base + e] = listI[q * KP + e];
        }
    }
}

}  // namespace
}  // namespace wv
