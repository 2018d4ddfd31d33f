// bq_kernels.hip -- gfx950 kernels of the BQ-compressed flat search
// (flat.searchByVectorQuantized, flat/index.go:460-532).
//
// Codes live word-major in HBM: codes[w * ccap + slot] = word w of the
// BinaryQuantizer code of the stored (normalised) row `slot`
// (compressionhelpers/binary_quantization.go:28-47), so a wave reading word w
// of 64 consecutive slots issues one coalesced 512 B load.
//
// Search, per batch of queries (all integer work until the rescoring):
//   k_bq_encode_rows   queries -> codes (same encoder as Add)
//   k_bq_blockmin      hamming distance of every (query, row) pair, reduced
//                      to the minimum per 256-row block; nothing else is
//                      written (VALU-bound: 2 x v_xor + 2 x v_bcnt per word)
//   k_bq_replay        one wave per query replays the reference's R-heap
//                      (priorityqueue.NewMax + insertToHeap over id order,
//                      flat/index.go:578-674) exactly: a block is visited only
//                      while the heap is short or its minimum is < top (the
//                      top never increases, so a skipped block cannot insert);
//                      visited blocks recompute their distances in-register.
//                      Then it pops the heap max-first (:485-487) and writes
//                      the R candidates in that pop order.
//   k_rescore          exact-order fp32 SingleDist of every candidate (shared
//                      with the uncompressed path)
//   k_bq_final         insertToHeap(heap, k, ...) in pop order + extractHeap
//                      (:525-531)
// Hamming ties are the rule, not the exception, so the replay is the path for
// every query: the selected set and its tie order are the reference's.
#pragma once

namespace wv {
namespace {  // internal linkage: each runtime unit compiles the kernels it launches

constexpr int BQBLK = 256;  // rows per block minimum (== EBLK)

// BinaryQuantizer.Encode of padded rows: bit (i mod 64) of word i/64 is set iff
// v[i] < 0 (NaN / +-0 -> 0).  Thread per (row, word); row r reads and writes
// slot = slots[r] (or r): rows[slot * ld ...] -> out[w * ldo + slot].
__global__ void k_bq_encode_rows(const float* __restrict__ rows, int64_t ld, int64_t n, int d,
                                 const uint32_t* __restrict__ slots, uint64_t* __restrict__ out, int64_t ldo) {
    const int words = (d + 63) >> 6;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * words) return;
    const int64_t r = i % n;  // consecutive threads -> consecutive rows: coalesced stores
    const int w = (int)(i / n);
    const int64_t slot = slots ? (int64_t)slots[r] : r;
    const float* src = rows + slot * ld + 64 * w;
    const int lim = d - 64 * w < 64 ? d - 64 * w : 64;
    uint64_t bits = 0;
    for (int b = 0; b < lim; b++)
        if (src[b] < 0.f) bits |= 1ull << b;
    out[(int64_t)w * ldo + slot] = bits;
}

// Block minima of the hamming distances.  Block (x, y): rows [256x, +256),
// listed queries [QPB*y, +QPB).  Thread = row; the row's words are read once
// (coalesced) and xor/popcounted against QPB query codes held in SGPRs.
// Query codes are word-major too: word w of query q at qcodes[w * ldq + q].
// bmin[f * nblk + x] = min over valid rows (+inf if none).
template <int QPB>
__global__ __launch_bounds__(256) void k_bq_blockmin(const uint64_t* __restrict__ codes, int64_t ccap, int words,
                                                     const uint32_t* __restrict__ valid, int64_t nslots,
                                                     const uint64_t* __restrict__ qcodes, int64_t ldq,
                                                     const int32_t* __restrict__ qlist, int nlist, int64_t nblk,
                                                     float* __restrict__ bmin) {
    __shared__ uint32_t red[4][QPB];
    const int64_t blk = blockIdx.x;
    const int f0 = blockIdx.y * QPB;
    const int64_t s = blk * BQBLK + threadIdx.x;
    const bool ok = s < nslots && ((valid[s >> 5] >> (s & 31)) & 1u);
    int qrow[QPB];
#pragma unroll
    for (int f = 0; f < QPB; f++) qrow[f] = qlist[(f0 + f) < nlist ? f0 + f : nlist - 1];
    uint32_t acc[QPB];
#pragma unroll
    for (int f = 0; f < QPB; f++) acc[f] = 0;
    const uint64_t* cp = codes + (s < nslots ? s : 0);
    for (int w = 0; w < words; w++) {
        const uint64_t x = cp[(int64_t)w * ccap];
#pragma unroll
        for (int f = 0; f < QPB; f++) acc[f] += (uint32_t)__popcll(x ^ qcodes[(int64_t)w * ldq + qrow[f]]);
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int f = 0; f < QPB; f++) {
        uint32_t m = ok ? acc[f] : 0xFFFFFFFFu;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, o));
        if (lane == 0) red[wv][f] = m;
    }
    __syncthreads();
    if (threadIdx.x < QPB && f0 + (int)threadIdx.x < nlist) {
        const int f = threadIdx.x;
        const uint32_t m = min(min(red[0][f], red[1][f]), min(red[2][f], red[3][f]));
        bmin[(int64_t)(f0 + f) * nblk + blk] = m == 0xFFFFFFFFu ? __builtin_inff() : (float)m;
    }
}

// Block minima, LDS-broadcast form (words <= NW <= 32).  Block = 256 queries
// (lane = query, its NW-word code in VGPRs) x a span of 256-row tiles.  Each
// tile is staged once into LDS row-major ([row][NW] u64, zero padded) from the
// word-major store (2 KiB coalesced per word), then every wave walks the 256
// rows reading each row with uniform-address ds_read_b128 (broadcast, no bank
// conflicts) against its 64 query codes in registers: per row and word
// 2 x v_xor_b32 + 2 x v_bcnt_u32_b32, the running minimum per lane, and one
// store per (query, tile).
template <int NW>
__global__ __launch_bounds__(256, 2) void k_bq_blockmin_lds(const uint64_t* __restrict__ codes, int64_t ccap,
                                                            int words, const uint32_t* __restrict__ valid,
                                                            int64_t nslots, const uint64_t* __restrict__ qcodes,
                                                            int64_t ldq, const int32_t* __restrict__ qlist, int nlist,
                                                            int64_t nblk, int64_t blk_per_span,
                                                            float* __restrict__ bmin) {
    __shared__ __attribute__((aligned(16))) uint64_t tile[BQBLK * NW];
    __shared__ uint32_t vb[BQBLK / 32];
    const int t = threadIdx.x;
    const int f = blockIdx.y * 256 + t;
    const bool fq = f < nlist;
    uint32_t qlo[NW], qhi[NW];
    {
        const int qr = qlist[fq ? f : nlist - 1];
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const uint64_t v = w < words ? qcodes[(int64_t)w * ldq + qr] : 0ull;
            qlo[w] = (uint32_t)v;
            qhi[w] = (uint32_t)(v >> 32);
        }
    }
    const int64_t b0 = (int64_t)blockIdx.x * blk_per_span;
    int64_t b1 = b0 + blk_per_span;
    if (b1 > nblk) b1 = nblk;
    for (int64_t blk = b0; blk < b1; blk++) {
        const int64_t s = blk * BQBLK + t;
        __syncthreads();  // previous tile consumed
#pragma unroll
        for (int w = 0; w < NW; w++)
            tile[t * NW + w] = (w < words && s < nslots) ? codes[(int64_t)w * ccap + s] : 0ull;
        if (t < BQBLK / 32) {
            const int64_t wi = blk * (BQBLK / 32) + t;
            vb[t] = (wi * 32 < nslots) ? valid[wi] : 0u;
        }
        __syncthreads();
        uint32_t mn = 0xFFFFFFFFu;
        for (int r0 = 0; r0 < BQBLK; r0 += 32) {
            const uint32_t vbits = vb[r0 >> 5];
            if (vbits == 0) continue;
#pragma unroll 2
            for (int r = 0; r < 32; r++) {
                const uint4* rp = reinterpret_cast<const uint4*>(&tile[(r0 + r) * NW]);
                uint32_t acc = 0;
#pragma unroll
                for (int c = 0; c < NW / 2; c++) {
                    const uint4 v = rp[c];
                    acc += __builtin_popcount(qlo[2 * c] ^ v.x);
                    acc += __builtin_popcount(qhi[2 * c] ^ v.y);
                    acc += __builtin_popcount(qlo[2 * c + 1] ^ v.z);
                    acc += __builtin_popcount(qhi[2 * c + 1] ^ v.w);
                }
                if ((vbits >> r) & 1u) mn = min(mn, acc);
            }
        }
        if (fq) bmin[(int64_t)f * nblk + blk] = mn == 0xFFFFFFFFu ? __builtin_inff() : (float)mn;
    }
}

// Exact replay of the R-heap of searchByVectorQuantized (one wave per listed
// query), then the max-first pop of the whole heap (flat/index.go:485-487).
// out_slot[li * R + i] = slot of the i-th popped item, out_n[li] = heap length.
// A visited block's 256 distances are recomputed with all loads issued up
// front (NW > 0: words <= NW known at compile time; NW == 0: generic loop).
// The heap is PHeap (16-byte records: one LDS round trip per sift level).
// REC: record insertions (rec_* non-null); a separate instantiation keeps the
// record's pointers out of the plain replay's scalar registers (the REC form
// spilled 335 SGPRs: 26.6 ms vs 17.5 ms per C4 launch)
// BLK: rows per block minimum -- 256 (the VALU minima) or 32 (the integer-MFMA
// minima, k_q8_blockkey<..., BQ>): with 32-row blocks a visited block is 32 rows
// (lane = row, lanes 32-63 take the next visitable block speculatively: its
// rows are offered only after the first block's, each against the heap top
// of that moment, so the insertions are the in-order ones)
template <int NW, bool REC, int BLK = BQBLK>
__global__ __launch_bounds__(64) void k_bq_replay(const uint64_t* __restrict__ codes, int64_t ccap, int words,
                                                  const uint32_t* __restrict__ valid, int64_t nslots,
                                                  const uint64_t* __restrict__ qcodes, int64_t ldq,
                                                  const int32_t* __restrict__ qlist, int nlist,
                                                  const float* __restrict__ bmin, int64_t nblk, int R,
                                                  uint64_t id_base, const uint64_t* __restrict__ in_ids,
                                                  const float* __restrict__ in_d, const int32_t* __restrict__ in_len,
                                                  int pop, uint64_t* __restrict__ out_ids, float* __restrict__ out_d,
                                                  int32_t* __restrict__ out_n, uint64_t* __restrict__ rec_ids,
                                                  float* __restrict__ rec_d, int32_t* __restrict__ rec_n, int cap,
                                                  const int32_t* __restrict__ skip) {
    // dynamic LDS: [R] heap records (PHeap) | [64] f32 | len
    extern __shared__ __attribute__((aligned(16))) unsigned char rsm[];
    HeapRec* hr = reinterpret_cast<HeapRec*>(rsm);
    float* s_d = reinterpret_cast<float*>(hr + R);
    int* s_len = reinterpret_cast<int*>(s_d + 64);
    const int lane = threadIdx.x;
    const int li = blockIdx.x;
    if (li >= nlist) return;
    if (skip && skip[li]) return;  // answered by k_bq_fast
    const uint64_t* qc = qcodes + qlist[li];  // word w at qc[w * ldq]
    const float* Bq = bmin + (int64_t)li * nblk;
    // heap state handed over by the previous shard (layout order), or empty
    const int len0 = in_len ? in_len[li] : 0;
    for (int i = lane; i < len0; i += 64) hr[i] = hr_make(in_ids[(int64_t)li * R + i], in_d[(int64_t)li * R + i]);
    if (lane == 0) {
        *s_len = len0;
        if (REC) rec_n[li] = 0;
    }
    __syncthreads();
    if constexpr (BLK == 32 && NW > 0) {
        // 32-row blocks, software-pipelined: the codes of the next two visitable
        // blocks (chosen under the top before the current insertions: a superset,
        // a block that stops qualifying only offers rows ph_offer rejects) load
        // while lane 0 inserts the current two blocks' rows.  Query words in
        // registers; a block's valid word and codes load together.
        uint64_t qw[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) qw[w] = w < words ? qc[(int64_t)w * ldq] : 0ull;
        // the block minima in windows of 16 chunks of 64 blocks: the next window
        // loads while this one is scanned (16 loads in flight instead of one
        // chunk ahead), and a chunk with no block under the top when its window
        // came up is never looked at again (the top only falls once the heap is full)
        float bw[16], bn[16];
        auto load_win = [&](float* dst, int64_t base) {
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const int64_t b = base + u * 64 + lane;
                dst[u] = b < nblk ? Bq[b] : __builtin_inff();
            }
        };
        auto win_mask = [&]() -> uint32_t {
            const int len = *s_len;
            const float top = len > 0 ? hr[0].d : 0.f;
            uint32_t m = 0;
#pragma unroll
            for (int u = 0; u < 16; u++)
                if (__ballot(bw[u] != __builtin_inff() && (len < R || top > bw[u]))) m |= 1u << u;
            return m;
        };
        int64_t wb0 = 0;
        load_win(bw, 0);
        load_win(bn, 1024);
        uint32_t wm = win_mask();
        int wi = -1;
        float bmc = __builtin_inff();
        uint64_t cmask = 0;
        auto next_blk = [&]() -> int64_t {
            const int len = *s_len;
            const float top = len > 0 ? hr[0].d : 0.f;
            while (true) {
                while (cmask) {
                    const int j = __builtin_ctzll(cmask);
                    cmask &= cmask - 1;
                    if (len < R || top > __shfl(bmc, j)) return wb0 + wi * 64 + j;
                }
                if (wi >= 0) wm &= ~((2u << wi) - 1u);
                if (wm) {
                    wi = __builtin_ctz(wm);
                    float v = bw[0];
#pragma unroll
                    for (int u = 1; u < 16; u++) v = wi == u ? bw[u] : v;
                    bmc = v;
                    cmask = __ballot(bmc != __builtin_inff() && (len < R || top > bmc));
                    continue;
                }
                wb0 += 1024;
                if (wb0 >= nblk) return -1;
#pragma unroll
                for (int u = 0; u < 16; u++) bw[u] = bn[u];
                load_win(bn, wb0 + 1024);
                wm = win_mask();
                wi = -1;
            }
        };
        // two pairs of blocks in flight: buffers A and B take alternate pairs, so
        // a pair's codes load while the two pairs before it are inserted
        uint64_t xa[NW], xb[NW];
        uint32_t va = 0, vb = 0;
        auto load = [&](uint64_t (&x)[NW], uint32_t& vword, int64_t pa, int64_t pb) {
            const int64_t blk = lane < 32 ? pa : pb;
            const int64_t srow = blk * 32 + (lane & 31);
            const bool in = blk >= 0 && srow < nslots;
            vword = blk >= 0 ? valid[blk] : 0u;
#pragma unroll
            for (int w = 0; w < NW; w++) x[w] = (in && w < words) ? codes[(int64_t)w * ccap + srow] : 0ull;
        };
        // the pair (pa, pb) in buffer x: its rows' distances, the pair after the
        // one in the other buffer (fa >= 0) into x, then the insertions in id order
        auto step = [&](uint64_t (&x)[NW], uint32_t& vword, int64_t& pa, int64_t& pb, int64_t fa) {
            const int64_t blk = lane < 32 ? pa : pb;
            const int64_t srow = blk * 32 + (lane & 31);
            const bool ok = blk >= 0 && srow < nslots && ((vword >> (lane & 31)) & 1u);
            uint32_t h = 0;
#pragma unroll
            for (int w = 0; w < NW; w++) h += (uint32_t)__popcll(x[w] ^ qw[w]);
            const float dist = (float)h;
            const int64_t na = fa >= 0 ? next_blk() : -1;
            const int64_t nb = na >= 0 ? next_blk() : -1;
            if (na >= 0) load(x, vword, na, nb);  // in flight during the insertions below
            const int len = *s_len;
            const float top = len > 0 ? hr[0].d : 0.f;
            uint64_t mask = __ballot(ok && (len < R || top > dist));
            if (mask) {
                s_d[lane] = dist;
                __syncthreads();
                if (lane == 0) {
                    PHeap hp{hr, *s_len};
                    while (mask) {  // block pa's rows (lanes 0-31), then pb's (32-63): id order
                        const int jj = __builtin_ctzll(mask);
                        mask &= mask - 1;
                        const float dj = s_d[jj];
                        const uint64_t sj = id_base + (uint64_t)((jj < 32 ? pa : pb) * 32 + (jj & 31));
                        const bool ins = ph_offer(hp, R, sj, dj);
                        if (REC && ins) {
                            const int c = rec_n[li];
                            if (c < cap) { rec_ids[(int64_t)li * cap + c] = sj; rec_d[(int64_t)li * cap + c] = dj; }
                            rec_n[li] = c < cap ? c + 1 : cap + 1;
                        }
                    }
                    *s_len = hp.len;
                }
                __syncthreads();
            }
            pa = na;
            pb = nb;
        };
        int64_t pa = next_blk();
        int64_t pb = pa >= 0 ? next_blk() : -1;
        if (pa >= 0) load(xa, va, pa, pb);
        int64_t qa = pa >= 0 ? next_blk() : -1;
        int64_t qb = qa >= 0 ? next_blk() : -1;
        if (qa >= 0) load(xb, vb, qa, qb);
        while (true) {
            if (pa < 0) break;
            step(xa, va, pa, pb, qa);
            if (qa < 0) break;
            step(xb, vb, qa, qb, pa);
        }
    } else
    for (int64_t b0 = 0; b0 < nblk; b0 += 64) {
        const float bm = (b0 + lane < nblk) ? Bq[b0 + lane] : __builtin_inff();
        int len = *s_len;
        float top = len > 0 ? hr[0].d : 0.f;
        uint64_t bmask = __ballot((b0 + lane < nblk) && bm != __builtin_inff() && (len < R || top > bm));
        while (bmask) {
            const int j = __builtin_ctzll(bmask);
            bmask &= bmask - 1;
            const float bmj = __shfl(bm, j);
            len = *s_len;
            top = len > 0 ? hr[0].d : 0.f;
            if (!(len < R || top > bmj)) continue;
            const int64_t r0 = (b0 + j) * BQBLK;
            float dist[BQBLK / 64];
            bool okv[BQBLK / 64];
#pragma unroll
            for (int sub = 0; sub < BQBLK / 64; sub++) {
                const int64_t s = r0 + sub * 64 + lane;
                okv[sub] = s < nslots && ((valid[s >> 5] >> (s & 31)) & 1u);
            }
            if (NW > 0) {
                uint64_t x[BQBLK / 64][NW > 0 ? NW : 1];
#pragma unroll
                for (int sub = 0; sub < BQBLK / 64; sub++)
#pragma unroll
                    for (int w = 0; w < (NW > 0 ? NW : 1); w++)
                        x[sub][w] = (okv[sub] && w < words) ? codes[(int64_t)w * ccap + r0 + sub * 64 + lane] : 0ull;
#pragma unroll
                for (int sub = 0; sub < BQBLK / 64; sub++) {
                    uint32_t h = 0;
#pragma unroll
                    for (int w = 0; w < (NW > 0 ? NW : 1); w++)
                        h += (uint32_t)__popcll(x[sub][w] ^ (w < words ? qc[(int64_t)w * ldq] : 0ull));
                    dist[sub] = (float)h;
                }
            } else {
#pragma unroll
                for (int sub = 0; sub < BQBLK / 64; sub++) {
                    uint32_t h = 0;
                    if (okv[sub])
                        for (int w = 0; w < words; w++)
                            h += (uint32_t)__popcll(codes[(int64_t)w * ccap + r0 + sub * 64 + lane] ^ qc[(int64_t)w * ldq]);
                    dist[sub] = (float)h;
                }
            }
#pragma unroll
            for (int sub = 0; sub < BQBLK / 64; sub++) {
                len = *s_len;
                top = len > 0 ? hr[0].d : 0.f;
                uint64_t mask = __ballot(okv[sub] && (len < R || top > dist[sub]));
                if (mask == 0) continue;
                s_d[lane] = dist[sub];
                __syncthreads();
                if (lane == 0) {
                    PHeap hp{hr, *s_len};
                    const int64_t sb = r0 + sub * 64;
                    while (mask) {
                        const int jj = __builtin_ctzll(mask);
                        mask &= mask - 1;
                        const float dj = s_d[jj];
                        const uint64_t sj = id_base + (uint64_t)(sb + jj);
                        const bool ins = ph_offer(hp, R, sj, dj);
                        if (REC && ins) {  // the parallel cross-shard replay's record (id order)
                            const int c = rec_n[li];
                            if (c < cap) { rec_ids[(int64_t)li * cap + c] = sj; rec_d[(int64_t)li * cap + c] = dj; }
                            rec_n[li] = c < cap ? c + 1 : cap + 1;
                        }
                    }
                    *s_len = hp.len;
                }
                __syncthreads();
            }
        }
    }
    if (lane == 0 && out_n) {
        PHeap hp{hr, *s_len};
        const int n = hp.len;
        if (pop) {  // pop order (max first) = idsSlice of flat/index.go:485-487
            for (int i = 0; i < n; i++) {
                uint64_t a; float b;
                ph_pop(hp, &a, &b);
                out_ids[(int64_t)li * R + i] = a;
                out_d[(int64_t)li * R + i] = b;
            }
        } else {  // the heap state itself, for the next shard
            for (int i = 0; i < n; i++) { out_ids[(int64_t)li * R + i] = hr_id(hr[i]); out_d[(int64_t)li * R + i] = hr[i].d; }
        }
        out_n[li] = n;
    }
}

// Per query the R smallest 256-row block minima of this shard, ascending
// (+inf padded): each is the exact hamming distance of one distinct row, so
// the R-th smallest over the shards before r bounds the R-heap's top at shard
// r's first row (the parallel cross-shard replay, weaviate_amd/sharded.py).
// Hamming distances are integers 0..64*words: a histogram per query in LDS.
__global__ __launch_bounds__(256) void k_bq_bounds(const float* __restrict__ bmin, int64_t nblk, int nbins, int R,
                                                   float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char hsm[];
    uint32_t* hist = reinterpret_cast<uint32_t*>(hsm);
    const int q = blockIdx.x;
    for (int i = threadIdx.x; i < nbins; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    const float* Bq = bmin + (int64_t)q * nblk;
    for (int64_t b = threadIdx.x; b < nblk; b += blockDim.x) {
        const float v = Bq[b];
        if (v < (float)nbins) atomicAdd(&hist[(int)v], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float* o = out + (int64_t)q * R;
        int n = 0;
        for (int v = 0; v < nbins && n < R; v++)
            for (uint32_t c = hist[v]; c > 0 && n < R; c--) o[n++] = (float)v;
        for (; n < R; n++) o[n] = __builtin_inff();
    }
}

// Exact-order SingleDist of candidate ids (lane per (listed query, entry)):
// ids [nlist][R] global, entries i < cnt[li]; only ids this shard holds
// (id_base <= id < id_base + nslots) are written.  Q row = qlist[li].
template <int METRIC, int VARIANT>
__global__ __launch_bounds__(64) void k_rescore_ids(const float* __restrict__ X, int dpad, const float* __restrict__ Q,
                                                    int d, const uint64_t* __restrict__ ids,
                                                    const int32_t* __restrict__ cnt, const int32_t* __restrict__ qlist,
                                                    int nlist, int R, uint64_t id_base, int64_t nslots,
                                                    float* __restrict__ outE) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)nlist * R) return;
    const int li = (int)(p / R), i = (int)(p % R);
    if (i >= cnt[li]) return;
    const uint64_t id = ids[p];
    if (id < id_base || id - id_base >= (uint64_t)nslots) return;
    outE[p] = exact_dist<METRIC, VARIANT>(Q + (int64_t)qlist[li] * dpad, X + (int64_t)(id - id_base) * dpad, d);
}

// k_bq_fast<NW, METRIC, VARIANT>: a replay-free answer when hamming ties
// cannot change it.  With h* the R-th smallest hamming distance,
// S the rows below h* and T the rows at h*, the R-heap of flat/index.go:578-674
// ends holding S plus some T' of T (which ones depends on the heap's tie
// order).  If the m = min(k, heap size) smallest exact distances over S u T are
// strictly increasing, strictly below the next one, and (when T was cut) all
// from S, every possible T' rescores (flat/index.go:490-531) to the same
// result, which is then written as the query's candidate list (m ids; the
// rescoring and k_bq_final run on it as on a replayed heap) and skip[li] = 1.
// Otherwise skip[li] = 0 and the replay runs.  Rows at or below h* are found
// from the 32-row block minima: blocks with minimum <= H_R (the R-th smallest
// block minimum) hold every such row.  One 256-thread workgroup per query.
constexpr int BQF_CB = 2048;  // candidate blocks
constexpr int BQF_RC = 2048;  // rows at or below H_R
constexpr int BQF_UC = 1024;  // rows at or below h*
constexpr int BQF_K = 64;     // k
template <int NW, int METRIC, int VARIANT>
__global__ __launch_bounds__(256) void k_bq_fast(const uint64_t* __restrict__ codes, int64_t ccap, int words,
                                                 const uint32_t* __restrict__ valid, int64_t nslots,
                                                 const uint64_t* __restrict__ qcodes, int64_t ldq,
                                                 const int32_t* __restrict__ qlist, int nlist,
                                                 const float* __restrict__ bmin, int64_t nblk, int R, int k,
                                                 const float* __restrict__ X, int dpad, const float* __restrict__ Q,
                                                 int d, uint64_t id_base, uint64_t* __restrict__ out_ids,
                                                 int32_t* __restrict__ out_n, int32_t* __restrict__ skip) {
    constexpr int HB = 64 * NW + 1;
    __shared__ uint32_t hist[4][HB];
    __shared__ uint32_t cblk[BQF_CB];
    __shared__ uint32_t rslot[BQF_RC];
    __shared__ uint16_t rh[BQF_RC];
    __shared__ uint32_t uslot[BQF_UC];
    __shared__ uint16_t uh[BQF_UC];
    __shared__ float ud[BQF_UC];
    __shared__ uint8_t upick[BQF_UC];
    __shared__ float rd[4];
    __shared__ int ri[4];
    __shared__ uint32_t pslot[BQF_K];
    __shared__ int s_ncb, s_nrow, s_nu, s_H, s_fail, s_tot;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = blockIdx.x;
    if (li >= nlist) return;
    const float* Bq = bmin + (int64_t)li * nblk;
    for (int i = tid; i < 4 * HB; i += 256) (&hist[0][0])[i] = 0u;
    if (tid == 0) { s_ncb = 0; s_nrow = 0; s_nu = 0; s_fail = k > BQF_K ? 1 : 0; }
    __syncthreads();
    // 1. histogram of the block minima (one copy per wave), H_R
    for (int64_t b = tid; b < nblk; b += 256) {
        const float v = Bq[b];
        if (v < (float)HB) atomicAdd(&hist[w][(int)v], 1u);
    }
    __syncthreads();
    for (int i = tid; i < HB; i += 256) hist[0][i] += hist[1][i] + hist[2][i] + hist[3][i];
    __syncthreads();
    // smallest H with count(<= H) >= R (HB - 1 when fewer): wave 0, a segment per lane
    auto threshold = [&](int want) {
        if (w == 0) {
            constexpr int SEG = (HB + 63) / 64;
            const int h0 = lane * SEG;
            uint32_t sum = 0;
            for (int h = h0; h < h0 + SEG && h < HB; h++) sum += hist[0][h];
            uint32_t incl = sum;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(incl, o);
                if (lane >= o) incl += t;
            }
            const uint64_t hit = __ballot(incl >= (uint32_t)want);
            if (hit == 0) {
                if (lane == 63) { s_H = HB - 1; s_tot = (int)incl; }
            } else if (lane == __builtin_ctzll(hit)) {
                uint32_t run = incl - sum;
                int h = h0;
                for (; h < h0 + SEG && h < HB; h++) {
                    run += hist[0][h];
                    if (run >= (uint32_t)want) break;
                }
                s_H = h;
                s_tot = (int)run;
            }
        }
        __syncthreads();
    };
    threshold(R);
    const int HR = s_H;
    // 2. the blocks holding every row at or below H_R
    for (int64_t b = tid; b < nblk; b += 256) {
        const float v = Bq[b];
        if (v <= (float)HR) {
            const int p = atomicAdd(&s_ncb, 1);
            if (p < BQF_CB) cblk[p] = (uint32_t)b; else s_fail = 1;
        }
    }
    for (int i = tid; i < HB; i += 256) hist[0][i] = 0u;
    __syncthreads();
    // 3. their rows' hamming distances (half a wave per block), rows <= H_R kept
    if (!s_fail) {
        const uint64_t* qc = qcodes + qlist[li];
        uint64_t qw[NW];
#pragma unroll
        for (int c = 0; c < NW; c++) qw[c] = c < words ? qc[(int64_t)c * ldq] : 0ull;
        const int ncb = s_ncb;
        for (int i = tid >> 5; i < ncb; i += 8) {
            const int64_t slot = (int64_t)cblk[i] * 32 + (tid & 31);
            const bool ok = slot < nslots && ((valid[slot >> 5] >> (slot & 31)) & 1u);
            uint32_t h = 0;
#pragma unroll
            for (int c = 0; c < NW; c++)
                if (c < words) h += (uint32_t)__popcll((ok ? codes[(int64_t)c * ccap + slot] : 0ull) ^ qw[c]);
            if (ok && h <= (uint32_t)HR) {
                atomicAdd(&hist[0][h], 1u);
                const int p = atomicAdd(&s_nrow, 1);
                if (p < BQF_RC) { rslot[p] = (uint32_t)slot; rh[p] = (uint16_t)h; } else s_fail = 1;
            }
        }
    }
    __syncthreads();
    if (s_fail) { if (tid == 0) skip[li] = 0; return; }
    // 4. h*; U = rows <= h* (the heap holds min(R, |U|) of them: all of U
    //    when |U| <= R, else S plus part of T)
    threshold(R);
    const int hs = s_H;
    const int nrow = s_nrow;
    for (int p = tid; p < nrow; p += 256)
        if (rh[p] <= hs) {
            const int u = atomicAdd(&s_nu, 1);
            if (u < BQF_UC) { uslot[u] = rslot[p]; uh[u] = rh[p]; upick[u] = 0; } else s_fail = 1;
        }
    __syncthreads();
    if (s_fail) { if (tid == 0) skip[li] = 0; return; }
    const int nu = s_nu;
    // 5. exact-order distances (the rescoring's createDistanceCalc, as k_rescore_ids)
    const float* qv = Q + (int64_t)qlist[li] * dpad;
    for (int u = tid; u < nu; u += 256) {
        const float v = exact_dist<METRIC, VARIANT>(qv, X + (int64_t)uslot[u] * dpad, d);
        ud[u] = v;
        if (!(v < __builtin_inff()) || !(v > -__builtin_inff())) s_fail = 1;  // NaN / inf: the replay decides
    }
    __syncthreads();
    if (s_fail) { if (tid == 0) skip[li] = 0; return; }
    // 6. the m (+1) smallest, one block-wide argmin each
    const int csz = nu < R ? nu : R;
    const int m = k < csz ? k : csz;
    const int picks = csz > m ? m + 1 : m;
    const bool cut = nu > R;
    float prev = -__builtin_inff();
    bool good = true;
    for (int j = 0; j < picks; j++) {
        float bv = __builtin_inff();
        int bi = -1;
        for (int u = tid; u < nu; u += 256) {
            const float v = ud[u];
            if (!upick[u] && (bi < 0 || v < bv)) { bv = v; bi = u; }
        }
        for (int o = 32; o > 0; o >>= 1) {
            const float ov = __shfl_xor(bv, o);
            const int oi = __shfl_xor(bi, o);
            if (oi >= 0 && (bi < 0 || ov < bv || (ov == bv && oi < bi))) { bv = ov; bi = oi; }
        }
        if (lane == 0) { rd[w] = bv; ri[w] = bi; }
        __syncthreads();
        bv = rd[0]; bi = ri[0];
        for (int x = 1; x < 4; x++)
            if (ri[x] >= 0 && (bi < 0 || rd[x] < bv || (rd[x] == bv && ri[x] < bi))) { bv = rd[x]; bi = ri[x]; }
        __syncthreads();
        // strictly increasing and finite; when T was cut, the m results from S
        if (!(bv > prev) || !(bv < __builtin_inff()) || bi < 0) good = false;
        if (j < m && cut && bi >= 0 && uh[bi] >= hs) good = false;
        prev = bv;
        if (!good) break;
        if (tid == 0) {
            upick[bi] = 1;
            if (j < m) pslot[j] = uslot[bi];
        }
        __syncthreads();
    }
    if (tid == 0) skip[li] = good ? 1 : 0;
    if (!good) return;
    for (int j = tid; j < m; j += 256) out_ids[(int64_t)li * R + j] = id_base + pslot[j];
    if (tid == 0) out_n[li] = m;
}

// Rescoring heap (flat/index.go:525-531): the candidates, in pop order (asc = 1:
// stored ascending, i.e. extractHeap order, read back to front), go
// through insertToHeap(heap, k, id, dist); extractHeap gives the result.
// One wave per listed query; lane 0 runs the heap in LDS ([k] u64 | [k] f32).
// world > 1: candE is [world][nlist][R] (each shard's exact distances of the
// ids it holds); the entry of id comes from shard min(id / id_stride, world-1).
__global__ __launch_bounds__(64) void k_bq_final(const uint64_t* __restrict__ cand_ids,
                                                 const float* __restrict__ candE,
                                                 const int32_t* __restrict__ cand_n, const int32_t* __restrict__ qlist,
                                                 int nlist, int R, int k, int world, uint64_t id_stride,
                                                 uint64_t* __restrict__ out_ids, float* __restrict__ out_d,
                                                 int32_t* __restrict__ out_n, int asc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char fsm[];
    uint64_t* hid = reinterpret_cast<uint64_t*>(fsm);
    float* hd = reinterpret_cast<float*>(hid + k);
    const int li = blockIdx.x;
    if (li >= nlist || threadIdx.x != 0) return;
    const int q = qlist[li];
    ReplayHeap hp{hid, hd, 0};
    const int n = cand_n[li];
    for (int ii = 0; ii < n; ii++) {
        const int i = asc ? n - 1 - ii : ii;  // asc: candidates extracted ascending, pop order = reversed
        const uint64_t id = cand_ids[(int64_t)li * R + i];
        uint64_t owner = 0;
        if (world > 1) { owner = id / id_stride; if (owner > (uint64_t)(world - 1)) owner = world - 1; }
        const float dist = candE[(int64_t)owner * nlist * R + (int64_t)li * R + i];
        if (hp.len < k) rh_insert(hp, id, dist);
        else if (hp.dist[0] > dist) { uint64_t a; float b; rh_pop(hp, &a, &b); rh_insert(hp, id, dist); }
    }
    const int m = hp.len;
    for (int i = m - 1; i >= 0; i--) {
        uint64_t a; float b;
        rh_pop(hp, &a, &b);
        out_ids[(int64_t)q * k + i] = a;
        out_d[(int64_t)q * k + i] = b;
    }
    out_n[q] = m;
}

}  // namespace
}  // namespace wv
