/*
 * oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C, scalar restatement of the reference's flat-index hot path, used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg to check the
 * HIP path.  Nothing under weaviate_amd/ links or calls this file.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the reference repo root).  Compiled with -ffp-contract=off so that the only
 * fused multiply-adds are the explicit fmaf() calls, placed exactly where the
 * reference's generated assembly uses vfmadd.
 *
 * Parity pins (tests/test_oracle.py): every distance kernel below is compared
 * bit-for-bit against the reference's own C sources compiled from
 * /root/reference by oracle/Makefile into oracle/_ref/libref.so, plus the
 * known-answer vectors of distancer/{l2,dot_product,cosine_dist,hamming}_test.go and
 * compressionhelpers/binary_quantization_test.go.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* distance kernels                                                           */
/* ------------------------------------------------------------------------- */

/* Final reduction shared by all four float kernels:
 * adapters/repos/db/vector/hnsw/distancer/c/l2_avx256_amd64.c:97-104
 *   acc0 = acc1 + acc0; acc2 = acc3 + acc2; acc0 = acc2 + acc0;
 *   t1 = hadd(acc0, acc0); t2 = hadd(t1, t1); t4 = lo128(t2) + hi128(t2)
 * lane l of the result t4[0] = ((v0+v1)+(v2+v3)) + ((v4+v5)+(v6+v7)). */
static float reduce_ymm4(float acc[4][8]) {
    float v[8];
    for (int l = 0; l < 8; l++) {
        float a01 = acc[1][l] + acc[0][l];
        float a23 = acc[3][l] + acc[2][l];
        v[l] = a23 + a01;
    }
    float h0 = v[0] + v[1], h1 = v[2] + v[3], h4 = v[4] + v[5], h5 = v[6] + v[7];
    float lo = h0 + h1, hi = h4 + h5;
    return lo + hi;
}

/* AVX-512 fold of the 8 zmm accumulators:
 * c/l2_avx512_amd64.c:100-112 (pairwise tree, then low/high 8 lanes folded
 * into acc[0]). */
static void fold_zmm8(float acc5[8][16], float acc[4][8]) {
    for (int j = 0; j < 16; j++) {
        acc5[0][j] = acc5[1][j] + acc5[0][j];
        acc5[2][j] = acc5[3][j] + acc5[2][j];
        acc5[4][j] = acc5[5][j] + acc5[4][j];
        acc5[6][j] = acc5[7][j] + acc5[6][j];
        acc5[0][j] = acc5[2][j] + acc5[0][j];
        acc5[4][j] = acc5[6][j] + acc5[4][j];
        acc5[0][j] = acc5[4][j] + acc5[0][j];
    }
    for (int l = 0; l < 8; l++) acc[0][l] = acc5[0][l] + acc[0][l];
    for (int l = 0; l < 8; l++) acc[0][l] = acc5[0][8 + l] + acc[0][l];
}

/* element op of each kernel: L2 = fma(d,d,acc) with d = a-b rounded; DOT = fma(a,b,acc) */
#define L2_STEP(acc, x, y) do { float _d = (x) - (y); (acc) = fmaf(_d, _d, (acc)); } while (0)
#define DOT_STEP(acc, x, y) do { (acc) = fmaf((x), (y), (acc)); } while (0)

/* l2_256: c/l2_avx256_amd64.c:14-107.
 * n<8 and tail: scalar mul then add (asm/l2_avx256_amd64.s vsubss/vmulss/vaddss). */
float or_l2_256(const float *a, const float *b, long len) {
    int n = (int)len;
    float sum = 0.f;
    if (n < 8) {
        do { float diff = a[0] - b[0]; float sq = diff * diff; sum = sum + sq; n--; a++; b++; } while (n > 0);
        return sum;
    }
    float acc[4][8] = {{0}};
    while (n >= 32) {
        for (int j = 0; j < 4; j++) for (int l = 0; l < 8; l++) L2_STEP(acc[j][l], a[8 * j + l], b[8 * j + l]);
        n -= 32; a += 32; b += 32;
    }
    while (n >= 8) {
        for (int l = 0; l < 8; l++) L2_STEP(acc[0][l], a[l], b[l]);
        n -= 8; a += 8; b += 8;
    }
    while (n) { float diff = a[0] - b[0]; float sq = diff * diff; sum = sum + sq; n--; a++; b++; }
    return sum + reduce_ymm4(acc);
}

/* l2_512: c/l2_avx512_amd64.c:14-197 (adds the n>=128 zmm block :43-122). */
float or_l2_512(const float *a, const float *b, long len) {
    int n = (int)len;
    float sum = 0.f;
    if (n < 8) {
        do { float diff = a[0] - b[0]; float sq = diff * diff; sum = sum + sq; n--; a++; b++; } while (n > 0);
        return sum;
    }
    float acc[4][8] = {{0}};
    if (n >= 128) {
        float acc5[8][16] = {{0}};
        do {
            for (int r = 0; r < 8; r++) for (int j = 0; j < 16; j++) L2_STEP(acc5[r][j], a[16 * r + j], b[16 * r + j]);
            n -= 128; a += 128; b += 128;
        } while (n >= 128);
        fold_zmm8(acc5, acc);
        if (!n) return sum + reduce_ymm4(acc);
    }
    while (n >= 32) {
        for (int j = 0; j < 4; j++) for (int l = 0; l < 8; l++) L2_STEP(acc[j][l], a[8 * j + l], b[8 * j + l]);
        n -= 32; a += 32; b += 32;
    }
    while (n >= 8) {
        for (int l = 0; l < 8; l++) L2_STEP(acc[0][l], a[l], b[l]);
        n -= 8; a += 8; b += 8;
    }
    while (n) { float diff = a[0] - b[0]; float sq = diff * diff; sum = sum + sq; n--; a++; b++; }
    return sum + reduce_ymm4(acc);
}

/* dot_256: c/dot_avx256_amd64.c:14-97.  n<8 and tail are FMA
 * (`sum += a*b` contracted by clang: asm/dot_avx256_amd64.s vfmadd231ss). */
float or_dot_256(const float *a, const float *b, long len) {
    int n = (int)len;
    float sum = 0.f;
    if (n < 8) {
        do { sum = fmaf(a[0], b[0], sum); n--; a++; b++; } while (n > 0);
        return sum;
    }
    float acc[4][8] = {{0}};
    while (n >= 32) {
        for (int j = 0; j < 4; j++) for (int l = 0; l < 8; l++) DOT_STEP(acc[j][l], a[8 * j + l], b[8 * j + l]);
        n -= 32; a += 32; b += 32;
    }
    while (n >= 8) {
        for (int l = 0; l < 8; l++) DOT_STEP(acc[0][l], a[l], b[l]);
        n -= 8; a += 8; b += 8;
    }
    while (n) { sum = fmaf(a[0], b[0], sum); n--; a++; b++; }
    return sum + reduce_ymm4(acc);
}

/* dot_512: c/dot_avx512_amd64.c:14-177. */
float or_dot_512(const float *a, const float *b, long len) {
    int n = (int)len;
    float sum = 0.f;
    if (n < 8) {
        do { sum = fmaf(a[0], b[0], sum); n--; a++; b++; } while (n > 0);
        return sum;
    }
    float acc[4][8] = {{0}};
    if (n >= 128) {
        float acc5[8][16] = {{0}};
        do {
            for (int r = 0; r < 8; r++) for (int j = 0; j < 16; j++) DOT_STEP(acc5[r][j], a[16 * r + j], b[16 * r + j]);
            n -= 128; a += 128; b += 128;
        } while (n >= 128);
        fold_zmm8(acc5, acc);
        if (!n) return sum + reduce_ymm4(acc);
    }
    while (n >= 32) {
        for (int j = 0; j < 4; j++) for (int l = 0; l < 8; l++) DOT_STEP(acc[j][l], a[8 * j + l], b[8 * j + l]);
        n -= 32; a += 32; b += 32;
    }
    while (n >= 8) {
        for (int l = 0; l < 8; l++) DOT_STEP(acc[0][l], a[l], b[l]);
        n -= 8; a += 8; b += 8;
    }
    while (n) { sum = fmaf(a[0], b[0], sum); n--; a++; b++; }
    return sum + reduce_ymm4(acc);
}

/* Float-element hamming: c/hamming_avx256_amd64.c:14-137 and
 * c/hamming_avx512_amd64.c.  Elements handled by SIMD compares use
 * _CMP_NEQ_OQ (NaN compares equal -> 0); the n<8 path and the scalar tail use
 * C `!=` (NaN -> 1).  In both variants the SIMD blocks are multiples of 8, so
 * the scalar elements are: all of them when n<8, otherwise the last n%8. */
float or_hamming_f32(const float *a, const float *b, long len) {
    int n = (int)len;
    int sum = 0;
    if (n < 8) {
        for (int i = 0; i < n; i++) sum += (a[i] != b[i]) ? 1 : 0;
        return (float)sum;
    }
    int simd = n - (n % 8);
    for (int i = 0; i < simd; i++) {
        /* ordered not-equal: false if either is NaN */
        int ord_neq = !(isnan(a[i]) || isnan(b[i])) && (a[i] != b[i]);
        sum += ord_neq;
    }
    for (int i = simd; i < n; i++) sum += (a[i] != b[i]) ? 1 : 0;
    return (float)sum;
}

/* distancer.HammingBitwise: distancer/hamming.go:63-68 ->
 * c/hamming_bitwise_avx256_amd64.c:43-127; exact popcount(x^y) summed as
 * uint64 then float32(res) (asm/hamming_amd64.go:69-83). */
float or_hamming_bitwise(const uint64_t *a, const uint64_t *b, long n) {
    uint64_t sum = 0;
    for (long i = 0; i < n; i++) sum += (uint64_t)__builtin_popcountll(a[i] ^ b[i]);
    return (float)sum;
}

/* distancer.Normalize: distancer/normalize.go:16-32.  Sequential fp32 sum of
 * v*v (not fused: Go amd64 default GOAMD64=v1 has no FMA contraction),
 * norm = float32(sqrt(float64(norm))), out[i] = v[i]/norm; zero -> zeros. */
void or_normalize(const float *v, float *out, long n) {
    float norm = 0.f;
    for (long i = 0; i < n; i++) { float sq = v[i] * v[i]; norm = norm + sq; }
    if (norm == 0.f) { for (long i = 0; i < n; i++) out[i] = 0.f; return; }
    norm = (float)sqrt((double)norm);
    for (long i = 0; i < n; i++) out[i] = v[i] / norm;
}

/* Provider.SingleDist + dispatch (distancer/l2.go:46, dot_product.go:68,
 * cosine_dist.go:42, hamming.go:80; l2_amd64.go:19-26). */
float or_single_dist(int metric, int variant, const float *a, const float *b, long n) {
    switch (metric) {
    case OR_L2:
        return variant == OR_AVX512 ? or_l2_512(a, b, n) : or_l2_256(a, b, n);
    case OR_DOT: {
        float d = variant == OR_AVX512 ? or_dot_512(a, b, n) : or_dot_256(a, b, n);
        return -d;
    }
    case OR_COSINE: {
        float d = variant == OR_AVX512 ? or_dot_512(a, b, n) : or_dot_256(a, b, n);
        float prod = 1.f - d;
        if (prod < 0) return 0.f;
        return prod;
    }
    case OR_HAMMING:
        return or_hamming_f32(a, b, n);
    }
    return NAN;
}

/* ------------------------------------------------------------------------- */
/* priority queue: adapters/repos/db/priorityqueue/queue.go:58-198 (NewMax)   */
/* ------------------------------------------------------------------------- */

static int h_less(const or_heap *h, int i, int j) { return h->dist[i] > h->dist[j]; } /* queue.go:61-64 */
static void h_swap(or_heap *h, int i, int j) {
    uint64_t ti = h->id[i]; h->id[i] = h->id[j]; h->id[j] = ti;
    float td = h->dist[i]; h->dist[i] = h->dist[j]; h->dist[j] = td;
}
/* queue.go:156-164 */
void or_heap_insert(or_heap *h, uint64_t id, float dist) {
    h->id[h->len] = id; h->dist[h->len] = dist; h->len++;
    int i = h->len - 1;
    while (i != 0 && h_less(h, i, (i - 1) / 2)) { h_swap(h, i, (i - 1) / 2); i = (i - 1) / 2; }
}
/* queue.go:182-198 (recursive heapify, written iteratively) */
static void h_heapify(or_heap *h, int i) {
    for (;;) {
        int left = 2 * i + 1, right = 2 * i + 2, smallest = i;
        if (left < h->len && h_less(h, left, i)) smallest = left;
        if (right < h->len && h_less(h, right, smallest)) smallest = right;
        if (smallest == i) return;
        h_swap(h, i, smallest);
        i = smallest;
    }
}
/* queue.go:85-91 */
void or_heap_pop(or_heap *h, uint64_t *id, float *dist) {
    *id = h->id[0]; *dist = h->dist[0];
    h->id[0] = h->id[h->len - 1]; h->dist[0] = h->dist[h->len - 1];
    h->len--;
    h_heapify(h, 0);
}
/* flat/index.go:665-674 insertToHeap */
void or_insert_to_heap(or_heap *h, int limit, uint64_t id, float dist) {
    if (h->len < limit) or_heap_insert(h, id, dist);
    else if (h->dist[0] > dist) { uint64_t a; float b; or_heap_pop(h, &a, &b); or_heap_insert(h, id, dist); }
}
/* flat/index.go:676-688 extractHeap: pop max-first, fill from the back */
int or_extract_heap(or_heap *h, uint64_t *ids, float *dists) {
    int n = h->len;
    for (int i = n - 1; i >= 0; i--) or_heap_pop(h, &ids[i], &dists[i]);
    return n;
}

/* ------------------------------------------------------------------------- */
/* flat index scan                                                             */
/* ------------------------------------------------------------------------- */

/* flat/index.go:578-619 findTopVectors, over an ID-indexed store: slot s holds
 * doc id s; present[s]!=0 means the LSM bucket has the key.  Scan is in
 * ascending id order (the replace bucket's big-endian key order); allow is a
 * per-slot bitmap (NULL = allow nil).  `heap` may hold a starting state (used
 * to replay a contiguous id range after a preceding range). */
int or_find_top_vectors(or_heap *heap, int limit, int metric, int variant,
                        const float *store, const uint8_t *present, long nslots, long d,
                        const float *query, long qd, const uint8_t *allow, long slot_begin, long slot_end) {
    for (long s = slot_begin; s < slot_end && s < nslots; s++) {
        if (!present[s]) continue;
        if (allow && !allow[s]) continue;
        if (qd != d) return OR_ERR_VECTOR_LENGTH; /* SingleDist: ErrVectorLength */
        float dist = or_single_dist(metric, variant, query, store + (size_t)s * d, d);
        or_insert_to_heap(heap, limit, (uint64_t)s, dist);
    }
    return 0;
}

/* flat/index.go:432-448 searchByVector (+ :690-697 normalized).
 * allow_nonnull && allow_empty -> empty result (index.go:590-594). */
int or_flat_search(int metric, int variant, const float *store, const uint8_t *present, long nslots,
                   long d, const float *query, long qd, int k, const uint8_t *allow, int allow_empty,
                   uint64_t *out_ids, float *out_dists, int *out_n) {
    *out_n = 0;
    if (allow && allow_empty) return 0;
    float *q = (float *)malloc(sizeof(float) * (qd > 0 ? qd : 1));
    if (metric == OR_COSINE) or_normalize(query, q, qd);
    else memcpy(q, query, sizeof(float) * qd);
    or_heap h;
    h.len = 0;
    h.id = (uint64_t *)malloc(sizeof(uint64_t) * (k + 1));
    h.dist = (float *)malloc(sizeof(float) * (k + 1));
    int rc = or_find_top_vectors(&h, k, metric, variant, store, present, nslots, d, q, qd, allow, 0, nslots);
    if (rc == 0) *out_n = or_extract_heap(&h, out_ids, out_dists);
    free(h.id); free(h.dist); free(q);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* binary quantization                                                          */
/* ------------------------------------------------------------------------- */

/* compressionhelpers/binary_quantization.go:28-47: bit (i%64) of word i/64 is
 * set iff vec[i] < 0; padding bits stay 0. */
void or_bq_encode(const float *vec, long d, uint64_t *code) {
    long blocks = (d + 63) >> 6;
    for (long b = 0; b < blocks; b++) code[b] = 0;
    for (long i = 0; i < d; i++)
        if (vec[i] < 0) code[i >> 6] |= (uint64_t)1 << (i & 63);
}

/* flat/index.go:413-421 searchTimeRescore + :460-532 searchByVectorQuantized
 * (cached and uncached paths visit ids in the same ascending order:
 * flat/quantizer.go:302-346).  codes: nslots x words, valid where present.
 * A present slot whose fp32 vector is missing keeps distance 0 (:507-509):
 * modelled by fp32_present[s]==0. */
int or_flat_search_bq(int metric, int variant, const float *store, const uint8_t *present,
                      const uint8_t *fp32_present, const uint64_t *codes, long nslots, long d,
                      const float *query, long qd, int k, int rescore_limit, const uint8_t *allow,
                      int allow_empty, uint64_t *out_ids, float *out_dists, int *out_n) {
    *out_n = 0;
    int rescore = rescore_limit > k ? rescore_limit : k;
    if (allow && allow_empty) return 0;
    long words = (d + 63) >> 6;
    float *q = (float *)malloc(sizeof(float) * (qd > 0 ? qd : 1));
    if (metric == OR_COSINE) or_normalize(query, q, qd);
    else memcpy(q, query, sizeof(float) * qd);
    long qwords = (qd + 63) >> 6;
    uint64_t *qcode = (uint64_t *)calloc(qwords > 0 ? qwords : 1, sizeof(uint64_t));
    or_bq_encode(q, qd, qcode);
    or_heap h;
    int cap = rescore > k ? rescore : k;
    h.len = 0;
    h.id = (uint64_t *)malloc(sizeof(uint64_t) * (cap + 1));
    h.dist = (float *)malloc(sizeof(float) * (cap + 1));
    int rc = 0;
    for (long s = 0; s < nslots; s++) {
        if (!present[s]) continue;
        if (allow && !allow[s]) continue;
        if (qwords != words) { rc = OR_ERR_HAMMING_LENGTH; break; }
        float dist = or_hamming_bitwise(codes + (size_t)s * words, qcode, words);
        or_insert_to_heap(&h, rescore, (uint64_t)s, dist);
    }
    if (rc == 0) {
        int n = h.len;
        uint64_t *ids = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
        float *dd = (float *)calloc(n + 1, sizeof(float));
        for (int i = 0; i < n; i++) { float tmp; or_heap_pop(&h, &ids[i], &tmp); }
        for (int i = 0; i < n; i++) {
            long s = (long)ids[i];
            if (!fp32_present[s]) continue; /* len(candidateAsBytes)==0 -> dist stays 0 */
            if (qd != d) { rc = OR_ERR_VECTOR_LENGTH; break; }
            dd[i] = or_single_dist(metric, variant, q, store + (size_t)s * d, d);
        }
        if (rc == 0) {
            for (int i = 0; i < n; i++) or_insert_to_heap(&h, k, ids[i], dd[i]);
            *out_n = or_extract_heap(&h, out_ids, out_dists);
        }
        free(ids); free(dd);
    }
    free(h.id); free(h.dist); free(q); free(qcode);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* SearchByVectorDistance: flat/index.go:699-761 + common/search_by_dist_params.go */
/* ------------------------------------------------------------------------- */

/* The reference's loop (`for shouldContinue, err = recursiveSearch(); cond; {}`)
 * has no post statement, so recursiveSearch runs exactly once with
 * totalLimit = DefaultSearchByDistInitialLimit (100); the loop then only
 * advances the params until MaxLimitReached (and never ends for maxLimit<0 --
 * this restatement returns instead).  Kept ids: dist <= target or
 * |dist-target| <= 1e-6 in float64 (usecases/floatcomp), stopping at the first
 * miss.  `searcher` results are passed in (the caller ran SearchByVector with
 * k=100). */
int or_filter_by_distance(const uint64_t *ids, const float *dists, int n, float target,
                          uint64_t *out_ids, float *out_dists) {
    int lim = n < 100 ? n : 100;
    int m = 0;
    for (int i = 0; i < lim; i++) {
        double diff = fabs((double)dists[i] - (double)target);
        if (dists[i] <= target || diff <= 1e-6) { out_ids[m] = ids[i]; out_dists[m] = dists[i]; m++; }
        else break;
    }
    return m;
}

/* ------------------------------------------------------------------------- */
/* synthetic data: counter-based generator shared with the HIP generator       */
/* (weaviate_amd/csrc/gen.hip); value depends only on (seed, row, col).        */
/* ------------------------------------------------------------------------- */
static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
uint64_t or_gen_bits(uint64_t seed, uint64_t row, uint64_t col) {
    return mix64(seed * 0x9E3779B97F4A7C15ULL + (row << 16) + col + 0x632BE59BD9B4E019ULL);
}
/* kind 0: U[-1,1) step 2^-23; kind 1: integer U{0..127}; kind 2: U[0,1) step 2^-24 */
float or_gen_value(int kind, uint64_t seed, uint64_t row, uint64_t col) {
    uint64_t h = or_gen_bits(seed, row, col);
    if (kind == 1) return (float)(h >> 57);
    if (kind == 2) return (float)(h >> 40) * 5.9604644775390625e-08f;
    return (float)(h >> 40) * 1.1920928955078125e-07f - 1.0f;
}
void or_gen_matrix(int kind, uint64_t seed, uint64_t row0, long rows, long d, float *out) {
    for (long r = 0; r < rows; r++)
        for (long c = 0; c < d; c++) out[(size_t)r * d + c] = or_gen_value(kind, seed, row0 + r, c);
}

/* in-place distancer.Normalize over n rows (test / baseline data prep) */
void or_normalize_rows(float *v, long n, long d) {
    float *tmp = (float *)malloc(sizeof(float) * (d > 0 ? d : 1));
    for (long r = 0; r < n; r++) {
        or_normalize(v + (size_t)r * d, tmp, d);
        memcpy(v + (size_t)r * d, tmp, sizeof(float) * d);
    }
    free(tmp);
}
