/*
 * rq.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Scalar C restatement of flat's two rotational-quantization modes
 * (flat/quantizer.go:85-99: "rq-8" and "rq-1"):
 *   - FastRotation (compressionhelpers/fast_rotation.go:30-122): rounds of
 *     random swaps (rng.Perm, :48-70) + random signs (rng.Float64() < 0.5,
 *     :30-40) followed by blocked Walsh-Hadamard transforms (256-blocks while
 *     >= 256 entries remain, else 64-blocks, normalise first: :154-288);
 *     rng = PCG(seed, 0x385ab5285169b1ac) (:77), seed DefaultFastRotationSeed;
 *   - RotationalQuantizer (8 bits): encode (rotational_quantization.go:182-213,
 *     RQCode layout :95-155, big-endian floats) and
 *     DistanceBetweenCompressedVectors (:294-306), which flat uses with the
 *     candidate first and the encoded query second (flat/index.go:555-560);
 *   - BinaryRotationalQuantizer (RaBitQ 1 bit): rounding vector
 *     (binary_rotational_quantization.go:38-70, PCG(seed, 0x4f8ebf70e130707f)
 *     Float32), data Encode (:158-187), 5-bit query encodeQuery (:254-314),
 *     BinaryRQDistancer.Distance (:364-385);
 *   - flat.searchByVectorQuantized (flat/index.go:460-532) over RQ codes.
 * Go's math/rand/v2 (Perm via Shuffle/uint64n, Float64, Float32) is restated
 * from the standard library's published algorithm (pq.c): the swap/sign/
 * rounding streams are PARITY UNPINNED (no Go toolchain here); the transform,
 * encoders and distance formulas are pinned by the reference tests' properties
 * (tests/test_rq_oracle.py).  Go float32 arithmetic is unfused (GOAMD64=v1),
 * so every expression below rounds after each operation (-ffp-contract=off).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define RQ_ROUNDS 3
#define RQ_ROT_SEED_INC 0x385ab5285169b1acULL
#define BRQ_ROUND_SEED_INC 0x4f8ebf70e130707fULL

struct or_rq {
    int bits;       /* 8 or 1 */
    int metric;     /* OR_L2 / OR_DOT / OR_COSINE */
    int input_dim;  /* as the quantizer stores it (BRQ pads to >= 256) */
    int D;          /* rotation output dim: multiple of 64 */
    int rounds;
    uint16_t *sI, *sJ; /* [rounds][D/2] swaps sorted by I */
    float *signs;      /* [rounds][D] */
    float *rounding;   /* BRQ only: [D] */
};

/* math/rand/v2 Float32: float32(Uint32()<<8>>8) / (1<<24), Uint32 = top 32 bits */
static float pcg_f32(pcg_t *p) {
    uint32_t u = (uint32_t)(pcg_u64(p) >> 32);
    return (float)((u << 8) >> 8) / 16777216.0f;
}

static int cmp_swap(const void *a, const void *b) {
    const uint16_t *x = (const uint16_t *)a, *y = (const uint16_t *)b;
    return (int)x[0] - (int)y[0];
}

/* NewFastRotation (fast_rotation.go:72-90) */
static void build_rotation(or_rq *r, int input_dim, uint64_t seed) {
    int D = 64;
    while (D < input_dim) D += 64;
    r->D = D;
    r->rounds = RQ_ROUNDS;
    r->sI = (uint16_t *)malloc(sizeof(uint16_t) * RQ_ROUNDS * (D / 2));
    r->sJ = (uint16_t *)malloc(sizeof(uint16_t) * RQ_ROUNDS * (D / 2));
    r->signs = (float *)malloc(sizeof(float) * RQ_ROUNDS * D);
    pcg_t p = {seed, RQ_ROT_SEED_INC};
    int *perm = (int *)malloc(sizeof(int) * D);
    uint16_t *pairs = (uint16_t *)malloc(sizeof(uint16_t) * D);
    for (int rd = 0; rd < RQ_ROUNDS; rd++) {
        /* randomSwaps: p := rng.Perm(n) (Shuffle: Fisher-Yates with uint64n) */
        for (int i = 0; i < D; i++) perm[i] = i;
        for (int i = D - 1; i > 0; i--) {
            int j = (int)pcg_u64n(&p, (uint64_t)(i + 1));
            int t = perm[i]; perm[i] = perm[j]; perm[j] = t;
        }
        for (int s = 0; s < D / 2; s++) {
            uint16_t a = (uint16_t)perm[2 * s], b = (uint16_t)perm[2 * s + 1];
            pairs[2 * s] = a < b ? a : b;
            pairs[2 * s + 1] = a < b ? b : a;
        }
        /* slices.SortFunc by I: the I values are distinct, so any sort agrees */
        qsort(pairs, (size_t)(D / 2), 2 * sizeof(uint16_t), cmp_swap);
        for (int s = 0; s < D / 2; s++) {
            r->sI[rd * (D / 2) + s] = pairs[2 * s];
            r->sJ[rd * (D / 2) + s] = pairs[2 * s + 1];
        }
        /* randomSigns */
        for (int i = 0; i < D; i++) r->signs[rd * D + i] = pcg_f64(&p) < 0.5 ? -1.0f : 1.0f;
    }
    free(perm);
    free(pairs);
}

or_rq *or_rq_new(int bits, int metric, int dims, uint64_t seed) {
    if (bits != 1 && bits != 8) return NULL;
    if (metric != OR_L2 && metric != OR_DOT && metric != OR_COSINE) return NULL;
    or_rq *r = (or_rq *)calloc(1, sizeof(or_rq));
    r->bits = bits;
    r->metric = metric;
    r->input_dim = (bits == 1 && dims < 256) ? 256 : dims; /* minCodeBits (:26, :40-42) */
    build_rotation(r, r->input_dim, seed);
    if (bits == 1) {
        r->rounding = (float *)malloc(sizeof(float) * r->D);
        pcg_t p = {seed, BRQ_ROUND_SEED_INC};
        for (int i = 0; i < r->D; i++) r->rounding[i] = pcg_f32(&p);
    }
    return r;
}

void or_rq_free(or_rq *r) {
    if (!r) return;
    free(r->sI); free(r->sJ); free(r->signs); free(r->rounding); free(r);
}

int or_rq_out_dim(const or_rq *r) { return r->D; }

/* exported tables for the tests: sI/sJ [rounds][D/2], signs [rounds][D], rounding [D] */
void or_rq_tables(const or_rq *r, uint16_t *sI, uint16_t *sJ, float *signs, float *rounding) {
    memcpy(sI, r->sI, sizeof(uint16_t) * r->rounds * (r->D / 2));
    memcpy(sJ, r->sJ, sizeof(uint16_t) * r->rounds * (r->D / 2));
    memcpy(signs, r->signs, sizeof(float) * r->rounds * r->D);
    if (rounding && r->rounding) memcpy(rounding, r->rounding, sizeof(float) * r->D);
}

/* Walsh-Hadamard transform of one block: scale every entry by `normalize`
 * first (fastWalshHadamardTransform16 multiplies on load), then butterflies
 * with strides 1, 2, 4, ... (fast_rotation.go:154-288 performs exactly these
 * butterflies; independent butterflies commute). */
static void fwht_block(float *x, int n, float normalize) {
    for (int i = 0; i < n; i++) x[i] = normalize * x[i];
    for (int h = 1; h < n; h <<= 1)
        for (int i = 0; i < n; i++)
            if ((i & h) == 0) {
                float a = x[i], b = x[i + h];
                x[i] = a + b;
                x[i + h] = a - b;
            }
}

void or_fwht64(float *x) { fwht_block(x, 64, 0.125f); }
void or_fwht256(float *x) { fwht_block(x, 256, 0.0625f); }

/* FastRotation.Rotate (fast_rotation.go:101-122); x has n <= D entries */
void or_rq_rotate(const or_rq *r, const float *x, long n, float *rx) {
    const int D = r->D;
    for (int i = 0; i < D; i++) rx[i] = i < n ? x[i] : 0.0f;
    for (int rd = 0; rd < r->rounds; rd++) {
        const uint16_t *sI = r->sI + rd * (D / 2), *sJ = r->sJ + rd * (D / 2);
        const float *sg = r->signs + rd * D;
        for (int s = 0; s < D / 2; s++) {
            int I = sI[s], J = sJ[s];
            float a = sg[I] * rx[J], b = sg[J] * rx[I];
            rx[I] = a;
            rx[J] = b;
        }
        int pos = 0;
        while (pos < D) {
            if (D - pos >= 256) { fwht_block(rx + pos, 256, 0.0625f); pos += 256; }
            else { fwht_block(rx + pos, 64, 0.125f); pos += 64; }
        }
    }
}

static void put_be(uint8_t *b, float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    b[0] = (uint8_t)(u >> 24); b[1] = (uint8_t)(u >> 16); b[2] = (uint8_t)(u >> 8); b[3] = (uint8_t)u;
}
static float get_be(const uint8_t *b) {
    uint32_t u = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
    float x;
    memcpy(&x, &u, 4);
    return x;
}

/* RotationalQuantizer.encode (rotational_quantization.go:182-213) with
 * bits = 8 into the RQCode layout [lower|step|codeSum|norm2 (BE f32)][D bytes].
 * norm2 = dotProduct(x, x) = -DotProductProvider.SingleDist (the SIMD kernel of
 * `variant`). */
void or_rq8_encode(const or_rq *r, int variant, const float *x, long n, uint8_t *code) {
    const int D = r->D;
    memset(code, 0, (size_t)D + 16);
    if (n == 0) return;
    if (n > D) n = D;
    float *rx = (float *)malloc(sizeof(float) * D);
    or_rq_rotate(r, x, n, rx);
    float lo = rx[0], hi = rx[0];
    for (int i = 1; i < D; i++) { if (rx[i] < lo) lo = rx[i]; if (rx[i] > hi) hi = rx[i]; }
    const float step = (hi - lo) / 255.0f;
    if (step <= 0) { free(rx); return; } /* ZeroRQCode */
    float codeSum = 0.0f;
    for (int i = 0; i < D; i++) {
        float t = (rx[i] - lo) / step;
        t = t + 0.5f;
        uint8_t c = (uint8_t)(long long)t;
        codeSum += (float)c;
        code[16 + i] = c;
    }
    float dot = variant == OR_AVX512 ? or_dot_512(x, x, n) : or_dot_256(x, x, n);
    put_be(code + 0, lo);
    put_be(code + 4, step);
    put_be(code + 8, step * codeSum);
    put_be(code + 12, dot); /* -(-dot) */
    free(rx);
}

static float rq_indicator_cos(int metric) { return metric == OR_COSINE ? 1.0f : 0.0f; }
static float rq_indicator_l2(int metric) { return metric == OR_L2 ? 1.0f : 0.0f; }

/* DistanceBetweenCompressedVectors (rotational_quantization.go:294-306),
 * x = candidate code, y = query code; dotByteImpl = uint32 sum of byte products */
float or_rq8_distance(const or_rq *r, const uint8_t *cx, const uint8_t *cy) {
    const int D = r->D;
    uint32_t dot = 0;
    for (int i = 0; i < D; i++) dot += (uint32_t)cx[16 + i] * (uint32_t)cy[16 + i];
    const float xl = get_be(cx), xs = get_be(cx + 4), xc = get_be(cx + 8), xn = get_be(cx + 12);
    const float yl = get_be(cy), ys = get_be(cy + 4), yc = get_be(cy + 8), yn = get_be(cy + 12);
    float a = (float)D * xl;
    a = a * yl;
    const float b = xl * yc;
    const float c = yl * xc;
    float d = xs * ys;
    d = d * (float)dot;
    float est = a + b;
    est = est + c;
    est = est + d;
    const float l2 = rq_indicator_l2(r->metric), cos = rq_indicator_cos(r->metric);
    float t = l2 * (xn + yn);
    t = t + cos;
    return t - (1.0f + l2) * est;
}

/* BinaryRotationalQuantizer.Encode (binary_rotational_quantization.go:158-187):
 * code[0] = step (low 32 bits) | squared norm (high 32 bits), then D/64 sign words */
void or_brq_encode(const or_rq *r, const float *x, long n, uint64_t *code) {
    const int D = r->D, W = D / 64;
    float *rx = (float *)malloc(sizeof(float) * D);
    or_rq_rotate(r, x, n, rx);
    float l2 = 0.0f, l1 = 0.0f;
    memset(code, 0, sizeof(uint64_t) * (1 + W));
    int i = 0;
    for (int b = 0; b < W; b++) {
        uint64_t bits = 0;
        for (int j = 0; j < 64; j++, i++) {
            if (rx[i] > 0) { bits |= 1ull << j; l1 += rx[i]; }
            else l1 += -rx[i];
            float sq = rx[i] * rx[i];
            l2 += sq;
        }
        code[1 + b] = bits;
    }
    free(rx);
    if (l1 == 0) return;
    const float step = l2 / l1;
    uint32_t us, un;
    memcpy(&us, &step, 4);
    memcpy(&un, &l2, 4);
    code[0] = ((uint64_t)un << 32) | us;
}

/* encodeQuery (:254-314): 5 bit planes [5][W], *dim = D (0 for the zero vector) */
void or_brq_encode_query(const or_rq *r, const float *x, long n, float *step_out, float *sqn_out, int *dim_out,
                         uint64_t *planes) {
    const int D = r->D, W = D / 64;
    float *rx = (float *)malloc(sizeof(float) * D);
    or_rq_rotate(r, x, n, rx);
    memset(planes, 0, sizeof(uint64_t) * 5 * W);
    float mx = 0.0f;
    for (int i = 0; i < D; i++) { float v = rx[i] < 0 ? -rx[i] : rx[i]; if (v > mx) mx = v; }
    *step_out = 0.0f; *sqn_out = 0.0f; *dim_out = 0;
    if (mx == 0) { free(rx); return; }
    const float step = mx / 31.0f;
    float sqn = 0.0f;
    int i = 0;
    for (int b = 0; b < W; b++) {
        for (int j = 0; j < 64; j++, i++) {
            float sq = rx[i] * rx[i];
            sqn += sq;
            float t = rx[i] + mx;
            t = t / (2.0f * step);
            t = t + r->rounding[i];
            uint64_t c = (uint64_t)t;
            for (int p = 0; p < 5; p++)
                if (c & (1ull << p)) planes[p * W + b] |= 1ull << j;
        }
    }
    *step_out = step;
    *sqn_out = sqn;
    *dim_out = D;
    free(rx);
}

/* BinaryRQDistancer.Distance (:364-385); both of its branches compute the same
 * exact integer, converted to float32 */
float or_brq_distance(const or_rq *r, float qstep, float qsqn, int qdim, const uint64_t *planes,
                      const uint64_t *cx) {
    const int W = r->D / 64;
    long dot = 0;
    if (qdim > 0) {
        dot = 31L * qdim;
        for (int p = 0; p < 5; p++) {
            long h = 0;
            for (int w = 0; w < W; w++) h += __builtin_popcountll(planes[p * W + w] ^ cx[1 + w]);
            dot -= h << (p + 1);
        }
    }
    uint32_t us = (uint32_t)cx[0], un = (uint32_t)(cx[0] >> 32);
    float xstep, xsqn;
    memcpy(&xstep, &us, 4);
    memcpy(&xsqn, &un, 4);
    float est = qstep * xstep;
    est = est * (float)dot;
    const float l2 = rq_indicator_l2(r->metric), cos = rq_indicator_cos(r->metric);
    float t = l2 * (xsqn + qsqn);
    t = t + cos;
    return t - (1.0f + l2) * est;
}

/* flat.searchByVectorQuantized (flat/index.go:460-532) for rq-8 / rq-1:
 * R-heap of quantized distances over the present rows in id order, popped
 * max-first, fp32 SingleDist rescoring, then insertToHeap(k) in pop order and
 * extractHeap.  codes: rq-8 [nslots][16+D] bytes, rq-1 [nslots][1+D/64] words. */
int or_flat_search_rq(const or_rq *r, int variant, const float *store, const uint8_t *present, const void *codes,
                      long nslots, long d, const float *query, long qd, int k, int rescore_limit,
                      const uint8_t *allow, int allow_empty, uint64_t *out_ids, float *out_dists, int *out_n) {
    *out_n = 0;
    const int R = rescore_limit > k ? rescore_limit : k;
    if (allow && allow_empty) return 0;
    if (qd != d) return OR_ERR_VECTOR_LENGTH;
    const int D = r->D, W = D / 64;
    float *q = (float *)malloc(sizeof(float) * (qd > 0 ? qd : 1));
    if (r->metric == OR_COSINE) or_normalize(query, q, qd);
    else memcpy(q, query, sizeof(float) * qd);
    uint8_t *qc8 = NULL;
    uint64_t *planes = NULL;
    float qstep = 0, qsqn = 0;
    int qdim = 0;
    if (r->bits == 8) {
        qc8 = (uint8_t *)malloc((size_t)D + 16);
        or_rq8_encode(r, variant, q, qd, qc8);
    } else {
        planes = (uint64_t *)malloc(sizeof(uint64_t) * 5 * W);
        or_brq_encode_query(r, q, qd, &qstep, &qsqn, &qdim, planes);
    }
    or_heap h;
    h.len = 0;
    h.id = (uint64_t *)malloc(sizeof(uint64_t) * (R + 1));
    h.dist = (float *)malloc(sizeof(float) * (R + 1));
    for (long s = 0; s < nslots; s++) {
        if (!present[s]) continue;
        if (allow && !allow[s]) continue;
        float dist;
        if (r->bits == 8) dist = or_rq8_distance(r, (const uint8_t *)codes + (size_t)s * (D + 16), qc8);
        else dist = or_brq_distance(r, qstep, qsqn, qdim, planes, (const uint64_t *)codes + (size_t)s * (W + 1));
        or_insert_to_heap(&h, R, (uint64_t)s, dist);
    }
    const int n = h.len;
    uint64_t *ids = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
    float *dd = (float *)calloc(n + 1, sizeof(float));
    for (int i = 0; i < n; i++) { float tmp; or_heap_pop(&h, &ids[i], &tmp); }
    for (int i = 0; i < n; i++) dd[i] = or_single_dist(r->metric, variant, q, store + (size_t)ids[i] * d, d);
    for (int i = 0; i < n; i++) or_insert_to_heap(&h, k, ids[i], dd[i]);
    *out_n = or_extract_heap(&h, out_ids, out_dists);
    free(ids); free(dd); free(h.id); free(h.dist); free(q); free(qc8); free(planes);
    return 0;
}

/* quantized distances of one query against every present row (tests) */
void or_rq_query_distances(const or_rq *r, int variant, const void *codes, long nslots, const float *query, long qd,
                           float *out) {
    const int D = r->D, W = D / 64;
    float *q = (float *)malloc(sizeof(float) * (qd > 0 ? qd : 1));
    if (r->metric == OR_COSINE) or_normalize(query, q, qd);
    else memcpy(q, query, sizeof(float) * qd);
    if (r->bits == 8) {
        uint8_t *qc = (uint8_t *)malloc((size_t)D + 16);
        or_rq8_encode(r, variant, q, qd, qc);
        for (long s = 0; s < nslots; s++) out[s] = or_rq8_distance(r, (const uint8_t *)codes + (size_t)s * (D + 16), qc);
        free(qc);
    } else {
        uint64_t *planes = (uint64_t *)malloc(sizeof(uint64_t) * 5 * W);
        float st, sq;
        int dim;
        or_brq_encode_query(r, q, qd, &st, &sq, &dim, planes);
        for (long s = 0; s < nslots; s++)
            out[s] = or_brq_distance(r, st, sq, dim, planes, (const uint64_t *)codes + (size_t)s * (W + 1));
        free(planes);
    }
    free(q);
}
