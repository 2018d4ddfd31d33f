/*
 * pq.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Scalar C restatement of the reference's product quantizer path:
 *   - Go math/rand/v2 PCG-DXSM source + Rand.IntN / Float64 / Perm (the Go
 *     standard library, not in /root/reference: restated from its published
 *     algorithm; no Go toolchain here, so this stream is PARITY UNPINNED);
 *   - kmeans.randomSubset / initializeRandom / updateCenters /
 *     updateCenterNeighbors / nearestWithPruning / nearestBruteForce / Fit
 *     (adapters/repos/db/vector/kmeans/kmeans.go:238-497), as configured by
 *     KMeansEncoder.Fit (compressionhelpers/kmeans_encoder.go:48-65: random
 *     init, graph pruning, 10 iterations, delta 0.01);
 *   - KMeansEncoder.Encode (kmeans_encoder.go:67-78), ProductQuantizer.Encode
 *     (product_quantization.go:426-432), DistanceLookUpTable.LookUp +
 *     Provider.Step / Wrap (product_quantization.go:85-104, distancer/l2.go:63-76,
 *     dot_product.go:87-98, cosine_dist.go:64-79);
 *   - hnsw.flatSearch with one worker (hnsw/flat_search.go:28-141, addResult
 *     :214-224) and rescore with one worker (hnsw/search.go:1047-1110).
 * The distance kernels are oracle.c's, pinned to the reference's compiled C.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* ---- Go math/rand/v2 ------------------------------------------------------ */

/* pcg.go: state = state * mul + inc (128-bit LCG) */
static void pcg_next(pcg_t *p, uint64_t *ohi, uint64_t *olo) {
    const uint64_t mulHi = 2549297995355413924ULL, mulLo = 4865540595714422341ULL;
    const uint64_t incHi = 6364136223846793005ULL, incLo = 1442695040888963407ULL;
    __uint128_t m = (__uint128_t)p->lo * mulLo;
    uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
    hi += p->hi * mulLo + p->lo * mulHi;
    __uint128_t s = (__uint128_t)lo + incLo;
    lo = (uint64_t)s;
    hi = hi + incHi + (uint64_t)(s >> 64);
    p->lo = lo;
    p->hi = hi;
    *ohi = hi;
    *olo = lo;
}

/* pcg.go Uint64: DXSM output */
uint64_t pcg_u64(pcg_t *p) {
    uint64_t hi, lo;
    pcg_next(p, &hi, &lo);
    const uint64_t cheapMul = 0xda942042e4dd58b5ULL;
    hi ^= hi >> 32;
    hi *= cheapMul;
    hi ^= hi >> 48;
    hi *= (lo | 1);
    return hi;
}

/* rand.go uint64n (64-bit platform): power of two mask, else Lemire */
uint64_t pcg_u64n(pcg_t *p, uint64_t n) {
    if ((n & (n - 1)) == 0) return pcg_u64(p) & (n - 1);
    __uint128_t m = (__uint128_t)pcg_u64(p) * n;
    uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
    if (lo < n) {
        uint64_t thresh = (0 - n) % n;
        while (lo < thresh) {
            m = (__uint128_t)pcg_u64(p) * n;
            hi = (uint64_t)(m >> 64);
            lo = (uint64_t)m;
        }
    }
    return hi;
}

double pcg_f64(pcg_t *p) { return (double)((pcg_u64(p) << 11) >> 11) / 9007199254740992.0; }

/* exported for tests: first `cnt` Uint64 draws of NewPCG(s1, s2) */
void or_pcg_stream(uint64_t s1, uint64_t s2, int cnt, uint64_t *out) {
    pcg_t p = {s1, s2};
    for (int i = 0; i < cnt; i++) out[i] = pcg_u64(&p);
}

/* kmeans.go:238-274 randomSubset(n, k, rng) */
static void random_subset(pcg_t *r, long n, int k, long *out) {
    if (k > n / 2) {
        long *perm = (long *)malloc(sizeof(long) * n);
        for (long i = 0; i < n; i++) perm[i] = i;
        for (long i = n - 1; i > 0; i--) { /* Shuffle: Fisher-Yates */
            long j = (long)pcg_u64n(r, (uint64_t)(i + 1));
            long t = perm[i]; perm[i] = perm[j]; perm[j] = t;
        }
        memcpy(out, perm, sizeof(long) * k);
        free(perm);
        return;
    }
    double *rank = (double *)malloc(sizeof(double) * n);
    unsigned char *seen = (unsigned char *)calloc(n, 1);
    long *keys = (long *)malloc(sizeof(long) * k);
    int cnt = 0;
    while (cnt < k) { /* m[r.IntN(n)] = r.Float64(): index first, then value */
        long i = (long)pcg_u64n(r, (uint64_t)n);
        double v = pcg_f64(r);
        if (!seen[i]) { seen[i] = 1; keys[cnt++] = i; }
        rank[i] = v;
    }
    /* sort by rank (insertion sort, stable; equal Float64 ranks do not occur) */
    for (int a = 1; a < k; a++) {
        long key = keys[a];
        int b = a - 1;
        while (b >= 0 && rank[keys[b]] > rank[key]) { keys[b + 1] = keys[b]; b--; }
        keys[b + 1] = key;
    }
    memcpy(out, keys, sizeof(long) * k);
    free(rank); free(seen); free(keys);
}

void or_random_subset(uint64_t seed, long n, int k, long *out) {
    pcg_t r = {seed, 0x385ab5285169b1acULL}; /* kmeans.go:50 */
    random_subset(&r, n, k, out);
}

/* ---- k-means ---------------------------------------------------------------- */
typedef struct { uint32_t idx; float dist; } nb_t;

static float l2(int variant, const float *a, const float *b, int ds) {
    return or_single_dist(OR_L2, variant, a, b, ds);
}

/* kmeans.go:302-332: float64 sums in data order, / size -> float32; empty keeps */
static void update_centers(const float *data, long n, long d, int seg, int ds, int k, const uint32_t *assign,
                           float *centers) {
    double *acc = (double *)calloc((size_t)k * ds, sizeof(double));
    uint32_t *sizes = (uint32_t *)calloc(k, sizeof(uint32_t));
    for (long i = 0; i < n; i++) {
        uint32_t c = assign[i];
        sizes[c]++;
        const float *x = data + (size_t)i * d + (size_t)seg * ds;
        for (int j = 0; j < ds; j++) acc[(size_t)c * ds + j] += (double)x[j];
    }
    for (int c = 0; c < k; c++) {
        if (sizes[c] == 0) continue;
        for (int j = 0; j < ds; j++) centers[(size_t)c * ds + j] = (float)(acc[(size_t)c * ds + j] / (double)sizes[c]);
    }
    free(acc); free(sizes);
}

static int cmp_nb(const void *a, const void *b) {
    const nb_t *x = (const nb_t *)a, *y = (const nb_t *)b;
    if (x->dist < y->dist) return -1;
    if (x->dist > y->dist) return 1;
    return x->idx < y->idx ? -1 : x->idx > y->idx; /* ties: index order (pdqsort's is unspecified) */
}

/* kmeans.go:398-417 */
static void update_center_neighbors(int variant, const float *centers, int k, int ds, nb_t *nb) {
    int *len = (int *)calloc(k, sizeof(int));
    for (int c1 = 0; c1 < k; c1++) {
        for (int c2 = c1 + 1; c2 < k; c2++) {
            float dist = l2(variant, centers + (size_t)c1 * ds, centers + (size_t)c2 * ds, ds);
            float de = (float)sqrt((double)dist);
            nb[(size_t)c1 * (k - 1) + len[c1]++] = (nb_t){(uint32_t)c2, de};
            nb[(size_t)c2 * (k - 1) + len[c2]++] = (nb_t){(uint32_t)c1, de};
        }
    }
    for (int c = 0; c < k; c++) qsort(nb + (size_t)c * (k - 1), k - 1, sizeof(nb_t), cmp_nb);
    free(len);
}

/* kmeans.go:373-383 */
static uint32_t nearest_brute(int variant, const float *x, const float *centers, int k, int ds) {
    float mn = 3.40282346638528859811704183484516925440e+38f;
    uint32_t idx = 0;
    for (int c = 0; c < k; c++) {
        float dd = l2(variant, x, centers + (size_t)c * ds, ds);
        if (dd < mn) { mn = dd; idx = (uint32_t)c; }
    }
    return idx;
}

/* kmeans.go:354-371 */
static uint32_t nearest_pruning(int variant, const float *x, const float *centers, int k, int ds, uint32_t prev,
                                const nb_t *nb) {
    float mn = l2(variant, centers + (size_t)prev * ds, x, ds);
    float cd = (float)sqrt((double)mn);
    uint32_t idx = prev;
    const nb_t *list = nb + (size_t)prev * (k - 1);
    for (int i = 0; i < k - 1; i++) {
        if (list[i].dist >= 2 * cd) break;
        float dd = l2(variant, x, centers + (size_t)list[i].idx * ds, ds);
        if (dd < mn) { mn = dd; idx = list[i].idx; }
    }
    return idx;
}

/* kmeans.go:458-497 Fit with RandomInitialization + GraphPruning (or
 * BruteForce, brute_force != 0: only used to check the pruning) on segment
 * `seg` of the rows.  Returns the iteration count (Metrics.Iterations), or
 * -1 for "not enough data to fit k-means". */
int or_kmeans_fit(const float *data, long n, long d, int seg, int ds, int k, uint64_t seed, int variant,
                  int iteration_threshold, float delta_threshold, int brute_force, float *centers) {
    if (n < k) return -1;
    uint32_t *assign = (uint32_t *)calloc(n, sizeof(uint32_t));
    if (k == 1) { /* computeCentroid */
        update_centers(data, n, d, seg, ds, k, assign, centers);
        free(assign);
        return 0;
    }
    memset(centers, 0, sizeof(float) * (size_t)k * ds);
    pcg_t r = {seed, 0x385ab5285169b1acULL};
    int iterations = 0;
    /* initializeRandom (:279-299) */
    long *sub = (long *)malloc(sizeof(long) * k);
    random_subset(&r, n, k, sub);
    for (int c = 0; c < k; c++) memcpy(centers + (size_t)c * ds, data + (size_t)sub[c] * d + (size_t)seg * ds, sizeof(float) * ds);
    free(sub);
    if (iteration_threshold == 0) { free(assign); return 0; }
    for (long i = 0; i < n; i++) assign[i] = nearest_brute(variant, data + (size_t)i * d + (size_t)seg * ds, centers, k, ds);
    iterations = 1;
    update_centers(data, n, d, seg, ds, k, assign, centers);
    nb_t *nb = (nb_t *)malloc(sizeof(nb_t) * (size_t)k * (k - 1));
    while (iterations < iteration_threshold) {
        update_center_neighbors(variant, centers, k, ds, nb);
        long changes = 0;
        for (long i = 0; i < n; i++) {
            uint32_t prev = assign[i];
            const float *x = data + (size_t)i * d + (size_t)seg * ds;
            uint32_t c = brute_force ? nearest_brute(variant, x, centers, k, ds)
                                     : nearest_pruning(variant, x, centers, k, ds, prev, nb);
            if (c != prev) { changes++; assign[i] = c; }
        }
        iterations++;
        update_centers(data, n, d, seg, ds, k, assign, centers);
        if ((float)changes <= delta_threshold * (float)n) break;
    }
    free(nb); free(assign);
    return iterations;
}

/* ---- encode / LUT / ADC ----------------------------------------------------- */

/* kmeans_encoder.go:67-78 over all segments (product_quantization.go:426-432) */
void or_pq_encode(const float *centers, int m, int k, int ds, int variant, const float *vec, uint8_t *code) {
    for (int s = 0; s < m; s++) {
        float mn = 3.40282346638528859811704183484516925440e+38f;
        int idx = 0;
        for (int c = 0; c < k; c++) {
            float dd = l2(variant, vec + (size_t)s * ds, centers + ((size_t)s * k + c) * ds, ds);
            if (dd < mn) { mn = dd; idx = c; }
        }
        code[s] = (uint8_t)idx;
    }
}

/* Provider.Step: sequential, unfused (l2.go:63-72, dot_product.go:87-94) */
static float step(int metric, const float *a, const float *b, int n) {
    float sum = 0.f;
    for (int i = 0; i < n; i++) {
        if (metric == OR_L2) { float diff = a[i] - b[i]; float sq = diff * diff; sum = sum + sq; }
        else { float p = a[i] * b[i]; sum = sum + p; }
    }
    return sum;
}

static float wrap(int metric, float x) {
    if (metric == OR_L2) return x;
    if (metric == OR_DOT) return -x;
    float w = 1.f - x;
    return w < 0 ? 0.f : w;
}

/* DistanceLookUpTable entries: LUT[s][c] = Step(query_seg_s, centroid_c) */
void or_pq_lut(int metric, const float *centers, int m, int k, int ds, const float *query, float *lut) {
    for (int s = 0; s < m; s++)
        for (int c = 0; c < k; c++)
            lut[(size_t)s * k + c] = step(metric, query + (size_t)s * ds, centers + ((size_t)s * k + c) * ds, ds);
}

/* LookUp (product_quantization.go:85-104): sum in segment order, then Wrap */
float or_pq_adc(int metric, const float *lut, int m, int k, const uint8_t *code) {
    float sum = 0.f;
    for (int s = 0; s < m; s++) sum = sum + lut[(size_t)s * k + code[s]];
    return wrap(metric, sum);
}

/* hnsw.flatSearch (flat_search.go:28-141) with one worker over the present
 * slots in id order, PQ distancer, then (rescore != 0) h.rescore with one worker
 * (search.go:1047-1110) using SingleDist(stored, query). limit = rescore ?
 * max(limit, k) : k.  query must already be normalised for cosine. */
int or_pq_flat_search(int metric, int variant, const float *centers, int m, int ks, int ds, const uint8_t *codes,
                      const float *store, const uint8_t *present, long nslots, const float *query, int k, int limit,
                      int rescore, uint64_t *out_ids, float *out_dists, int *out_n) {
    if (!rescore || limit < k) limit = k;
    float *lut = (float *)malloc(sizeof(float) * (size_t)m * ks);
    or_pq_lut(metric, centers, m, ks, ds, query, lut);
    or_heap loc, res;
    loc.id = (uint64_t *)malloc(sizeof(uint64_t) * (limit + 2)); loc.dist = (float *)malloc(sizeof(float) * (limit + 2)); loc.len = 0;
    res.id = (uint64_t *)malloc(sizeof(uint64_t) * (limit + 2)); res.dist = (float *)malloc(sizeof(float) * (limit + 2)); res.len = 0;
    for (long s = 0; s < nslots; s++) {
        if (!present[s]) continue;
        or_insert_to_heap(&loc, limit, (uint64_t)s, or_pq_adc(metric, lut, m, ks, codes + (size_t)s * m));
    }
    while (loc.len > 0) { /* merge: pop local max-first, addResult into results */
        uint64_t id; float dd;
        or_heap_pop(&loc, &id, &dd);
        or_insert_to_heap(&res, limit, id, dd);
    }
    if (rescore) {
        int n = res.len;
        uint64_t *ids = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
        for (int i = n - 1; i >= 0; i--) { float t; or_heap_pop(&res, &ids[i], &t); }
        for (int i = 0; i < n; i++) { /* addID: Insert, then Pop while Len > k */
            float dd = or_single_dist(metric, variant, store + (size_t)ids[i] * (size_t)m * ds, query, (long)m * ds);
            or_heap_insert(&res, ids[i], dd);
            if (res.len > k) { uint64_t a; float b; or_heap_pop(&res, &a, &b); }
        }
        free(ids);
    }
    *out_n = or_extract_heap(&res, out_ids, out_dists);
    free(lut); free(loc.id); free(loc.dist); free(res.id); free(res.dist);
    return 0;
}
