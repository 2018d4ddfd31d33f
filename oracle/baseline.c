/*
 * baseline.c -- TEST INFRASTRUCTURE / CPU BASELINE ONLY.
 *
 * Multi-threaded CPU flat search timed beside the GPU in bench.py's
 * cpu_baseline leg.  It restates the reference's per-query sequential scan
 * (flat/index.go:578-619 findTopVectors -> :665-674 insertToHeap ->
 * :676-688 extractHeap) with one query per thread, like
 * compressionhelpers.Concurrently (compressionhelpers/utils.go:25-42).
 *
 * The per-pair distance is either the oracle's scalar restatement or -- when
 * bl_set_ref_kernels() is given the symbols of oracle/_ref/libref.so -- the
 * reference's own AVX2/AVX-512 C kernels compiled from /root/reference
 * (distancer/c/{l2,dot}_avx{256,512}_amd64.c).  The store is one contiguous array (no LSM cursor,
 * no byte decode), so this is an upper bound on Weaviate's CPU QPS.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef void (*ref_kernel)(float *a, float *b, float *res, long *len);
static ref_kernel g_ref[4]; /* l2_256, l2_512, dot_256, dot_512 */

void bl_set_ref_kernels(void *l2_256, void *l2_512, void *dot_256, void *dot_512) {
    g_ref[0] = (ref_kernel)l2_256; g_ref[1] = (ref_kernel)l2_512;
    g_ref[2] = (ref_kernel)dot_256; g_ref[3] = (ref_kernel)dot_512;
}

typedef struct {
    int metric, variant, use_ref, k;
    const float *store; long n, d;
    const float *queries; long nq;
    uint64_t *out_ids; float *out_dists; int *out_n;
    int tid, nthreads;
} job_t;

static float pair_dist(const job_t *j, const float *q, const float *x) {
    if (!j->use_ref) return or_single_dist(j->metric, j->variant, q, x, j->d);
    long len = j->d;
    float r = 0.f;
    int is512 = j->variant == OR_AVX512;
    if (j->metric == OR_L2) { g_ref[is512 ? 1 : 0]((float *)q, (float *)x, &r, &len); return r; }
    g_ref[is512 ? 3 : 2]((float *)q, (float *)x, &r, &len);
    if (j->metric == OR_DOT) return -r;
    float p = 1.f - r; /* cosine_dist.go:50-55 */
    return p < 0 ? 0.f : p;
}

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    or_heap h;
    h.id = (uint64_t *)malloc(sizeof(uint64_t) * (j->k + 1));
    h.dist = (float *)malloc(sizeof(float) * (j->k + 1));
    for (long qi = j->tid; qi < j->nq; qi += j->nthreads) {
        const float *q = j->queries + (size_t)qi * j->d;
        h.len = 0;
        for (long s = 0; s < j->n; s++)
            or_insert_to_heap(&h, j->k, (uint64_t)s, pair_dist(j, q, j->store + (size_t)s * j->d));
        j->out_n[qi] = or_extract_heap(&h, j->out_ids + (size_t)qi * j->k, j->out_dists + (size_t)qi * j->k);
    }
    free(h.id); free(h.dist);
    return NULL;
}

/* queries must already be normalized for cosine (flat/index.go:690-697). */
int bl_flat_search_batch(int metric, int variant, int use_ref, const float *store, long n, long d,
                         const float *queries, long nq, int k, int nthreads,
                         uint64_t *out_ids, float *out_dists, int *out_n) {
    if (use_ref && !g_ref[0]) return -1;
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    job_t *jobs = (job_t *)malloc(sizeof(job_t) * nthreads);
    for (int t = 0; t < nthreads; t++) {
        job_t j = {metric, variant, use_ref, k, store, n, d, queries, nq, out_ids, out_dists, out_n, t, nthreads};
        jobs[t] = j;
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th); free(jobs);
    return 0;
}

/* ---- BQ: searchByVectorQuantized (flat/index.go:460-532), one query per thread ---- */
typedef void (*ref_hbw)(uint64_t *a, uint64_t *b, uint64_t *res, long *len, uint8_t *lookup, uint64_t *consts);
static ref_hbw g_ref_hbw;
static uint8_t g_lookup[32] = {0, 1, 1, 2, 1, 2, 2, 3, 1, 2, 2, 3, 2, 3, 3, 4, 0, 1, 1, 2, 1, 2, 2, 3, 1, 2, 2, 3, 2, 3, 3, 4};
static uint64_t g_consts[5] = {0x5555555555555555ull, 0x3333333333333333ull, 0x0F0F0F0F0F0F0F0Full,
                               0x0101010101010101ull, 0x0F0F0F0F0F0F0F0Full};

/* hamming_bitwise_256 from oracle/_ref (asm/hamming_amd64.go:69-80 passes the
 * lookup table and popcount constants) */
void bl_set_ref_hamming(void *hamming_bitwise_256) { g_ref_hbw = (ref_hbw)hamming_bitwise_256; }

typedef struct {
    job_t base;
    const uint64_t *codes; long words; int rescore;
} bq_job_t;

static void *bq_worker(void *arg) {
    bq_job_t *bj = (bq_job_t *)arg;
    job_t *j = &bj->base;
    int R = bj->rescore;
    or_heap h;
    h.id = (uint64_t *)malloc(sizeof(uint64_t) * (R + 1));
    h.dist = (float *)malloc(sizeof(float) * (R + 1));
    uint64_t *cand = (uint64_t *)malloc(sizeof(uint64_t) * (R + 1));
    float *cd = (float *)malloc(sizeof(float) * (R + 1));
    uint64_t *qc = (uint64_t *)malloc(sizeof(uint64_t) * (bj->words + 1));
    for (long qi = j->tid; qi < j->nq; qi += j->nthreads) {
        const float *q = j->queries + (size_t)qi * j->d;
        or_bq_encode(q, j->d, qc);
        h.len = 0;
        for (long s = 0; s < j->n; s++) {
            float dist;
            const uint64_t *x = bj->codes + (size_t)s * bj->words;
            if (j->use_ref && g_ref_hbw) {
                uint64_t res = 0; long len = bj->words;
                g_ref_hbw((uint64_t *)x, qc, &res, &len, g_lookup, g_consts);
                dist = (float)res;
            } else {
                dist = or_hamming_bitwise(x, qc, bj->words);
            }
            or_insert_to_heap(&h, R, (uint64_t)s, dist);
        }
        int n = h.len;
        for (int i = 0; i < n; i++) { float t; or_heap_pop(&h, &cand[i], &t); }
        for (int i = 0; i < n; i++) cd[i] = pair_dist(j, q, j->store + (size_t)cand[i] * j->d);
        for (int i = 0; i < n; i++) or_insert_to_heap(&h, j->k, cand[i], cd[i]);
        j->out_n[qi] = or_extract_heap(&h, j->out_ids + (size_t)qi * j->k, j->out_dists + (size_t)qi * j->k);
    }
    free(h.id); free(h.dist); free(cand); free(cd); free(qc);
    return NULL;
}

/* store: normalised fp32 rows [n][d]; codes: [n][words] of the stored rows;
 * queries normalised already for cosine. */
int bl_flat_search_bq_batch(int metric, int variant, int use_ref, const float *store, const uint64_t *codes,
                            long n, long d, const float *queries, long nq, int k, int rescore_limit, int nthreads,
                            uint64_t *out_ids, float *out_dists, int *out_n) {
    if (use_ref && !g_ref[0]) return -1;
    if (nthreads < 1) nthreads = 1;
    int R = rescore_limit > k ? rescore_limit : k;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    bq_job_t *jobs = (bq_job_t *)malloc(sizeof(bq_job_t) * nthreads);
    for (int t = 0; t < nthreads; t++) {
        job_t j = {metric, variant, use_ref, k, store, n, d, queries, nq, out_ids, out_dists, out_n, t, nthreads};
        jobs[t].base = j;
        jobs[t].codes = codes;
        jobs[t].words = (d + 63) / 64;
        jobs[t].rescore = R;
        pthread_create(&th[t], NULL, bq_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th); free(jobs);
    return 0;
}

/* ---- PQ: flatSearch over PQ codes (hnsw/flat_search.go, one worker), one query per thread ---- */
typedef struct {
    int metric, k, m, ks, ds;
    const float *centers; const uint8_t *codes; long n;
    const float *queries; long nq;
    uint64_t *out_ids; float *out_dists; int *out_n;
    int tid, nthreads;
} pq_job_t;

static void *pq_worker(void *arg) {
    pq_job_t *j = (pq_job_t *)arg;
    float *lut = (float *)malloc(sizeof(float) * (size_t)j->m * j->ks);
    or_heap h, r;
    h.id = (uint64_t *)malloc(sizeof(uint64_t) * (j->k + 1)); h.dist = (float *)malloc(sizeof(float) * (j->k + 1));
    r.id = (uint64_t *)malloc(sizeof(uint64_t) * (j->k + 1)); r.dist = (float *)malloc(sizeof(float) * (j->k + 1));
    for (long qi = j->tid; qi < j->nq; qi += j->nthreads) {
        const float *q = j->queries + (size_t)qi * j->m * j->ds;
        or_pq_lut(j->metric, j->centers, j->m, j->ks, j->ds, q, lut);
        h.len = 0; r.len = 0;
        for (long s = 0; s < j->n; s++)
            or_insert_to_heap(&h, j->k, (uint64_t)s, or_pq_adc(j->metric, lut, j->m, j->ks, j->codes + (size_t)s * j->m));
        while (h.len > 0) { uint64_t id; float dd; or_heap_pop(&h, &id, &dd); or_insert_to_heap(&r, j->k, id, dd); }
        j->out_n[qi] = or_extract_heap(&r, j->out_ids + (size_t)qi * j->k, j->out_dists + (size_t)qi * j->k);
    }
    free(lut); free(h.id); free(h.dist); free(r.id); free(r.dist);
    return NULL;
}

int bl_pq_search_batch(int metric, const float *centers, int m, int ks, int ds, const uint8_t *codes, long n,
                       const float *queries, long nq, int k, int nthreads, uint64_t *out_ids, float *out_dists,
                       int *out_n) {
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    pq_job_t *jobs = (pq_job_t *)malloc(sizeof(pq_job_t) * nthreads);
    for (int t = 0; t < nthreads; t++) {
        pq_job_t jj = {metric, k, m, ks, ds, centers, codes, n, queries, nq, out_ids, out_dists, out_n, t, nthreads};
        jobs[t] = jj;
        pthread_create(&th[t], NULL, pq_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th); free(jobs);
    return 0;
}
