/*
 * scale.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Oracles at the BASELINE configurations' full sizes (10M x 768, a 6.25M x
 * 1536 BQ shard) without a host copy of the corpus: the synthetic rows are
 * regenerated from the counter-based generator (or_gen_value, identical to
 * the GPU's k_gen) and prepared exactly as flat.Add prepares them
 * (flat/index.go:371-378: cosine rows through distancer.Normalize).  The
 * distance kernels, the heap and the BQ search are the restatements of
 * oracle.c (same functions), run over row ranges on worker threads.
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* one generated + prepared row (flat.Add: Normalize for cosine, flat/index.go:376-378) */
static void gen_row(int kind, uint64_t seed, long r, long d, int metric, float *buf, float *out) {
    for (long c = 0; c < d; c++) buf[c] = or_gen_value(kind, seed, (uint64_t)r, (uint64_t)c);
    if (metric == OR_COSINE) or_normalize(buf, out, d);
    else memcpy(out, buf, sizeof(float) * d);
}

typedef struct {
    int kind, metric, variant;
    uint64_t seed;
    long r0, r1, n, d, nq;
    const float *queries;
    float *out;
} dist_job;

static void *dist_worker(void *p) {
    dist_job *j = (dist_job *)p;
    float *buf = (float *)malloc(sizeof(float) * j->d);
    float *row = (float *)malloc(sizeof(float) * j->d);
    for (long r = j->r0; r < j->r1; r++) {
        gen_row(j->kind, j->seed, r, j->d, j->metric, buf, row);
        for (long q = 0; q < j->nq; q++)
            j->out[q * j->n + r] = or_single_dist(j->metric, j->variant, j->queries + q * j->d, row, j->d);
    }
    free(buf);
    free(row);
    return NULL;
}

/* Provider.SingleDist(query_q, row_r) for rows [0, n) of the generated corpus;
 * queries already prepared (normalised for cosine, flat/index.go:690-697).
 * out[q * n + r]. */
int or_gen_dists(int kind, uint64_t seed, long n, long d, int metric, int variant, const float *queries, long nq,
                 int nthreads, float *out) {
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    dist_job *jobs = (dist_job *)malloc(sizeof(dist_job) * nthreads);
    const long per = (n + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        dist_job *j = &jobs[t];
        j->kind = kind; j->metric = metric; j->variant = variant; j->seed = seed;
        j->r0 = t * per; j->r1 = j->r0 + per < n ? j->r0 + per : n;
        j->n = n; j->d = d; j->nq = nq; j->queries = queries; j->out = out;
        pthread_create(&th[t], NULL, dist_worker, j);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    return 0;
}

/* flat/index.go:578-688 over precomputed distances of rows [0, n) (every row
 * present, no allow list): insertToHeap in id order, then extractHeap. */
int or_heap_scan(const float *dists, long n, int k, uint64_t *out_ids, float *out_dists) {
    or_heap h;
    h.len = 0;
    h.id = (uint64_t *)malloc(sizeof(uint64_t) * (k + 1));
    h.dist = (float *)malloc(sizeof(float) * (k + 1));
    for (long r = 0; r < n; r++) or_insert_to_heap(&h, k, (uint64_t)r, dists[r]);
    int m = or_extract_heap(&h, out_ids, out_dists);
    free(h.id);
    free(h.dist);
    return m;
}

typedef struct {
    int kind, metric;
    uint64_t seed;
    long r0, r1, d, words;
    uint64_t *codes;
} code_job;

static void *code_worker(void *p) {
    code_job *j = (code_job *)p;
    float *buf = (float *)malloc(sizeof(float) * j->d);
    float *row = (float *)malloc(sizeof(float) * j->d);
    for (long r = j->r0; r < j->r1; r++) {
        gen_row(j->kind, j->seed, r, j->d, j->metric, buf, row);
        or_bq_encode(row, j->d, j->codes + r * j->words);
    }
    free(buf);
    free(row);
    return NULL;
}

typedef struct {
    int kind, metric, variant, k, rescore_limit;
    uint64_t seed;
    long n, d, words, q0, q1;
    const uint64_t *codes;
    const float *queries;
    uint64_t *out_ids;
    float *out_d;
    int *out_n;
} bq_job;

/* flat/index.go:460-532 searchByVectorQuantized (as or_flat_search_bq, every
 * row present and holding its fp32 vector), rows regenerated for rescoring */
static void *bq_worker(void *p) {
    bq_job *j = (bq_job *)p;
    const int R = j->rescore_limit > j->k ? j->rescore_limit : j->k;
    float *q = (float *)malloc(sizeof(float) * j->d);
    float *buf = (float *)malloc(sizeof(float) * j->d);
    float *row = (float *)malloc(sizeof(float) * j->d);
    uint64_t *qcode = (uint64_t *)calloc(j->words, sizeof(uint64_t));
    or_heap h;
    h.id = (uint64_t *)malloc(sizeof(uint64_t) * (R + 1));
    h.dist = (float *)malloc(sizeof(float) * (R + 1));
    uint64_t *ids = (uint64_t *)malloc(sizeof(uint64_t) * (R + 1));
    float *dd = (float *)malloc(sizeof(float) * (R + 1));
    for (long qi = j->q0; qi < j->q1; qi++) {
        const float *query = j->queries + qi * j->d;
        if (j->metric == OR_COSINE) or_normalize(query, q, j->d);
        else memcpy(q, query, sizeof(float) * j->d);
        or_bq_encode(q, j->d, qcode);
        h.len = 0;
        for (long s = 0; s < j->n; s++)
            or_insert_to_heap(&h, R, (uint64_t)s, or_hamming_bitwise(j->codes + s * j->words, qcode, j->words));
        const int n = h.len;
        for (int i = 0; i < n; i++) { float t; or_heap_pop(&h, &ids[i], &t); }
        for (int i = 0; i < n; i++) {
            gen_row(j->kind, j->seed, (long)ids[i], j->d, j->metric, buf, row);
            dd[i] = or_single_dist(j->metric, j->variant, q, row, j->d);
        }
        for (int i = 0; i < n; i++) or_insert_to_heap(&h, j->k, ids[i], dd[i]);
        j->out_n[qi] = or_extract_heap(&h, j->out_ids + qi * j->k, j->out_d + qi * j->k);
    }
    free(q); free(buf); free(row); free(qcode); free(h.id); free(h.dist); free(ids); free(dd);
    return NULL;
}

/* BQ flat search of nq raw queries over the generated corpus rows [0, n):
 * codes built on nthreads workers, then the queries split over the workers. */
int or_bq_search_gen(int kind, uint64_t seed, long n, long d, int metric, int variant, const float *queries, long nq,
                     int k, int rescore_limit, int nthreads, uint64_t *out_ids, float *out_d, int *out_n) {
    if (nthreads < 1) nthreads = 1;
    const long words = (d + 63) / 64;
    uint64_t *codes = (uint64_t *)malloc(sizeof(uint64_t) * words * (n > 0 ? n : 1));
    if (!codes) return -1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    code_job *cj = (code_job *)malloc(sizeof(code_job) * nthreads);
    const long per = (n + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        code_job *j = &cj[t];
        j->kind = kind; j->metric = metric; j->seed = seed; j->d = d; j->words = words; j->codes = codes;
        j->r0 = t * per; j->r1 = j->r0 + per < n ? j->r0 + per : n;
        pthread_create(&th[t], NULL, code_worker, j);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    bq_job *bj = (bq_job *)malloc(sizeof(bq_job) * nthreads);
    const long qper = (nq + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        bq_job *j = &bj[t];
        j->kind = kind; j->metric = metric; j->variant = variant; j->k = k; j->rescore_limit = rescore_limit;
        j->seed = seed; j->n = n; j->d = d; j->words = words; j->codes = codes; j->queries = queries;
        j->out_ids = out_ids; j->out_d = out_d; j->out_n = out_n;
        j->q0 = t * qper; j->q1 = j->q0 + qper < nq ? j->q0 + qper : nq;
        if (j->q0 > nq) j->q0 = nq;
        pthread_create(&th[t], NULL, bq_worker, j);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(bj); free(cj); free(th); free(codes);
    return 0;
}

/* ---- rq-8 / rq-1 at full size (bench self-check) --------------------------- */
typedef struct {
    const or_rq *rq;
    int kind, metric, variant, bits;
    uint64_t seed;
    long r0, r1, d;
    size_t clen;  /* bytes per code: rq-8 16 + D, rq-1 8 (1 + D / 64) */
    uint8_t *codes;
} rq_code_job;

static void *rq_code_worker(void *p) {
    rq_code_job *j = (rq_code_job *)p;
    float *buf = (float *)malloc(sizeof(float) * j->d);
    float *row = (float *)malloc(sizeof(float) * j->d);
    for (long r = j->r0; r < j->r1; r++) {
        gen_row(j->kind, j->seed, r, j->d, j->metric, buf, row);
        if (j->bits == 8) or_rq8_encode(j->rq, j->variant, row, j->d, j->codes + (size_t)r * j->clen);
        else or_brq_encode(j->rq, row, j->d, (uint64_t *)(j->codes + (size_t)r * j->clen));
    }
    free(buf);
    free(row);
    return NULL;
}

typedef struct {
    const or_rq *rq;
    int kind, metric, variant, bits, k, rescore_limit;
    uint64_t seed;
    long n, d, q0, q1;
    size_t clen;
    const uint8_t *codes;
    const float *queries;
    uint64_t *out_ids;
    float *out_d;
    int *out_n;
} rq_job;

/* or_flat_search_rq (rq.c) with every row present and the rescoring rows
 * regenerated instead of read from a store */
static void *rq_worker(void *p) {
    rq_job *j = (rq_job *)p;
    const int R = j->rescore_limit > j->k ? j->rescore_limit : j->k;
    const int D = or_rq_out_dim(j->rq), W = D / 64;
    float *q = (float *)malloc(sizeof(float) * j->d);
    float *buf = (float *)malloc(sizeof(float) * j->d);
    float *row = (float *)malloc(sizeof(float) * j->d);
    uint8_t *qc8 = (uint8_t *)malloc((size_t)D + 16);
    uint64_t *planes = (uint64_t *)malloc(sizeof(uint64_t) * 5 * (W > 0 ? W : 1));
    or_heap h;
    h.id = (uint64_t *)malloc(sizeof(uint64_t) * (R + 1));
    h.dist = (float *)malloc(sizeof(float) * (R + 1));
    uint64_t *ids = (uint64_t *)malloc(sizeof(uint64_t) * (R + 1));
    float *dd = (float *)malloc(sizeof(float) * (R + 1));
    for (long qi = j->q0; qi < j->q1; qi++) {
        const float *query = j->queries + qi * j->d;
        if (j->metric == OR_COSINE) or_normalize(query, q, j->d);
        else memcpy(q, query, sizeof(float) * j->d);
        float qstep = 0, qsqn = 0;
        int qdim = 0;
        if (j->bits == 8) or_rq8_encode(j->rq, j->variant, q, j->d, qc8);
        else or_brq_encode_query(j->rq, q, j->d, &qstep, &qsqn, &qdim, planes);
        h.len = 0;
        for (long s = 0; s < j->n; s++) {
            const uint8_t *c = j->codes + (size_t)s * j->clen;
            const float dist = j->bits == 8 ? or_rq8_distance(j->rq, c, qc8)
                                            : or_brq_distance(j->rq, qstep, qsqn, qdim, planes, (const uint64_t *)c);
            or_insert_to_heap(&h, R, (uint64_t)s, dist);
        }
        const int n = h.len;
        for (int i = 0; i < n; i++) { float t; or_heap_pop(&h, &ids[i], &t); }
        for (int i = 0; i < n; i++) {
            gen_row(j->kind, j->seed, (long)ids[i], j->d, j->metric, buf, row);
            dd[i] = or_single_dist(j->metric, j->variant, q, row, j->d);
        }
        for (int i = 0; i < n; i++) or_insert_to_heap(&h, j->k, ids[i], dd[i]);
        j->out_n[qi] = or_extract_heap(&h, j->out_ids + qi * j->k, j->out_d + qi * j->k);
    }
    free(q); free(buf); free(row); free(qc8); free(planes); free(h.id); free(h.dist); free(ids); free(dd);
    return NULL;
}

/* flat rq-8 / rq-1 search (flat/index.go:460-532) of nq raw queries over the
 * generated corpus rows [0, n): codes built on nthreads workers, then the
 * queries split over the workers.  -1 when the code array cannot be allocated. */
int or_rq_search_gen(int bits, int kind, uint64_t seed, long n, long d, int metric, int variant, const float *queries,
                     long nq, int k, int rescore_limit, int nthreads, uint64_t *out_ids, float *out_d, int *out_n) {
    if (nthreads < 1) nthreads = 1;
    or_rq *rq = or_rq_new(bits, metric, (int)d, 0x535ab5105169b1dfULL);
    if (!rq) return -1;
    const int D = or_rq_out_dim(rq);
    const size_t clen = bits == 8 ? (size_t)D + 16 : sizeof(uint64_t) * (size_t)(1 + D / 64);
    uint8_t *codes = (uint8_t *)malloc(clen * (size_t)(n > 0 ? n : 1));
    if (!codes) { or_rq_free(rq); return -1; }
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    rq_code_job *cj = (rq_code_job *)malloc(sizeof(rq_code_job) * nthreads);
    const long per = (n + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        rq_code_job *j = &cj[t];
        j->rq = rq; j->kind = kind; j->metric = metric; j->variant = variant; j->bits = bits; j->seed = seed;
        j->d = d; j->clen = clen; j->codes = codes;
        j->r0 = t * per; j->r1 = j->r0 + per < n ? j->r0 + per : n;
        if (j->r0 > n) j->r0 = n;
        pthread_create(&th[t], NULL, rq_code_worker, j);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    rq_job *qj = (rq_job *)malloc(sizeof(rq_job) * nthreads);
    const long qper = (nq + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        rq_job *j = &qj[t];
        j->rq = rq; j->kind = kind; j->metric = metric; j->variant = variant; j->bits = bits; j->k = k;
        j->rescore_limit = rescore_limit; j->seed = seed; j->n = n; j->d = d; j->clen = clen; j->codes = codes;
        j->queries = queries; j->out_ids = out_ids; j->out_d = out_d; j->out_n = out_n;
        j->q0 = t * qper; j->q1 = j->q0 + qper < nq ? j->q0 + qper : nq;
        if (j->q0 > nq) j->q0 = nq;
        pthread_create(&th[t], NULL, rq_worker, j);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(qj); free(cj); free(th); free(codes);
    or_rq_free(rq);
    return 0;
}
