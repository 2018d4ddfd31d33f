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
