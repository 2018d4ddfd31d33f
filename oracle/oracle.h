/* oracle.h -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's
 * flat-index hot path (see oracle.c).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this. */
#ifndef WV_ORACLE_H
#define WV_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_L2 = 0, OR_DOT = 1, OR_COSINE = 2, OR_HAMMING = 3 };
enum { OR_AVX256 = 1, OR_AVX512 = 2 };
enum { OR_ERR_VECTOR_LENGTH = -1, OR_ERR_HAMMING_LENGTH = -2 };

typedef struct {
    uint64_t *id;
    float *dist;
    int len;
} or_heap;

float or_l2_256(const float *a, const float *b, long n);
float or_l2_512(const float *a, const float *b, long n);
float or_dot_256(const float *a, const float *b, long n);
float or_dot_512(const float *a, const float *b, long n);
float or_hamming_f32(const float *a, const float *b, long n);
float or_hamming_bitwise(const uint64_t *a, const uint64_t *b, long n);
void or_normalize(const float *v, float *out, long n);
float or_single_dist(int metric, int variant, const float *a, const float *b, long n);

void or_heap_insert(or_heap *h, uint64_t id, float dist);
void or_heap_pop(or_heap *h, uint64_t *id, float *dist);
void or_insert_to_heap(or_heap *h, int limit, uint64_t id, float dist);
int or_extract_heap(or_heap *h, uint64_t *ids, float *dists);

int or_find_top_vectors(or_heap *heap, int limit, int metric, int variant, const float *store,
                        const uint8_t *present, long nslots, long d, const float *query, long qd,
                        const uint8_t *allow, long slot_begin, long slot_end);
int or_flat_search(int metric, int variant, const float *store, const uint8_t *present, long nslots,
                   long d, const float *query, long qd, int k, const uint8_t *allow, int allow_empty,
                   uint64_t *out_ids, float *out_dists, int *out_n);

void or_bq_encode(const float *vec, long d, uint64_t *code);
int or_flat_search_bq(int metric, int variant, const float *store, const uint8_t *present,
                      const uint8_t *fp32_present, const uint64_t *codes, long nslots, long d,
                      const float *query, long qd, int k, int rescore_limit, const uint8_t *allow,
                      int allow_empty, uint64_t *out_ids, float *out_dists, int *out_n);

int or_filter_by_distance(const uint64_t *ids, const float *dists, int n, float target,
                          uint64_t *out_ids, float *out_dists);

/* pq.c: Go math/rand/v2 PCG-DXSM restatement shared with rq.c */
typedef struct { uint64_t hi, lo; } pcg_t;
uint64_t pcg_u64(pcg_t *p);
uint64_t pcg_u64n(pcg_t *p, uint64_t n);
double pcg_f64(pcg_t *p);

/* pq.c: product quantizer (see its header) */
void or_pcg_stream(uint64_t s1, uint64_t s2, int cnt, uint64_t *out);
void or_random_subset(uint64_t seed, long n, int k, long *out);
int or_kmeans_fit(const float *data, long n, long d, int seg, int ds, int k, uint64_t seed, int variant,
                  int iteration_threshold, float delta_threshold, int brute_force, float *centers);
void or_pq_encode(const float *centers, int m, int k, int ds, int variant, const float *vec, uint8_t *code);
void or_pq_lut(int metric, const float *centers, int m, int k, int ds, const float *query, float *lut);
float or_pq_adc(int metric, const float *lut, int m, int k, const uint8_t *code);
int or_pq_flat_search(int metric, int variant, const float *centers, int m, int ks, int ds, const uint8_t *codes,
                      const float *store, const uint8_t *present, long nslots, const float *query, int k, int limit,
                      int rescore, uint64_t *out_ids, float *out_dists, int *out_n);

/* sq.c: scalar quantizer + generic hnsw.flatSearch (see its header) */
void or_sq_fit(const float *data, long n, long d, float *out_ab);
void or_sq_encode(float a, float b, const float *vec, long d, uint8_t *code);
float or_sq_distance(int metric, float a, float b, long d, const uint8_t *x, const uint8_t *y);
int or_hnsw_flat_search(const float *cdist, const float *edist, const uint8_t *present, long nslots, int k, int limit,
                        int rescore, int trim, uint64_t *out_ids, float *out_dists, int *out_n);

/* rq.c: rotational quantization rq-8 / rq-1 (see its header) */
typedef struct or_rq or_rq;
or_rq *or_rq_new(int bits, int metric, int dims, uint64_t seed);
void or_rq_free(or_rq *r);
int or_rq_out_dim(const or_rq *r);
void or_rq_tables(const or_rq *r, uint16_t *sI, uint16_t *sJ, float *signs, float *rounding);
void or_fwht64(float *x);
void or_fwht256(float *x);
void or_rq_rotate(const or_rq *r, const float *x, long n, float *rx);
void or_rq8_encode(const or_rq *r, int variant, const float *x, long n, uint8_t *code);
float or_rq8_distance(const or_rq *r, const uint8_t *cx, const uint8_t *cy);
void or_brq_encode(const or_rq *r, const float *x, long n, uint64_t *code);
void or_brq_encode_query(const or_rq *r, const float *x, long n, float *step_out, float *sqn_out, int *dim_out,
                         uint64_t *planes);
float or_brq_distance(const or_rq *r, float qstep, float qsqn, int qdim, const uint64_t *planes,
                      const uint64_t *cx);
int or_flat_search_rq(const or_rq *r, int variant, const float *store, const uint8_t *present, const void *codes,
                      long nslots, long d, const float *query, long qd, int k, int rescore_limit,
                      const uint8_t *allow, int allow_empty, uint64_t *out_ids, float *out_dists, int *out_n);
void or_rq_query_distances(const or_rq *r, int variant, const void *codes, long nslots, const float *query, long qd,
                           float *out);

/* scale.c: oracles at full BASELINE sizes over the regenerated corpus */
int or_gen_dists(int kind, uint64_t seed, long n, long d, int metric, int variant, const float *queries, long nq,
                 int nthreads, float *out);
int or_heap_scan(const float *dists, long n, int k, uint64_t *out_ids, float *out_dists);
int or_bq_search_gen(int kind, uint64_t seed, long n, long d, int metric, int variant, const float *queries, long nq,
                     int k, int rescore_limit, int nthreads, uint64_t *out_ids, float *out_d, int *out_n);
int or_rq_search_gen(int bits, int kind, uint64_t seed, long n, long d, int metric, int variant, const float *queries,
                     long nq, int k, int rescore_limit, int nthreads, uint64_t *out_ids, float *out_d, int *out_n);

uint64_t or_gen_bits(uint64_t seed, uint64_t row, uint64_t col);
float or_gen_value(int kind, uint64_t seed, uint64_t row, uint64_t col);
void or_gen_matrix(int kind, uint64_t seed, uint64_t row0, long rows, long d, float *out);
void or_normalize_rows(float *v, long n, long d);

#ifdef __cplusplus
}
#endif
#endif
