/* sq.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).  Scalar restatement of
 *   - compressionhelpers.ScalarQuantizer (scalar_quantization.go):
 *     NewScalarQuantizer (:73-97), codeFor (:114-122), Encode (:124-137),
 *     DistanceBetweenCompressedVectors (:45-57), norm (:207-209), with
 *     l2SquaredByteImpl / dotByteImpl as the exact integer sums they compute;
 *   - hnsw.flatSearch with one worker (hnsw/flat_search.go:28-141, addResult
 *     :214-224) + h.rescore with one worker (hnsw/search.go:1047-1110) over
 *     caller-supplied compressor and exact distances of every slot.
 * Float32 arithmetic is unfused (built with -ffp-contract=off), as Go on amd64
 * evaluates these expressions. */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

void or_sq_fit(const float *data, long n, long d, float *out_ab) {
    float a = 0.f, b = n > 0 && d > 0 ? data[0] : 0.f;
    for (long i = 0; i < n; i++)
        for (long j = 0; j < d; j++) {
            const float x = data[i * d + j];
            if (x < b) {
                a += b - x;
                b = x;
            } else if (x - b > a) {
                a = x - b;
            }
        }
    out_ab[0] = a;
    out_ab[1] = b;
}

static uint8_t code_for(float x, float a, float b) {
    if (x < b) return 0;
    if (x - b > a) return 255;
    float t = x - b;
    t = t * 255.0f;
    t = t / a;
    if (t != t) return 0;
    return (uint8_t)((int64_t)floor((double)t) & 255);
}

/* code: d bytes + big-endian uint32 sum + big-endian uint32 sum of squares */
void or_sq_encode(float a, float b, const float *vec, long d, uint8_t *code) {
    uint32_t sum = 0, sum2 = 0;
    for (long i = 0; i < d; i++) {
        code[i] = code_for(vec[i], a, b);
        sum += code[i];
        sum2 += (uint32_t)code[i] * code[i];
    }
    for (int i = 0; i < 4; i++) code[d + i] = (uint8_t)(sum >> (24 - 8 * i));
    for (int i = 0; i < 4; i++) code[d + 4 + i] = (uint8_t)(sum2 >> (24 - 8 * i));
}

static uint32_t be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* metric OR_L2 / OR_DOT / OR_COSINE; returns NAN for others (reference error) */
float or_sq_distance(int metric, float a, float b, long d, const uint8_t *x, const uint8_t *y) {
    const float a2 = (a * a) / 65025.0f;
    const float ab = (a * b) / 255.0f;
    const float ib2 = (b * b) * (float)d;
    if (metric == OR_L2) {
        uint32_t s = 0;
        for (long i = 0; i < d; i++) {
            const int32_t t = (int32_t)x[i] - (int32_t)y[i];
            s += (uint32_t)(t * t);
        }
        return a2 * (float)s;
    }
    if (metric != OR_DOT && metric != OR_COSINE) return NAN;
    uint32_t dt = 0;
    for (long i = 0; i < d; i++) dt += (uint32_t)x[i] * y[i];
    const uint32_t nn = be32(x + d) + be32(y + d);
    float t = a2 * (float)dt;
    const float u = ab * (float)nn;
    t = t + u;
    t = t + ib2;
    return metric == OR_DOT ? -t : 1.0f - t;
}

/* present[s]: the slot is searched (allow list & node exists); cdist[s] the
 * compressor distance, edist[s] the rescoring distance.  limit / trim /
 * rescore as the caller computed them (searchTimeEF, RescoreLimit). */
int or_hnsw_flat_search(const float *cdist, const float *edist, const uint8_t *present, long nslots, int k, int limit,
                        int rescore, int trim, uint64_t *out_ids, float *out_dists, int *out_n) {
    if (limit < k) limit = k;
    or_heap loc, res;
    loc.id = (uint64_t *)malloc(sizeof(uint64_t) * (limit + 2)); loc.dist = (float *)malloc(sizeof(float) * (limit + 2)); loc.len = 0;
    res.id = (uint64_t *)malloc(sizeof(uint64_t) * (limit + 2)); res.dist = (float *)malloc(sizeof(float) * (limit + 2)); res.len = 0;
    for (long s = 0; s < nslots; s++)
        if (present[s]) or_insert_to_heap(&loc, limit, (uint64_t)s, cdist[s]);
    while (loc.len > 0) { /* merge: pop local max-first, addResult into results */
        uint64_t id; float dd;
        or_heap_pop(&loc, &id, &dd);
        or_insert_to_heap(&res, limit, id, dd);
    }
    if (rescore) {
        if (trim > 0)
            while (res.len > trim) { uint64_t a; float b; or_heap_pop(&res, &a, &b); }
        int n = res.len;
        uint64_t *ids = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
        for (int i = n - 1; i >= 0; i--) { float t; or_heap_pop(&res, &ids[i], &t); }
        for (int i = 0; i < n; i++) { /* addID: Insert, then Pop while Len > k */
            or_heap_insert(&res, ids[i], edist[ids[i]]);
            if (res.len > k) { uint64_t a; float b; or_heap_pop(&res, &a, &b); }
        }
        free(ids);
    }
    /* results popped max-first into the tail (flat_search.go:130-137) */
    const int m = res.len;
    for (int i = m - 1; i >= 0; i--) {
        uint64_t a; float b;
        or_heap_pop(&res, &a, &b);
        if (i < k) { out_ids[i] = a; out_dists[i] = b; }
    }
    *out_n = m < k ? m : k;
    free(loc.id); free(loc.dist); free(res.id); free(res.dist);
    return 0;
}
