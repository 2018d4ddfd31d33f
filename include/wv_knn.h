/*
 * wv_knn.h -- C ABI of the MI355X (gfx950) flat-index engine.
 *
 * Drop-in boundary for Weaviate's flat vector index and distancer hot path
 * (SURVEY.md §8b).  Every entry point names the reference interface it
 * replaces (paths relative to the reference repo root).  A Go shim would bind
 * these through cgo; the Python mirror in weaviate_amd/ binds
 * them through ctypes.
 *
 * Conventions:
 *  - plain pointers + sizes only; host pointers are borrowed for the call and
 *    copied (cgo forbids retaining Go pointers);  *_device entry points take
 *    device pointers on the index's GPU;
 *  - returns WV_OK (0) or a negative WV_ERR_*; wv_last_error() gives the
 *    reference's error text for the calling thread;
 *  - every entry point is thread-safe (calls on one index are serialised).
 */
#ifndef WV_KNN_H
#define WV_KNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define WV_OK 0
#define WV_ERR_INVALID (-1)        /* bad argument                                  */
#define WV_ERR_VECTOR_LENGTH (-2)  /* distancer.ErrVectorLength (distancer/errors.go:16) */
#define WV_ERR_INSERT (-3)         /* flat ValidateBeforeInsert / AddBatch errors   */
#define WV_ERR_HIP (-4)            /* HIP runtime failure                           */
#define WV_ERR_UNSUPPORTED (-5)    /* configuration not supported                   */
#define WV_ERR_QUANTIZER (-6)      /* "quantizer not initialized" (flat/index.go:463) */

/* distance providers: Shard.initVectorIndex (shard_init_vector.go:56-73) */
#define WV_METRIC_L2_SQUARED 0     /* "l2-squared" distancer/l2.go                  */
#define WV_METRIC_DOT 1            /* "dot"        distancer/dot_product.go         */
#define WV_METRIC_COSINE_DOT 2     /* "cosine-dot" distancer/cosine_dist.go         */
#define WV_METRIC_HAMMING 3        /* "hamming"    distancer/hamming.go             */

/* compression: flatent.UserConfig (entities/vectorindex/flat/config.go:43-82) */
#define WV_COMPRESSION_NONE 0
#define WV_COMPRESSION_BQ 1
/* PQ: ProductQuantizer (compressionhelpers/product_quantization.go) with the
 * KMeans encoder; searched like hnsw.flatSearch (hnsw/flat_search.go:28-141) */
#define WV_COMPRESSION_PQ 2
/* flat's rotational quantizers (flat/quantizer.go:31-36, :85-99): "rq-8" =
 * RotationalQuantizer (compressionhelpers/rotational_quantization.go) with 8
 * bits, "rq-1" = BinaryRotationalQuantizer (binary_rotational_quantization.go);
 * both seeded with DefaultFastRotationSeed (fast_rotation.go:27), created at the
 * first Add (flat/index.go:338-360), searched by searchByVectorQuantized
 * (:460-532) with rescore_limit = RQ.RescoreLimit */
#define WV_COMPRESSION_RQ8 3
#define WV_COMPRESSION_RQ1 4
/* HNSW's scalar quantizer (compressionhelpers/scalar_quantization.go,
 * NewHNSWSQCompressor compression.go:634-662): 8-bit codes over the trained
 * range [b, b + a]; searched like hnsw.flatSearch (see
 * wv_index_hnsw_flat_search) after wv_index_sq_fit / wv_index_sq_restore */
#define WV_COMPRESSION_SQ 5

/* which reference SIMD kernel's fp32 accumulation order to reproduce
 * (distancer/l2_amd64.go:19-26: AVX-512 only if AMX-BF16 && AVX512) */
#define WV_VARIANT_AUTO 0          /* same rule as the reference, on this host's CPU */
#define WV_VARIANT_AVX256 1
#define WV_VARIANT_AVX512 2

typedef struct wv_index wv_index;

/* flat.Config + flatent.UserConfig subset (flat/config.go:22-48) */
typedef struct wv_config {
    int32_t metric;          /* WV_METRIC_*                                           */
    int32_t dims;            /* 0 = fixed by the first Add (flat/index.go:338-360)    */
    int32_t compression;     /* WV_COMPRESSION_*                                      */
    int32_t rescore_limit;   /* BQ.RescoreLimit (default -1 => k, flat/index.go:413)  */
    int32_t device;          /* HIP device ordinal                                    */
    int32_t variant;         /* WV_VARIANT_*                                          */
    uint64_t id_base;        /* first doc id of this shard: slot = id - id_base       */
    const char *root_path;   /* only used in error texts (flat/index.go:837)          */
    /* PQ only (ent.PQConfig, entities/vectorindex/hnsw/pq_config.go) */
    int32_t pq_segments;     /* m: must divide dims                                   */
    int32_t pq_centroids;    /* ks <= 256                                             */
    int32_t pq_training_limit; /* rows used by Fit (<= 0: all)                        */
    int32_t pq_rescore;      /* 1: rescore the limit candidates with fp32 (h.rescore) */
} wv_config;

const char *wv_last_error(void);
int wv_resolve_variant(int32_t requested); /* -> WV_VARIANT_AVX256 / _AVX512 */

/* flat.New (flat/index.go:76-125) / Drop+Shutdown */
int wv_index_create(const wv_config *cfg, wv_index **out);
void wv_index_destroy(wv_index *idx);
/* pre-size the id-indexed store (cache.Grow analogue, cache/sharded_lock_cache.go) */
int wv_index_reserve(wv_index *idx, uint64_t nslots);

/* flat.ValidateBeforeInsert (flat/index.go:823-842) */
int wv_index_validate_before_insert(wv_index *idx, int64_t d);
/* flat.Add (flat/index.go:362-390): validate, normalise (cosine), upsert */
int wv_index_add(wv_index *idx, uint64_t id, const float *vec, int64_t d);
/* flat.AddBatch (flat/index.go:289-308): n rows of d floats */
int wv_index_add_batch(wv_index *idx, const uint64_t *ids, const float *vecs, int64_t n, int64_t d);
/* bulk load of ids [first_id, first_id+n) from a device buffer (PostStartup /
 * restore path, flat/index.go:867-1033) */
int wv_index_add_range_device(wv_index *idx, uint64_t first_id, const float *d_vecs, int64_t n, int64_t d);
/* flat.Delete (flat/index.go:392-411) */
int wv_index_delete(wv_index *idx, const uint64_t *ids, int64_t n);
/* flat.ContainsDoc (flat/index.go:1035-1055) */
int wv_index_contains_doc(wv_index *idx, uint64_t id);
/* flat.AlreadyIndexed (flat/index.go:1156-1158) */
uint64_t wv_index_already_indexed(wv_index *idx);
int32_t wv_index_dims(wv_index *idx);

/* ---- the rest of db.VectorIndex (adapters/repos/db/vector_index.go:25-54) -- */
/* flat.Iterate (flat/index.go:1057-1079): fn(id, user) for every stored id in
 * ascending order until fn returns 0 (snapshot taken under the index lock; fn
 * runs without it). */
int wv_index_iterate(wv_index *idx, int (*fn)(uint64_t id, void *user), void *user);
/* flat.QueryVectorDistancer(query).DistanceFunc(id) for n ids
 * (flat/index.go:1160-1240): SingleDist(normalised query, stored row); with
 * option "cache" = 1 on a BQ / RQ index, the quantized distance of the cached
 * code (createDistanceCalcQuantized, :534-566).  Missing ids fail as the
 * reference's empty bucket read does ("<qd> vs 0: vector lengths don't
 * match").  out_rc (may be NULL): per-id status; NULL returns the first
 * failure. */
int wv_index_query_distances(wv_index *idx, const float *query, int64_t qd, const uint64_t *ids, int64_t n,
                             float *out, int32_t *out_rc);
/* flat.Preload (flat/index.go:844-865): compressed index -> the row's code is
 * stored (rows and codes live together here; AlreadyIndexed unchanged);
 * uncompressed -> no-op. */
int wv_index_preload(wv_index *idx, uint64_t id, const float *vec, int64_t d);
/* flat.UpdateUserConfig (flat/index.go:763-776): applies the rescore limit
 * (extractCompressionRescore, :170-180). */
int wv_index_update_user_config(wv_index *idx, const wv_config *updated);
/* flat.ValidateUserConfigUpdate (flat/index.go:1106-1154): distance, pq, bq,
 * rq, rq.bits immutable -> "<name> is immutable: attempted change from ..." */
int wv_validate_user_config_update(const wv_config *initial, const wv_config *updated);
/* flat.CompressionStats (flat/index.go:1246-1249): UncompressedStats{} ->
 * type "none", ratio 1.0 */
int wv_index_compression_stats(wv_index *idx, char *type_out, int64_t type_cap, double *ratio);

/* flat.SearchByVector (flat/index.go:423-448 + :578-688) for nq queries.
 * allow_mode 0: allow list nil; 1: allow list = allow_ids[0..n_allow) (may be
 * empty -> empty results, flat/index.go:590-594).
 * out_ids/out_dists: nq x k, ascending, reference heap tie order; out_counts[nq]. */
int wv_index_search_by_vector_batch(wv_index *idx, const float *queries, int64_t nq, int64_t d, int32_t k,
                                    const uint64_t *allow_ids, int64_t n_allow, int32_t allow_mode,
                                    uint64_t *out_ids, float *out_dists, int32_t *out_counts);

/* flat.SearchByVector (flat/index.go:423-448) for nq queries, each under its
 * own allow list: query q uses allow_ids[allow_offsets[q] .. allow_offsets[q+1])
 * when allow_modes[q] == 1 (may be empty -> no results), no list when 0.
 * allow_offsets has nq+1 entries.  Results equal nq one-query calls of
 * wv_index_search_by_vector_batch (the concurrent filtered callers of
 * shard_read.go:415-424 in one launch); options "pqa" (default 1: one shared
 * block-key launch over the lists' union), "pqa_keys" (default 1: int8 dot /
 * cosine keys up to 768 dims masked per query, so each query's keys cover its
 * own rows only) and "pqa_budget_mb" (per-query bitmap memory per launch,
 * default 4096). */
int wv_index_search_by_vector_batch_multi_allow(wv_index *idx, const float *queries, int64_t nq, int64_t d,
                                                int32_t k, const uint64_t *allow_ids, const int64_t *allow_offsets,
                                                const int32_t *allow_modes, uint64_t *out_ids, float *out_dists,
                                                int32_t *out_counts);

/* The same with the lists as dense bitmaps -- the form of helpers.AllowList's
 * roaring bitmap (shard_read.go:401-413) -- instead of id arrays: query q's
 * list is the doc ids i with bit (i & 31) of word allow_bits[q * words + (i >> 5)]
 * set, when allow_modes[q] == 1 (ids past words * 32 are not listed).  At
 * 1M rows a 5 % list is 125 KB as a bitmap against 400 KB of ids.  Results
 * equal wv_index_search_by_vector_batch_multi_allow over the same lists. */
int wv_index_search_by_vector_batch_multi_allow_bitmap(wv_index *idx, const float *queries, int64_t nq, int64_t d,
                                                       int32_t k, const uint32_t *allow_bits, int64_t words,
                                                       const int32_t *allow_modes, uint64_t *out_ids,
                                                       float *out_dists, int32_t *out_counts);

/* flat.SearchByVector for ONE query (flat/index.go:423-448), the call a
 * goroutine makes (shard_read.go:415-424).  Thread-safe; concurrent callers on
 * one index are coalesced into batched launches (micro-batcher, batcher.hip):
 * a caller that finds no batch running leads the next one, waiting up to the
 * "batch_window_us" option (default 1000) for company -- and no longer once as
 * many callers are pending as were in the system during the previous batch --
 * at most "batch_max" (default 4096) queries per launch, grouped by (d, k); requests carrying
 * their own allow lists share a launch through
 * wv_index_search_by_vector_batch_multi_allow (a dense list -- over 1/64 of
 * its slot span -- travels as a slot bitmap the calling thread builds in a
 * page-locked row of its own, option "batch_rows", default 1).  Results and
 * errors equal those of a one-query wv_index_search_by_vector_batch.
 * out_ids/out_dists capacity k. */
int wv_index_search_by_vector(wv_index *idx, const float *query, int64_t d, int32_t k, const uint64_t *allow_ids,
                              int64_t n_allow, int32_t allow_mode, uint64_t *out_ids, float *out_dists,
                              int32_t *out_count);

/* out[3] = single-query calls, batched launches, largest batch so far */
int wv_index_batcher_stats(wv_index *idx, int64_t *out);

/* flat.SearchByVectorDistance (flat/index.go:699-761); out_* capacity >= 100 */
int wv_index_search_by_vector_distance(wv_index *idx, const float *query, int64_t d, float target_distance,
                                       int64_t max_limit, const uint64_t *allow_ids, int64_t n_allow,
                                       int32_t allow_mode, uint64_t *out_ids, float *out_dists,
                                       int32_t *out_count);

/* ProductQuantizer.Fit (product_quantization.go:378-424) on the stored rows
 * (the first pq_training_limit present rows in id order), one KMeansEncoder per
 * segment (kmeans_encoder.go:48-65: random init, graph pruning, 10 iterations,
 * delta 0.01) with PCG seed `seed + segment` (the reference seeds from
 * rand.Uint64()); then Encode of every stored row.  Later Adds are encoded. */
int wv_index_pq_fit(wv_index *idx, uint64_t seed);
/* NewProductQuantizerWithEncoders (:193-203): install centers [m][ks][ds], encode rows */
int wv_index_pq_set_centers(wv_index *idx, const float *centers, int64_t n_floats);
/* the trained codebook [m][ks][ds] (KMeansEncoder.ExposeDataForRestore order) */
int wv_index_pq_centers(wv_index *idx, float *out, int64_t n_floats);
/* codes of slots [0, n) as [n][m] bytes (ProductQuantizer.Encode of the stored rows) */
int wv_index_pq_codes(wv_index *idx, uint8_t *out, int64_t n);
/* out[4] = {m, ks, ds, trained} */
int wv_index_pq_info(wv_index *idx, int32_t *out);
/* PQDistancer.Distance (product_quantization.go:360-368) of `query` (as given)
 * against n codes [n][m]: LUT (DistanceLookUpTable) sums + Wrap */
int wv_index_pq_distance(wv_index *idx, const float *query, int64_t d, const uint8_t *codes, int64_t n,
                         float *out);

/* Rotational quantizer state: out[4] = {bits (8 / 1 / 0), rotation output dim D,
 * code length in bytes (rq-8: 16 + D, rq-1: 8 * (1 + D/64)), created} */
int wv_index_rq_info(wv_index *idx, int32_t *out);
/* codes of slots [0, n) in the reference's compressed-bucket formats
 * (flat/index.go:201-232 stores quantizer.Encode output): rq-8 RQCode
 * [lower|step|codeSum|norm2 as big-endian float32][D bytes]
 * (rotational_quantization.go:95-155); rq-1 RQOneBitCode little-endian u64
 * words [step (low 32) | squaredNorm (high 32)][D/64 sign words]
 * (binary_rotational_quantization.go:92-148).  out: n * code length bytes. */
int wv_index_rq_codes(wv_index *idx, void *out, int64_t n);
/* the quantized distance the scan uses (flat/index.go:536-560: rq-8
 * DistanceBetweenCompressedVectors(candidate, EncodeBytes(query)); rq-1
 * NewDistancer(query).Distance(candidate)) of nq queries (normalised for
 * cosine like SearchByVector) against slots [0, n): out [nq][n], +inf where a
 * slot holds no vector */
int wv_index_rq_distances(wv_index *idx, const float *queries, int64_t nq, int64_t d, float *out, int64_t n);

/* ScalarQuantizer: NewScalarQuantizer (scalar_quantization.go:73-97) trained
 * on the first training_limit stored vectors in id order (<= 0: all; the
 * reference samples hnsw.compress's cache dump, hnsw/compress.go:31-68), then
 * every stored vector encoded (Encode, :124-137) and later Adds encoded on
 * insert.  Errors: empty index ("compress command cannot be executed before
 * inserting some data", hnsw/compress.go:34-36). */
int wv_index_sq_fit(wv_index *idx, int64_t training_limit);
/* RestoreScalarQuantizer (scalar_quantization.go:99-112): "invalid range value
 * while restoring SQ settings" when a == 0 */
int wv_index_sq_restore(wv_index *idx, float a, float b);
/* out[0] = a, out[1] = b, out[2] = ready (0/1), out[3] = bytes per code (d + 8) */
int wv_index_sq_info(wv_index *idx, float *out);
/* the reference's code bytes of slots [0, n): out [n][d + 8] (codes, big-endian
 * sum, big-endian sum of squares) */
int wv_index_sq_codes(wv_index *idx, uint8_t *out, int64_t n);

/* hnsw.flatSearch (hnsw/flat_search.go:28-141, one worker: flatSearchConcurrency
 * > 1 makes the reference's tie order nondeterministic) + h.rescore
 * (hnsw/search.go:1047-1110, one worker) over the compressed vectors of a BQ /
 * PQ / SQ / rq-8 / rq-1 index: the filtered brute force that
 * hnsw.SearchByVector runs when the allow list is below flatSearchCutoff
 * (search.go:78-92).  limit = searchTimeEF(k) (search.go:44-76; options "ef"
 * (default -1 = dynamic), "ef_min" 100, "ef_max" 500, "ef_factor" 8) when
 * shouldRescore (search.go:182-189: compressed, option "hnsw_rescore" = 1,
 * and for SQ / RQ rescore_limit != 0), else k; SQ / RQ trim the results to
 * rescore_limit before rescoring when rescore_limit >= k.  Distances:
 * CompressorDistancer.DistanceToNode, rescoring SingleDist(query, vector).
 * Outputs [nq][k] ascending + counts; allow_mode as
 * wv_index_search_by_vector_batch. */
int wv_index_hnsw_flat_search(wv_index *idx, const float *queries, int64_t nq, int64_t d, int32_t k,
                              const uint64_t *allow_ids, int64_t n_allow, int32_t allow_mode, uint64_t *out_ids,
                              float *out_dists, int32_t *out_counts);

/* Device-resident batch search for sharded / benchmark callers.
 * mode 0: like SearchByVector (kout = k, tie cases resolved by heap replay).
 * mode 1: shard-local candidates: kout = k+1 verified results per query and
 *         d_flags[q] = 1 where the query needs the cross-shard replay.
 * stream: hipStream_t to order against (NULL = the null stream). */
int wv_index_search_device(wv_index *idx, const float *d_queries, int64_t nq, int64_t d, int32_t k, int32_t mode,
                           uint64_t *d_ids, float *d_dists, int32_t *d_counts, int32_t *d_flags, void *stream);

/* Cross-shard exact replay (distributed tie path): continue the
 * reference heap (priorityqueue NewMax + insertToHeap, flat/index.go:578-674)
 * over this shard's id range for the query rows listed in h_qlist, starting
 * from heap states in layout order h_in_ids/h_in_dists/h_in_len [nlist x k]
 * (NULL = empty heaps).  extract=0 writes the updated heap states to h_out_*;
 * extract=1 applies extractHeap (flat/index.go:676-688) and writes ascending
 * results.  d_queries are the raw query rows on the index's device. */
int wv_index_replay(wv_index *idx, const float *d_queries, int64_t nq, int64_t d, int32_t k,
                    const int32_t *h_qlist, int32_t nlist, const uint64_t *h_in_ids, const float *h_in_dists,
                    const int32_t *h_in_len, int32_t extract, uint64_t *h_out_ids, float *h_out_dists,
                    int32_t *h_out_len);
/* wv_index_replay on device buffers, ordered on `stream` (NULL = the null
 * stream), no host synchronisation: d_qlist[nlist], heap states
 * d_in_* / d_out_* [nlist x k] in layout order (d_in_len NULL = empty heaps);
 * extract=1 writes ascending results by list position.  When the index's last
 * search was wv_index_search_device over the same nq queries (no write since),
 * its block keys bound the scan (only blocks that can insert are visited);
 * otherwise every row's exact distance is computed. */
int wv_index_replay_device(wv_index *idx, const float *d_queries, int64_t nq, int64_t d, int32_t k,
                           const int32_t *d_qlist, int32_t nlist, const uint64_t *d_in_ids, const float *d_in_dists,
                           const int32_t *d_in_len, int32_t extract, uint64_t *d_out_ids, float *d_out_dists,
                           int32_t *d_out_len, void *stream);

/* Sharded BQ search (flat.searchByVectorQuantized over contiguous id-range
 * shards): the reference R-heap (flat/index.go:470-487) runs
 * across the shards in id order.
 * 1. wv_index_bq_begin: every shard, in parallel: encode the queries
 *    (normalised for cosine) and compute this shard's hamming block minima.
 * 2. wv_index_bq_replay: shard r continues the heaps of shard r-1 (device
 *    [nq][R] ids/dists in layout order + [nq] lengths; NULL = empty heaps);
 *    pop = 0 writes the heap states, pop = 1 (last shard) the candidates in
 *    the reference's pop order.  R = max(rescore_limit, k).
 * 3. wv_index_bq_rescore: exact SingleDist of the candidates this shard holds
 *    into d_E (other entries untouched).
 * 4. wv_bq_final: the rescoring heap (:525-531) over the candidates, with E
 *    gathered [world][nq][R]: the entry of an id comes from shard
 *    min(id / id_stride, world - 1).  Outputs [nq][k]. */
/* Sharded exact search in two phases (weaviate_amd/sharded.py):
 * phase 1: block keys + local candidate blocks of nq device queries;
 *   d_topA [nq][k+1] = this shard's k+1 smallest block-key A values, d_eps [nq]
 *   its per-query error bound.  WV_ERR_UNSUPPORTED when the index is not on the
 *   block-key path (callers then use wv_index_search_device mode 1);
 * phase 2: given every shard's d_topA / d_eps gathered ([world][nq][k+1],
 *   [world][nq]), cut the candidates with the global (k+1)-th smallest key and
 *   return mode 1's outputs (kout = k+1 verified results + flags). */
int wv_index_shard_phase1(wv_index *idx, const float *d_queries, int64_t nq, int64_t d, int32_t k, float *d_topA,
                          float *d_eps, void *stream);
int wv_index_shard_phase2(wv_index *idx, int32_t world, int64_t nq, const float *d_topA_all, const float *d_eps_all,
                          int32_t k, uint64_t *d_ids, float *d_dists, int32_t *d_counts, int32_t *d_flags,
                          void *stream);
/* wv_index_replay_device for every query with d_flags[q] != 0 (list built on
 * the device, no host synchronisation); states d_in_* and results d_out_*
 * indexed by query ([nq x k], [nq]), rows of unflagged queries untouched.
 * Needs this index's block keys of the same batch. */
/* Parallel cross-shard replay: every shard r >= 1 replays the
 * listed queries from a full heap of k copies of T_r (an upper bound of the
 * real heap top at its first row: the k-th smallest known bound of the shards
 * before it) and records every insertion in id order (d_rec_* [nlist x cap],
 * count cap + 1 = overflow); shard 0 replays from empty heaps
 * (wv_index_replay_device).  wv_heap_merge_records then applies insertToHeap
 * over the records of shards 1..world-1 (d_rec_* [world][nlist][cap]) on shard
 * 0's states and extracts: equal to the serial chain; d_unresolved[li] = 1
 * where a record overflowed (the caller replays those serially). */
int wv_index_replay_record_device(wv_index *idx, const float *d_queries, int64_t nq, int64_t d, int32_t k,
                                  const int32_t *d_qlist, int32_t nlist, const uint64_t *d_in_ids,
                                  const float *d_in_dists, const int32_t *d_in_len, int32_t cap, uint64_t *d_rec_ids,
                                  float *d_rec_dists, int32_t *d_rec_n, void *stream);
int wv_heap_merge_records(int32_t device, int32_t nlist, int32_t k, int32_t world, int32_t cap,
                          const uint64_t *d_st_ids, const float *d_st_dists, const int32_t *d_st_n,
                          const uint64_t *d_rec_ids, const float *d_rec_dists, const int32_t *d_rec_n,
                          uint64_t *d_out_ids, float *d_out_dists, int32_t *d_out_n, int32_t *d_unresolved,
                          void *stream);
int wv_index_replay_flags_device(wv_index *idx, const float *d_queries, int64_t nq, int64_t d, int32_t k,
                                 const int32_t *d_flags, const uint64_t *d_in_ids, const float *d_in_dists,
                                 const int32_t *d_in_len, int32_t extract, uint64_t *d_out_ids, float *d_out_dists,
                                 int32_t *d_out_len, void *stream);

int wv_index_bq_begin(wv_index *idx, const float *d_queries, int64_t nq, int64_t d, int32_t k, void *stream);
int wv_index_bq_replay(wv_index *idx, const uint64_t *d_in_ids, const float *d_in_dists, const int32_t *d_in_len,
                       int32_t pop, uint64_t *d_out_ids, float *d_out_dists, int32_t *d_out_len, void *stream);
int wv_index_bq_rescore(wv_index *idx, const uint64_t *d_ids, const int32_t *d_len, float *d_E, void *stream);
int wv_bq_final(int32_t device, int64_t nq, int32_t R, int32_t k, int32_t world, uint64_t id_stride,
                const uint64_t *d_ids, const int32_t *d_len, const float *d_E, uint64_t *d_out_ids, float *d_out_dists,
                int32_t *d_out_counts, void *stream);
/* Parallel form of step 2 (replaces the serial R-heap chain of
 * flat/index.go:470-487 across shards): wv_index_bq_bounds gives per query the
 * R smallest 256-row block minima of this shard ([nq][R] ascending, +inf
 * padded; each the exact hamming distance of one distinct row).  After an
 * all-gather, shard r >= 1 replays from a full heap of R copies of T_r (the
 * R-th smallest bound of the shards before it, >= the real heap top at its
 * first row) and records every insertion in id order
 * (wv_index_bq_replay_record: d_rec_* [nq][cap], count cap + 1 = overflow);
 * shard 0 runs wv_index_bq_replay (pop = 0).  wv_heap_merge_records (k = R)
 * applies the records on shard 0's states = the chain's final heaps, extracted
 * ascending (pop order reversed). */
int wv_index_bq_bounds(wv_index *idx, float *d_out, void *stream);
int wv_index_bq_replay_record(wv_index *idx, const uint64_t *d_in_ids, const float *d_in_dists,
                              const int32_t *d_in_len, int32_t cap, uint64_t *d_rec_ids, float *d_rec_dists,
                              int32_t *d_rec_n, void *stream);

/* Sharded hnsw flat search over compressed vectors (hnsw/flat_search.go:28-141
 * + h.rescore, hnsw/search.go:1047-1110, the search a trained PQ index
 * (search_pq) or an SQ index (search_hnsw_flat) runs; and flat's rq-8 / rq-1
 * searchByVectorQuantized, flat/index.go:460-532 (search_rq); weaviate_amd/sharded.py
 * ShardedQuantSearch).  Every shard holds a contiguous id range and the same
 * quantizer (wv_index_pq_set_centers / wv_index_sq_restore).  The worker heap
 * of limit R spans the shards in id order, exactly as BQ's R-heap above:
 *   wv_index_quant_begin     query state + the compressed distances of every row
 *                            of this shard to the batch (one group, <= 16 GiB)
 *                            and their 256-row block minima; out[4] = {R, block
 *                            count, rescore, final form};
 *   wv_index_quant_blockmin  the minima [nq][blocks] (each the distance of one
 *                            distinct row: the R smallest bound the heap top);
 *   wv_index_quant_replay    the worker heap over this shard from states d_in_*
 *                            ([nq][R] by query, NULL = empty): extract = 1 ->
 *                            ascending, 0 -> the state;
 *   wv_index_quant_replay_record  the same from R copies of a bound, recording
 *                            insertions (count cap + 1 = overflow);
 *   wv_index_quant_finish    from the merged worker heap (ascending, global ids):
 *                            the result without rescoring, else the rescoring
 *                            candidates (global ids, after the SQ trim);
 *   wv_index_quant_rescore   exact SingleDist of the candidates this shard holds;
 *   wv_quant_rescore_final   the rescoring heap over the [world][nq][R]
 *                            distance tiles (the entry of id from shard
 *                            min(id / id_stride, world - 1)): form 0 =
 *                            h.rescore, 1 = searchByVectorQuantized's heap
 *                            (flat/index.go:525-531) for flat rq-8 / rq-1
 *                            indexes (search_rq: every worker-heap item is a
 *                            candidate). */
int wv_index_quant_begin(wv_index *idx, const float *d_queries, int64_t nq, int64_t d, int32_t k, int64_t *out,
                         void *stream);
/* the largest batch wv_index_quant_begin takes on this shard (larger batches run
 * the protocol per query chunk, the chunk agreed by all ranks) */
int wv_index_quant_max_batch(wv_index *idx, int32_t k, int32_t world, int64_t *out);
int wv_index_quant_blockmin(wv_index *idx, float *d_out, void *stream);
int wv_index_quant_replay(wv_index *idx, const uint64_t *d_in_ids, const float *d_in_dists, const int32_t *d_in_len,
                          int32_t extract, uint64_t *d_out_ids, float *d_out_dists, int32_t *d_out_len, void *stream);
int wv_index_quant_replay_record(wv_index *idx, const uint64_t *d_in_ids, const float *d_in_dists,
                                 const int32_t *d_in_len, int32_t cap, uint64_t *d_rec_ids, float *d_rec_dists,
                                 int32_t *d_rec_n, void *stream);
int wv_index_quant_finish(wv_index *idx, const uint64_t *d_asc_ids, const float *d_asc_dists, const int32_t *d_asc_len,
                          uint64_t *d_out_ids, float *d_out_dists, int32_t *d_out_counts, uint64_t *d_cand_ids,
                          int32_t *d_cand_n, void *stream);
int wv_index_quant_rescore(wv_index *idx, const uint64_t *d_cand_ids, const int32_t *d_cand_n, float *d_E,
                           void *stream);
int wv_quant_rescore_final(int32_t device, int32_t form, int64_t nq, int32_t R, int32_t k, int32_t world,
                           uint64_t id_stride,
                           const uint64_t *d_cand_ids, const int32_t *d_cand_n, const float *d_E_all,
                           uint64_t *d_out_ids, float *d_out_dists, int32_t *d_out_counts, void *stream);

/* Merge shard-local candidate lists (mode-1 search outputs of G shards, each
 * [nq x (k+1)], gathered shard-major on this device) into the final top-k by
 * (distance, id); d_out_flags[q]=1 when a shard flagged q or the merged top
 * k+1 distances tie, i.e. the cross-shard replay must decide. */
int wv_merge_shards(int32_t device, int32_t nshards, int64_t nq, int32_t k, const uint64_t *d_ids,
                    const float *d_dists, const int32_t *d_counts, const int32_t *d_flags, uint64_t *d_out_ids,
                    float *d_out_dists, int32_t *d_out_counts, int32_t *d_out_flags, void *stream);

/* ---- the corpus sharded over GPUs, searched from one process ---------------
 * Weaviate searches every shard of a node inside one Go process and merges the
 * shard results there (adapters/repos/db/index.go:1928-2071, the merge
 * sortby_distances.go:20-48).  wv_multi holds the shards of the ranks
 * [rank0, rank0 + n_local) of a world of `world` ranks; rank r holds the doc
 * ids [r * id_stride, (r+1) * id_stride) (the last rank: every id above), so
 * one search over all ranks equals one flat index over the whole corpus bit
 * for bit (ids, distances, tie order: the two-phase protocol of DESIGN.md §4,
 * driven by the library, collectives on a transport it owns):
 *   WV_TRANSPORT_RCCL   one RCCL communicator per local shard (librccl.so.1,
 *                       bound at run time).  n_local == world: one process holds
 *                       every GPU (unique_id may be NULL); otherwise one process
 *                       per GPU group, all created with the 128-byte id that
 *                       wv_rccl_unique_id gave rank 0 (the host passes it on);
 *   WV_TRANSPORT_LOCAL  every rank is a shard of this process (devices may
 *                       repeat): device copies, for tests and cost models.
 * Every compression of the flat index: exact fp32 (two-phase block keys), BQ
 * (the R-heap of flat/index.go:460-532 across the shards + rescoring), rq-8 /
 * rq-1, trained PQ and SQ (the worker heap across the shards + rescoring:
 * DESIGN.md §4b); allow lists through the _allow / _multi_allow calls. */
#define WV_TRANSPORT_LOCAL 0
#define WV_TRANSPORT_RCCL 1
/*   WV_TRANSPORT_HOST   one local shard per process; every collective staged
 *                       through host memory and handed to the caller's
 *                       functions (e.g. a gloo / MPI / TCP all-gather): a
 *                       multi-process world without RCCL, or several processes
 *                       sharing one GPU in tests.  allgather: send[bytes] from
 *                       this rank -> recv[world][bytes]; broadcast: root's
 *                       buf[bytes] -> buf on every rank; both return 0 on success. */
#define WV_TRANSPORT_HOST 2
typedef int (*wv_host_allgather_fn)(const void *send, void *recv, int64_t bytes, void *user);
typedef int (*wv_host_broadcast_fn)(void *buf, int64_t bytes, int32_t root, void *user);
typedef struct wv_multi wv_multi;
typedef struct wv_multi_config {
    wv_config index;          /* every shard's config; .device / .id_base are set per shard */
    int32_t world;            /* ranks in the world                                      */
    int32_t rank0;            /* global rank of local shard 0                            */
    int32_t n_local;          /* shards held by this process (ranks rank0 ..)            */
    const int32_t *devices;   /* [n_local] HIP device of each local shard                */
    uint64_t id_stride;       /* doc ids per rank                                        */
    int32_t transport;        /* WV_TRANSPORT_*                                          */
    const void *unique_id;    /* RCCL over processes: rank 0's wv_rccl_unique_id bytes   */
    wv_host_allgather_fn host_allgather; /* WV_TRANSPORT_HOST                           */
    wv_host_broadcast_fn host_broadcast;
    void *host_user;
} wv_multi_config;
int wv_rccl_unique_id(void *out, int64_t cap); /* cap >= 128 */
int wv_multi_create(const wv_multi_config *cfg, wv_multi **out);
void wv_multi_destroy(wv_multi *m);
/* local shard i's index (owned by m): bulk loads, options, stats */
wv_index *wv_multi_shard(wv_multi *m, int32_t local);
/* flat.AddBatch routed by id to the owning local shard (an id of another
 * process's rank is an error) */
int wv_multi_add_batch(wv_multi *m, const uint64_t *ids, const float *vecs, int64_t n, int64_t d);
/* SearchByVector over all ranks: queries / outputs on local shard 0's device,
 * ordered after and before `stream` (NULL: synchronous).  Every process of a
 * multi-process world calls it with the same queries and gets the results. */
int wv_multi_search_device(wv_multi *m, const float *d_queries, int64_t nq, int64_t d, int32_t k, uint64_t *d_ids,
                           float *d_dists, int32_t *d_counts, void *stream);
/* the same from host buffers (nq x k outputs, ascending, reference tie order) */
int wv_multi_search_by_vector_batch(wv_multi *m, const float *queries, int64_t nq, int64_t d, int32_t k,
                                    uint64_t *out_ids, float *out_dists, int32_t *out_counts);
/* Filtered SearchByVector over every shard: each shard searches under its part
 * of the allow list (shard_read.go:401-413 -> flat SearchByVector(..., allowList),
 * :466; merged as index.go:2067-2071), equal to one flat index under the whole
 * list.  allow_mode 0: no list; 1: allow_ids[0..n_allow) (host, doc ids; ids of
 * other processes' ranks are ignored; empty -> no results, flat/index.go:590-594).
 * Every search kind of the shards takes it: exact, BQ, rq-8 / rq-1, trained PQ,
 * SQ.  The shards' handles must not be searched while a multi search runs. */
int wv_multi_search_by_vector_batch_allow(wv_multi *m, const float *queries, int64_t nq, int64_t d, int32_t k,
                                          const uint64_t *allow_ids, int64_t n_allow, int32_t allow_mode,
                                          uint64_t *out_ids, float *out_dists, int32_t *out_counts);
/* the same on device queries / outputs (local shard 0's device, `stream`) */
int wv_multi_search_device_allow(wv_multi *m, const float *d_queries, int64_t nq, int64_t d, int32_t k,
                                 const uint64_t *allow_ids, int64_t n_allow, int32_t allow_mode, uint64_t *d_ids,
                                 float *d_dists, int32_t *d_counts, void *stream);
/* every query under its own allow list (allow_offsets[nq+1], allow_modes[nq], as
 * wv_index_search_by_vector_batch_multi_allow); results equal nq one-query
 * filtered calls.  Queries with identical lists share one search. */
int wv_multi_search_by_vector_batch_multi_allow(wv_multi *m, const float *queries, int64_t nq, int64_t d, int32_t k,
                                                const uint64_t *allow_ids, const int64_t *allow_offsets,
                                                const int32_t *allow_modes, uint64_t *out_ids, float *out_dists,
                                                int32_t *out_counts);
/* SearchByVectorDistance over every shard (flat/index.go:699-761 per shard,
 * shard_read.go:439, merged by index.go:2067-2071); out_* capacity >= 100 */
int wv_multi_search_by_vector_distance(wv_multi *m, const float *query, int64_t d, float target_distance,
                                       int64_t max_limit, const uint64_t *allow_ids, int64_t n_allow,
                                       int32_t allow_mode, uint64_t *out_ids, float *out_dists, int32_t *out_count);
/* PQ shards: ProductQuantizer.Fit on the first trainingLimit present rows in
 * doc-id order over all shards (one process: gathered from the shards in rank
 * order; a world over processes: they must all lie on rank 0), the codebook
 * installed on every shard; _set_centers installs a codebook trained elsewhere. */
int wv_multi_pq_fit(wv_multi *m, uint64_t seed);
int wv_multi_pq_set_centers(wv_multi *m, const float *centers, int64_t n_floats);
/* "sim" = 1: local shards run each stage one after another, timed alone
 * (wv_multi_stage_ms); "rec_cap" (tests): capacity of the parallel replay's
 * insertion records (0 = max(256, 16 k), BQ 2R, quantized 2R + 64; a record
 * that overflows sends its query -- compressed: its chunk -- down the serial
 * chain); "chain" = 1 (tests): compressed searches take the serial chain; any
 * other key is set on every shard */
int wv_multi_set_option(wv_multi *m, const char *key, int64_t value);
/* out[n]: searches, flagged queries, overflowed records, chain hops, last
 * search's flagged and overflowed queries, world, rank0, n_local, transport,
 * last search's host time in the call and of it blocked in its host syncs (us) */
int wv_multi_stats(wv_multi *m, int64_t *out, int32_t n);
/* option sim: per-shard stage times averaged over the searches since "sim"
 * was last set, out[stage][n_local] for
 * stages phase 1, phase 2, merge, replay, record merge, chain, collectives
 * (the last one host-timed, in out[6][0]) */
int wv_multi_stage_ms(wv_multi *m, double *out, int32_t n_local_cap);

/* Provider.SingleDist batched over n pairs of d floats, exact reference order
 * (distancer/provider.go:14-24). Runs on device `device`. */
int wv_distance_batch(int32_t device, int32_t metric, int32_t variant, const float *a, const float *b, int64_t n,
                      int64_t d, float *out);
/* distancer.HammingBitwise batched (distancer/hamming.go:63-68) */
int wv_hamming_bitwise_batch(int32_t device, const uint64_t *a, const uint64_t *b, int64_t n, int64_t words,
                             float *out);
/* BinaryQuantizer.Encode batched (compressionhelpers/binary_quantization.go:28-47) */
int wv_bq_encode_batch(int32_t device, const float *vecs, int64_t n, int64_t d, uint64_t *out_codes);
/* distancer.Normalize batched (distancer/normalize.go:16-32) */
int wv_normalize_batch(int32_t device, const float *vecs, int64_t n, int64_t d, float *out);

/* synthetic data (bench/tests): kind 0 U[-1,1), 1 integer U{0..127}, 2 U[0,1) */
int wv_gen_device(int32_t device, int32_t kind, uint64_t seed, uint64_t row0, int64_t rows, int64_t d, float *d_out,
                  void *stream);

/* counters (docs/metrics.md analogue) */
typedef struct wv_stats {
    uint64_t queries;
    uint64_t batches;
    uint64_t replayed_queries;
    uint64_t mfma_launches;
    double last_select_ms;   /* k_mfma_select time of the last batch (HIP events) */
    double last_total_ms;
    uint64_t last_group_queries; /* queries in the timed (first) group of the last quantized batch */
    uint64_t last_route;     /* exact fp32 search route of the last batch: WV_ROUTE_* */
    uint64_t last_scan_rows; /* slots the last host-API batch scanned (an allow list: its slot span) */
} wv_stats;
/* wv_stats.last_route: which key / select kernel the last exact batch ran */
#define WV_ROUTE_NONE 0
#define WV_ROUTE_QS_BF16 1   /* k_qs_blockkey (bf16 block keys, d <= 768) */
#define WV_ROUTE_QS_W4 2     /* k_qs_blockkey_w4 (bf16 block keys, 768 < d <= 1536) */
#define WV_ROUTE_QS_INT8 3   /* k_q8_blockkey (int8 block keys, 384 < d <= 1536) */
#define WV_ROUTE_F32_SELECT 4 /* k_mfma_select3 (f32 MFMA select) */
#define WV_ROUTE_GEMV 5      /* k_gemv_select (HBM-streaming GEMV, small batches) */
#define WV_ROUTE_BQ_INT8 6   /* BQ block minima: k_q8_blockkey over +-1 code planes (integer MFMA) */
#define WV_ROUTE_BQ_VALU 7   /* BQ block minima: k_bq_blockmin_lds / k_bq_blockmin (xor + popcount) */
#define WV_ROUTE_PQ_INT8 8   /* PQ: k_q8_blockkey over the centred int8 reconstruction plane (l2-squared) */
#define WV_ROUTE_Q8_GEMV 9   /* k_q8_gemv (int8 block keys of <= 32 queries streamed through registers) */
#define WV_ROUTE_RQ8_INT8 10 /* flat rq-8: k_rq8_keys (exact rq-8 block minima on the integer MFMA) */
int wv_index_stats(wv_index *idx, wv_stats *out);

/* Diagnostic hook (tests): the last MFMA batch's candidates [nq][KP]:
 * approximate distances A, exact distances E, slots I (0xFFFFFFFF = none), and
 * per-query the eps of k_finalize's exactness proof.  Call with A == NULL to
 * get *KP only. */
int wv_index_debug_candidates(wv_index *idx, float *A, float *E, uint32_t *I, float *eps, int64_t nq, int32_t *KP);

/* Diagnostic hook (tests) of the block-key path: query q of the last batch
 * (first query chunk): its smallest approximate distance of every 32-row block
 * (A space, +inf for a block without a valid row) into A[*nb] and its error
 * bound eps(q).  Call with A == NULL to read *nb only. */
int wv_index_debug_blockkeys(wv_index *idx, int64_t q, float *A, float *eps, int64_t *nb);

/* Diagnostic hook (tests) of the BQ search: query q of the last BQ batch (one
 * query group): the minimum hamming distance of every block of *blk_rows rows
 * (256 on the VALU route, 32 on the integer-MFMA route; +inf without a valid
 * row) into mins[*nblk].  mins == NULL: the sizes only. */
int wv_index_debug_bqmin(wv_index *idx, int64_t q, float *mins, int64_t *nblk, int64_t *blk_rows);

/* tuning / testing knobs: "margin" (extra candidates of the f32 select
 * kernel, default 8), "force_replay" (1 = resolve every query by heap
 * replay), "spans" (0 = auto), "kernel" (0 = auto: 7 = bf16 block-key path
 * (qs_kernels.hip, the default for the exact fp32 search up to 1536 dims),
 * 6 = HBM-streaming GEMV, 3 = f32 MFMA select; other values are rejected),
 * "replay_par" (flagged-query replay form, default 2), "rp_few" (device-counted
 * replay lists up to this long take the one-launch 8-wave form, default 16),
 * "bq_fast" (1 = BQ queries whose rescored result no hamming tie can change
 * skip the R-heap replay, k_bq_fast; default 0: slower on C4),
 * "exact_bm" / "exact_cap"
 * / "exact_filter" (block-key exact pass forms; exact_filter 1 = bf16-plane row
 * bound in the capped pass, default), "replay_dbg" (1 = clock diagnostics of
 * the one-wave replay, printed), "pq_cand" (1 = minima-only PQ search, 0 = the
 * full ADC matrix), "pq_adc3" (1 = queries-on-lanes ADC for 256 centroids,
 * 0 = k_pq_adc2), "bq_kernel" (1 = generic BQ kernels), "timing" (1 = record
 * kernel times with HIP events), "batch_window_us" / "batch_max"
 * (micro-batcher, see wv_index_search_by_vector), "cache" (BQ.Cache /
 * RQ.Cache, default 0: see wv_index_query_distances) */
int wv_index_set_option(wv_index *idx, const char *key, int64_t value);

/* ---- LSM on-disk format: restore from flat's vectors bucket ----------------
 * Host-only (no GPU call).  Replace-strategy segment files as written by
 * lsmkv (segmentindex/header.go:24-42, segment_serialization.go:34-166,
 * segmentindex/segment_file.go:274-341 for the v1 CRC32 trailer).
 * validate_checksum != 0 checks the trailer of version >= 1 segments
 * (the bucket option enableChecksumValidation, segment.go:262-272). */

/* out[6] = level, version, secondary index count, strategy, indexStart, file size */
int wv_lsm_segment_header(const char *path, int32_t validate_checksum, int64_t *out);

/* Walk the data region [16, indexStart) node by node (ParseReplaceNode).
 * Fills up to cap entries (any array may be NULL): node [start, end) offsets,
 * tombstone flag, key as a big-endian uint64 when the key is 8 bytes (else
 * UINT64_MAX).  *out_n = number of nodes.  Non-replace strategy -> error
 * "unsupported strategy in segment: ...". */
int wv_lsm_segment_scan(const char *path, int32_t validate_checksum, int64_t *node_start, int64_t *node_end,
                        uint8_t *tombstone, uint64_t *key_id, int64_t cap, int64_t *out_n);

/* Replaces the startup path of flat.New → initBuckets → PostStartup
 * (flat/index.go:236-282, 867-1033): segments of the vectors bucket, oldest
 * first; key = big-endian uint64 id, value = d little-endian float32
 * (flat/index.go:204-208, 317-336).  Newest entry per key wins, tombstones
 * delete.  Live vectors are uploaded as stored (the bucket already holds the
 * values Add wrote, normalised for cosine: PostStartup reads them unchanged);
 * the compressed codes are re-derived from those fp32 values, which the
 * BQ/RQ/PQ encoders determine uniquely.  out[3] (may be NULL) = live
 * vectors uploaded, tombstoned keys, nodes read.  AlreadyIndexed becomes the
 * live count (flat/index.go:278-279). */
int wv_index_load_segments(wv_index *idx, const char *const *paths, int32_t n_paths, int32_t validate_checksum,
                           int64_t *out);

#ifdef __cplusplus
}
#endif
#endif /* WV_KNN_H */
