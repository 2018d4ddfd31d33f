"""ctypes binding of the C ABI in include/wv_knn.h.

The library is the product: if libwvknn.so is missing or fails to load, every
entry point raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libwvknn.so")

WV_OK = 0
WV_ERR_INVALID = -1
WV_ERR_VECTOR_LENGTH = -2
WV_ERR_INSERT = -3
WV_ERR_HIP = -4
WV_ERR_UNSUPPORTED = -5
WV_ERR_QUANTIZER = -6

METRIC_L2 = 0
METRIC_DOT = 1
METRIC_COSINE = 2
METRIC_HAMMING = 3

VARIANT_AUTO = 0
VARIANT_AVX256 = 1
VARIANT_AVX512 = 2

COMPRESSION_NONE = 0
COMPRESSION_BQ = 1
COMPRESSION_PQ = 2
COMPRESSION_RQ8 = 3
COMPRESSION_RQ1 = 4
COMPRESSION_SQ = 5


class WvConfig(C.Structure):
    _fields_ = [
        ("metric", C.c_int32),
        ("dims", C.c_int32),
        ("compression", C.c_int32),
        ("rescore_limit", C.c_int32),
        ("device", C.c_int32),
        ("variant", C.c_int32),
        ("id_base", C.c_uint64),
        ("root_path", C.c_char_p),
        ("pq_segments", C.c_int32),
        ("pq_centroids", C.c_int32),
        ("pq_training_limit", C.c_int32),
        ("pq_rescore", C.c_int32),
    ]


class WvMultiConfig(C.Structure):
    _fields_ = [
        ("index", WvConfig),
        ("world", C.c_int32),
        ("rank0", C.c_int32),
        ("n_local", C.c_int32),
        ("devices", C.POINTER(C.c_int32)),
        ("id_stride", C.c_uint64),
        ("transport", C.c_int32),
        ("unique_id", C.c_void_p),
        ("host_allgather", C.c_void_p),
        ("host_broadcast", C.c_void_p),
        ("host_user", C.c_void_p),
    ]


# WV_TRANSPORT_HOST callbacks (include/wv_knn.h)
HOST_ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p)
HOST_BROADCAST_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p)


class WvStats(C.Structure):
    _fields_ = [
        ("queries", C.c_uint64),
        ("batches", C.c_uint64),
        ("replayed_queries", C.c_uint64),
        ("mfma_launches", C.c_uint64),
        ("last_select_ms", C.c_double),
        ("last_total_ms", C.c_double),
        ("last_group_queries", C.c_uint64),
        ("last_route", C.c_uint64),
        ("last_scan_rows", C.c_uint64),
    ]


# wv_stats.last_route (include/wv_knn.h WV_ROUTE_*)
ROUTES = {0: "none", 1: "qs_bf16", 2: "qs_w4", 3: "qs_int8", 4: "f32_select", 5: "gemv", 6: "bq_int8", 7: "bq_valu",
          8: "pq_int8", 9: "q8_gemv", 10: "rq8_int8"}


P = C.c_void_p
# flat.Iterate callback: int fn(uint64_t id, void *user)
ITERATE_FN = C.CFUNCTYPE(C.c_int, C.c_uint64, C.c_void_p)
i32, i64, u64, f32 = C.c_int32, C.c_int64, C.c_uint64, C.c_float
pf32 = C.POINTER(C.c_float)
pu64 = C.POINTER(C.c_uint64)
pi32 = C.POINTER(C.c_int32)

# name -> (restype, argtypes); every symbol declared in include/wv_knn.h
SIGNATURES = {
    "wv_last_error": (C.c_char_p, []),
    "wv_resolve_variant": (C.c_int, [i32]),
    "wv_index_create": (C.c_int, [C.POINTER(WvConfig), C.POINTER(P)]),
    "wv_index_destroy": (None, [P]),
    "wv_index_reserve": (C.c_int, [P, u64]),
    "wv_index_validate_before_insert": (C.c_int, [P, i64]),
    "wv_index_add": (C.c_int, [P, u64, pf32, i64]),
    "wv_index_add_batch": (C.c_int, [P, pu64, pf32, i64, i64]),
    "wv_index_add_range_device": (C.c_int, [P, u64, P, i64, i64]),
    "wv_index_delete": (C.c_int, [P, pu64, i64]),
    "wv_index_contains_doc": (C.c_int, [P, u64]),
    "wv_index_already_indexed": (u64, [P]),
    "wv_index_dims": (i32, [P]),
    "wv_index_iterate": (C.c_int, [P, P, P]),
    "wv_index_query_distances": (C.c_int, [P, pf32, i64, pu64, i64, pf32, pi32]),
    "wv_index_preload": (C.c_int, [P, u64, pf32, i64]),
    "wv_index_update_user_config": (C.c_int, [P, C.POINTER(WvConfig)]),
    "wv_validate_user_config_update": (C.c_int, [C.POINTER(WvConfig), C.POINTER(WvConfig)]),
    "wv_index_compression_stats": (C.c_int, [P, C.c_char_p, i64, C.POINTER(C.c_double)]),
    "wv_index_search_by_vector_batch": (C.c_int, [P, pf32, i64, i64, i32, pu64, i64, i32, pu64, pf32, pi32]),
    "wv_index_search_by_vector_batch_multi_allow": (C.c_int, [P, pf32, i64, i64, i32, pu64, P, pi32, pu64, pf32,
                                                              pi32]),
    "wv_index_search_by_vector_batch_multi_allow_bitmap": (C.c_int, [P, pf32, i64, i64, i32, P, i64, pi32, pu64,
                                                                     pf32, pi32]),
    "wv_index_search_by_vector_distance": (C.c_int, [P, pf32, i64, f32, i64, pu64, i64, i32, pu64, pf32, pi32]),
    "wv_index_search_device": (C.c_int, [P, P, i64, i64, i32, i32, P, P, P, P, P]),
    "wv_index_replay_device": (C.c_int, [P, P, i64, i64, i32, P, i32, P, P, P, i32, P, P, P, P]),
    "wv_index_shard_phase1": (C.c_int, [P, P, i64, i64, i32, P, P, P]),
    "wv_index_shard_phase2": (C.c_int, [P, i32, i64, P, P, i32, P, P, P, P, P]),
    "wv_index_replay_flags_device": (C.c_int, [P, P, i64, i64, i32, P, P, P, P, i32, P, P, P, P]),
    "wv_index_replay_record_device": (C.c_int, [P, P, i64, i64, i32, P, i32, P, P, P, i32, P, P, P, P]),
    "wv_heap_merge_records": (C.c_int, [i32, i32, i32, i32, i32, P, P, P, P, P, P, P, P, P, P, P]),
    "wv_index_replay": (C.c_int, [P, P, i64, i64, i32, pi32, i32, pu64, pf32, pi32, i32, pu64, pf32, pi32]),
    "wv_merge_shards": (C.c_int, [i32, i32, i64, i32, P, P, P, P, P, P, P, P, P]),
    "wv_rccl_unique_id": (C.c_int, [P, i64]),
    "wv_multi_create": (C.c_int, [C.POINTER(WvMultiConfig), C.POINTER(P)]),
    "wv_multi_destroy": (None, [P]),
    "wv_multi_shard": (P, [P, i32]),
    "wv_multi_add_batch": (C.c_int, [P, pu64, pf32, i64, i64]),
    "wv_multi_search_device": (C.c_int, [P, P, i64, i64, i32, P, P, P, P]),
    "wv_multi_search_by_vector_batch": (C.c_int, [P, pf32, i64, i64, i32, pu64, pf32, pi32]),
    "wv_multi_search_by_vector_batch_allow": (C.c_int, [P, pf32, i64, i64, i32, pu64, i64, i32, pu64, pf32, pi32]),
    "wv_multi_search_device_allow": (C.c_int, [P, P, i64, i64, i32, pu64, i64, i32, P, P, P, P]),
    "wv_multi_search_by_vector_batch_multi_allow": (C.c_int, [P, pf32, i64, i64, i32, pu64, P, pi32, pu64, pf32,
                                                              pi32]),
    "wv_multi_search_by_vector_distance": (C.c_int, [P, pf32, i64, f32, i64, pu64, i64, i32, pu64, pf32, pi32]),
    "wv_multi_pq_fit": (C.c_int, [P, u64]),
    "wv_multi_pq_set_centers": (C.c_int, [P, pf32, i64]),
    "wv_multi_set_option": (C.c_int, [P, C.c_char_p, i64]),
    "wv_multi_stats": (C.c_int, [P, C.POINTER(C.c_int64), i32]),
    "wv_multi_stage_ms": (C.c_int, [P, C.POINTER(C.c_double), i32]),
    "wv_distance_batch": (C.c_int, [i32, i32, i32, pf32, pf32, i64, i64, pf32]),
    "wv_hamming_bitwise_batch": (C.c_int, [i32, pu64, pu64, i64, i64, pf32]),
    "wv_bq_encode_batch": (C.c_int, [i32, pf32, i64, i64, pu64]),
    "wv_normalize_batch": (C.c_int, [i32, pf32, i64, i64, pf32]),
    "wv_gen_device": (C.c_int, [i32, i32, u64, u64, i64, i64, P, P]),
    "wv_index_stats": (C.c_int, [P, C.POINTER(WvStats)]),
    "wv_index_debug_candidates": (C.c_int, [P, pf32, pf32, C.POINTER(C.c_uint32), pf32, i64, pi32]),
    "wv_index_debug_blockkeys": (C.c_int, [P, i64, pf32, pf32, C.POINTER(C.c_int64)]),
    "wv_index_bq_begin": (C.c_int, [P, P, i64, i64, i32, P]),
    "wv_index_bq_replay": (C.c_int, [P, P, P, P, i32, P, P, P, P]),
    "wv_index_bq_bounds": (C.c_int, [P, P, P]),
    "wv_index_bq_replay_record": (C.c_int, [P, P, P, P, i32, P, P, P, P]),
    "wv_index_bq_rescore": (C.c_int, [P, P, P, P, P]),
    "wv_bq_final": (C.c_int, [i32, i64, i32, i32, i32, u64, P, P, P, P, P, P, P]),
    "wv_index_quant_begin": (C.c_int, [P, P, i64, i64, i32, P, P]),
    "wv_index_quant_blockmin": (C.c_int, [P, P, P]),
    "wv_index_quant_max_batch": (C.c_int, [P, i32, i32, P]),
    "wv_index_debug_bqmin": (C.c_int, [P, i64, P, P, P]),
    "wv_index_quant_replay": (C.c_int, [P, P, P, P, i32, P, P, P, P]),
    "wv_index_quant_replay_record": (C.c_int, [P, P, P, P, i32, P, P, P, P]),
    "wv_index_quant_finish": (C.c_int, [P, P, P, P, P, P, P, P, P, P]),
    "wv_index_quant_rescore": (C.c_int, [P, P, P, P, P]),
    "wv_quant_rescore_final": (C.c_int, [i32, i32, i64, i32, i32, i32, u64, P, P, P, P, P, P, P]),
    "wv_index_pq_fit": (C.c_int, [P, u64]),
    "wv_index_pq_set_centers": (C.c_int, [P, pf32, i64]),
    "wv_index_pq_centers": (C.c_int, [P, pf32, i64]),
    "wv_index_pq_codes": (C.c_int, [P, C.POINTER(C.c_uint8), i64]),
    "wv_index_pq_info": (C.c_int, [P, pi32]),
    "wv_index_pq_distance": (C.c_int, [P, pf32, i64, C.POINTER(C.c_uint8), i64, pf32]),
    "wv_index_rq_info": (C.c_int, [P, pi32]),
    "wv_index_rq_codes": (C.c_int, [P, P, i64]),
    "wv_index_rq_distances": (C.c_int, [P, pf32, i64, i64, pf32, i64]),
    "wv_index_sq_fit": (C.c_int, [P, i64]),
    "wv_index_sq_restore": (C.c_int, [P, f32, f32]),
    "wv_index_sq_info": (C.c_int, [P, pf32]),
    "wv_index_sq_codes": (C.c_int, [P, C.POINTER(C.c_uint8), i64]),
    "wv_index_hnsw_flat_search": (C.c_int, [P, pf32, i64, i64, i32, pu64, i64, i32, pu64, pf32, pi32]),
    "wv_index_set_option": (C.c_int, [P, C.c_char_p, i64]),
    "wv_lsm_segment_header": (C.c_int, [C.c_char_p, i32, C.POINTER(C.c_int64)]),
    "wv_lsm_segment_scan": (C.c_int, [C.c_char_p, i32, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                      C.POINTER(C.c_uint8), pu64, i64, C.POINTER(C.c_int64)]),
    "wv_index_search_by_vector": (C.c_int, [P, pf32, i64, i32, pu64, i64, i32, pu64, pf32, pi32]),
    "wv_index_batcher_stats": (C.c_int, [P, C.POINTER(C.c_int64)]),
    "wv_index_load_segments": (C.c_int, [P, C.POINTER(C.c_char_p), i32, i32, C.POINTER(C.c_int64)]),
}

_lib = None


def load() -> C.CDLL:
    """Load libwvknn.so (raises if missing -- no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    # torch (if present) must load its HIP runtime first: our DT_NEEDED
    # libamdhip64.so.7 then binds to the same copy, so device pointers and
    # streams are shared with torch (one HIP runtime per process).
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    # WV_LIB_PATH: a timing-experiment build (tools/build_dbg.sh) in place of the product library
    path = os.environ.get("WV_LIB_PATH", LIB_PATH)
    if not os.path.exists(path):
        raise RuntimeError(
            f"weaviate_amd: {path} not built; run `python -m weaviate_amd.build` "
            "(the HIP library is required, there is no CPU fallback)")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class WeaviateError(RuntimeError):
    """Carries the reference's error text (wv_last_error)."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


def check(rc: int) -> None:
    if rc != WV_OK:
        msg = load().wv_last_error()
        raise WeaviateError(rc, msg.decode() if msg else f"error {rc}")
