"""Host-side mirror of Weaviate's flat vector index (adapters/repos/db/vector/flat).

Same method names, argument meaning and error behaviour as the reference's
`db.VectorIndex` implementation for the flat index (vector_index.go:25-54,
flat/index.go), backed by the gfx950 engine through the C ABI.  Vectors and
queries are numpy float32 arrays; doc ids are uint64.
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import WeaviateError, check

# Shard.initVectorIndex distance names (shard_init_vector.go:56-73)
DISTANCES = {
    "": _lib.METRIC_COSINE,
    "cosine": _lib.METRIC_COSINE,
    "cosine-dot": _lib.METRIC_COSINE,
    "dot": _lib.METRIC_DOT,
    "l2-squared": _lib.METRIC_L2,
    "hamming": _lib.METRIC_HAMMING,
}
VARIANTS = {"auto": _lib.VARIANT_AUTO, "avx256": _lib.VARIANT_AVX256, "avx512": _lib.VARIANT_AVX512}
PROVIDER_TYPE = {_lib.METRIC_L2: "l2-squared", _lib.METRIC_DOT: "dot", _lib.METRIC_COSINE: "cosine-dot",
                 _lib.METRIC_HAMMING: "hamming"}


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _uptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint64))


def _iptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


class AllowList:
    """helpers.AllowList (helpers/allow_list.go:19-37): a set of doc ids."""

    def __init__(self, ids: Iterable[int] = ()):
        self.ids = np.unique(np.asarray(list(ids), dtype=np.uint64))

    def is_empty(self) -> bool:
        return self.ids.size == 0


def _allow_args(allow: Optional[AllowList]):
    if allow is None:
        return None, 0, 0, None
    ids = np.ascontiguousarray(allow.ids, dtype=np.uint64)
    return _uptr(ids), ids.size, 1, ids


def make_config(distance: str = "cosine", dims: int = 0, device: int = 0, variant: str = "auto",
                root_path: bytes = b"", id_base: int = 0, bq: bool = False, rescore_limit: int = -1,
                pq: Optional[dict] = None, rq: Optional[dict] = None, sq: bool = False) -> "_lib.WvConfig":
    """flatent.UserConfig subset -> wv_config (include/wv_knn.h)."""
    if distance not in DISTANCES:
        raise WeaviateError(_lib.WV_ERR_INVALID, f"unrecognized or unsupported distance metric {distance!r}")
    # pq: ent.PQConfig subset {"segments", "centroids" (256), "trainingLimit" (100000), "rescore" (True)}
    pqc = dict(pq or {})
    # rq: flatent RQ config subset {"bits": 8 | 1} (entities/vectorindex/flat/config.go:27, :199-201);
    # its RescoreLimit is `rescore_limit`
    rqc = dict(rq or {})
    if rq is not None and int(rqc.get("bits", 8)) not in (1, 8):
        raise WeaviateError(_lib.WV_ERR_INVALID, "rq bits must be 1 or 8")
    comp = (_lib.COMPRESSION_BQ if bq else _lib.COMPRESSION_PQ if pq is not None
            else (_lib.COMPRESSION_RQ8 if int(rqc.get("bits", 8)) == 8 else _lib.COMPRESSION_RQ1)
            if rq is not None else _lib.COMPRESSION_SQ if sq else _lib.COMPRESSION_NONE)
    return _lib.WvConfig(DISTANCES[distance], int(dims), comp, int(rescore_limit), int(device),
                         VARIANTS[variant], int(id_base), root_path, int(pqc.get("segments", 0)),
                         int(pqc.get("centroids", 256)), int(pqc.get("trainingLimit", 100000)),
                         1 if pqc.get("rescore", True) else 0)


def validate_user_config_update(initial: dict, updated: dict) -> None:
    """flat.ValidateUserConfigUpdate (flat/index.go:1106-1154); dicts of
    make_config keyword arguments.  Raises WeaviateError on an immutable change."""
    a, b = make_config(**initial), make_config(**updated)
    check(_lib.load().wv_validate_user_config_update(C.byref(a), C.byref(b)))


class FlatIndex:
    """flat.New (flat/index.go:76-125) with the VectorIndex surface used on the
    hot path: Add, AddBatch, Delete, SearchByVector, SearchByVectorDistance,
    ValidateBeforeInsert, ContainsDoc, AlreadyIndexed."""

    def __init__(self, distance: str = "cosine", dims: int = 0, device: int = 0, variant: str = "auto",
                 root_path: str = "", id_base: int = 0, bq: bool = False, rescore_limit: int = -1,
                 pq: Optional[dict] = None, rq: Optional[dict] = None, sq: bool = False):
        self._l = _lib.load()
        self._root = root_path.encode()
        self._cfg_args = dict(distance=distance, dims=dims, device=device, variant=variant, root_path=self._root,
                              id_base=id_base, bq=bq, rescore_limit=rescore_limit, pq=pq, rq=rq, sq=sq)
        cfg = make_config(**self._cfg_args)
        h = C.c_void_p()
        check(self._l.wv_index_create(C.byref(cfg), C.byref(h)))
        self._h = h
        self.metric = DISTANCES[distance]
        self.bq = bool(bq)
        self.pq = pq is not None
        self.rq = rq is not None
        self.sq = bool(sq)
        self.rescore_limit = int(rescore_limit)
        self.device = device
        self.id_base = id_base

    # -- lifecycle --------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._l.wv_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def type(self) -> str:  # flat.Type (flat/index.go:1242)
        return "flat"

    def distancer_type(self) -> str:  # Provider.Type()
        return PROVIDER_TYPE[self.metric]

    def compressed(self) -> bool:  # flat.Compressed (flat/index.go): BQ quantizer built at New; PQ once fit
        return self.bq or (self.pq and self.pq_info()["trained"]) or (self.rq and self.rq_info()["created"])

    # -- rotational quantization (flat "rq-8" / "rq-1") ---------------------
    def rq_info(self) -> dict:
        out = np.zeros(4, np.int32)
        check(self._l.wv_index_rq_info(self._h, _iptr(out)))
        return {"bits": int(out[0]), "output_dim": int(out[1]), "code_bytes": int(out[2]), "created": bool(out[3])}

    def rq_codes(self, n: int) -> np.ndarray:
        """Codes of slots [0, n) in the reference formats: rq-8 uint8 [n][16 + D]
        (RQCode), rq-1 uint64 [n][1 + D/64] (RQOneBitCode)."""
        info = self.rq_info()
        if info["bits"] == 8:
            out = np.zeros((n, info["code_bytes"]), np.uint8)
        else:
            out = np.zeros((n, info["code_bytes"] // 8), np.uint64)
        check(self._l.wv_index_rq_codes(self._h, out.ctypes.data, int(n)))
        return out

    def rq_distances(self, queries, n: int) -> np.ndarray:
        """Quantized scan distances of queries [nq][d] against slots [0, n)."""
        q = np.ascontiguousarray(np.atleast_2d(queries), dtype=np.float32)
        out = np.zeros((q.shape[0], n), np.float32)
        check(self._l.wv_index_rq_distances(self._h, _fptr(q), q.shape[0], q.shape[1], _fptr(out), int(n)))
        return out

    def debug_candidates(self, nq: int):
        """Diagnostic: (A, E, slots, eps) of the last MFMA batch (see wv_knn.h)."""
        kp = C.c_int32()
        check(self._l.wv_index_debug_candidates(self._h, None, None, None, None, int(nq), C.byref(kp)))
        A = np.zeros((nq, kp.value), np.float32)
        E = np.zeros_like(A)
        I = np.zeros((nq, kp.value), np.uint32)
        eps = np.zeros(nq, np.float32)
        check(self._l.wv_index_debug_candidates(self._h, _fptr(A), _fptr(E), I.ctypes.data_as(C.POINTER(C.c_uint32)),
                                                _fptr(eps), int(nq), C.byref(kp)))
        return A, E, I, eps

    def debug_blockkeys(self, q: int):
        """Diagnostic: (A_block[nb], eps) of query q of the last block-key batch
        (see wv_index_debug_blockkeys in include/wv_knn.h)."""
        nb = C.c_int64(0)
        check(self._l.wv_index_debug_blockkeys(self._h, int(q), None, None, C.byref(nb)))
        A = np.zeros(nb.value, np.float32)
        eps = np.zeros(1, np.float32)
        check(self._l.wv_index_debug_blockkeys(self._h, int(q), _fptr(A), _fptr(eps), C.byref(nb)))
        return A, float(eps[0])

    def debug_bqmin(self, q: int, rows: int = 256) -> np.ndarray:
        """Diagnostic: the block minima of hamming distances of query q of the
        last BQ batch (wv_index_debug_bqmin in include/wv_knn.h), reduced to
        blocks of `rows` rows (a multiple of the route's block size)."""
        nb, br = C.c_int64(0), C.c_int64(0)
        check(self._l.wv_index_debug_bqmin(self._h, int(q), None, C.byref(nb), C.byref(br)))
        out = np.zeros(nb.value, np.float32)
        check(self._l.wv_index_debug_bqmin(self._h, int(q), _fptr(out), C.byref(nb), C.byref(br)))
        f = rows // br.value
        if f > 1:
            m = -(-out.size // f) * f
            out = np.concatenate([out, np.full(m - out.size, np.inf, np.float32)]).reshape(-1, f).min(axis=1)
        return out

    # -- product quantizer (compressionhelpers.ProductQuantizer) -----------
    def pq_info(self) -> dict:
        out = (C.c_int32 * 4)()
        check(self._l.wv_index_pq_info(self._h, out))
        return {"segments": out[0], "centroids": out[1], "ds": out[2], "trained": bool(out[3])}

    def pq_fit(self, seed: int = 0) -> None:
        """ProductQuantizer.Fit on the stored rows + Encode of every row."""
        check(self._l.wv_index_pq_fit(self._h, int(seed) & (2**64 - 1)))

    def pq_centers(self) -> np.ndarray:
        i = self.pq_info()
        out = np.zeros((i["segments"], i["centroids"], i["ds"]), dtype=np.float32)
        check(self._l.wv_index_pq_centers(self._h, _fptr(out), out.size))
        return out

    def pq_set_centers(self, centers) -> None:
        c = np.ascontiguousarray(centers, dtype=np.float32)
        check(self._l.wv_index_pq_set_centers(self._h, _fptr(c), c.size))

    def pq_codes(self, n: int) -> np.ndarray:
        m = self.pq_info()["segments"]
        out = np.zeros((n, m), dtype=np.uint8)
        check(self._l.wv_index_pq_codes(self._h, out.ctypes.data_as(C.POINTER(C.c_uint8)), n))
        return out

    def pq_distance(self, query, codes) -> np.ndarray:
        """PQDistancer.Distance of `query` (as given) against code rows."""
        q = np.ascontiguousarray(query, dtype=np.float32)
        c = np.ascontiguousarray(codes, dtype=np.uint8)
        out = np.zeros(c.shape[0], dtype=np.float32)
        check(self._l.wv_index_pq_distance(self._h, _fptr(q), q.size, c.ctypes.data_as(C.POINTER(C.c_uint8)),
                                           c.shape[0], _fptr(out)))
        return out

    # -- scalar quantizer (HNSW's SQ compressor) ----------------------------
    def sq_fit(self, training_limit: int = 0) -> None:
        """NewScalarQuantizer over the first training_limit stored vectors (id
        order; <= 0: all) + Encode of every stored vector."""
        check(self._l.wv_index_sq_fit(self._h, int(training_limit)))

    def sq_restore(self, a: float, b: float) -> None:  # RestoreScalarQuantizer
        check(self._l.wv_index_sq_restore(self._h, float(a), float(b)))

    def sq_info(self) -> dict:
        out = np.zeros(4, np.float32)
        check(self._l.wv_index_sq_info(self._h, _fptr(out)))
        return {"a": float(out[0]), "b": float(out[1]), "ready": bool(out[2]), "code_bytes": int(out[3])}

    def sq_codes(self, n: int) -> np.ndarray:
        """Codes of slots [0, n) in the reference byte format [n][d + 8]."""
        out = np.zeros((n, self.sq_info()["code_bytes"]), np.uint8)
        check(self._l.wv_index_sq_codes(self._h, out.ctypes.data_as(C.POINTER(C.c_uint8)), int(n)))
        return out

    def hnsw_flat_search(self, queries, k: int, allow: Optional[AllowList] = None):
        """hnsw.flatSearch + h.rescore over the compressed vectors (BQ / PQ / SQ /
        RQ): wv_index_hnsw_flat_search.  Options "ef", "ef_min", "ef_max",
        "ef_factor", "hnsw_rescore" (set_option) are the hnsw UserConfig's.
        Returns (ids[nq,k], dists[nq,k], counts[nq])."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        nq, d = q.shape
        kk = max(int(k), 1)
        ids = np.zeros((nq, kk), dtype=np.uint64)
        dists = np.zeros((nq, kk), dtype=np.float32)
        counts = np.zeros(nq, dtype=np.int32)
        ap, na, mode, _keep = _allow_args(allow)
        check(self._l.wv_index_hnsw_flat_search(self._h, _fptr(q), nq, d, int(k), ap, na, mode, _uptr(ids),
                                                _fptr(dists), _iptr(counts)))
        return ids, dists, counts

    def reserve(self, nslots: int) -> None:
        check(self._l.wv_index_reserve(self._h, int(nslots)))

    def set_option(self, key: str, value: int) -> None:
        check(self._l.wv_index_set_option(self._h, key.encode(), int(value)))

    def stats(self) -> dict:
        s = _lib.WvStats()
        check(self._l.wv_index_stats(self._h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in s._fields_}

    # -- insert path ------------------------------------------------------
    def validate_before_insert(self, vector) -> None:  # flat/index.go:823-842
        check(self._l.wv_index_validate_before_insert(self._h, len(vector)))

    def add(self, id: int, vector) -> None:  # flat/index.go:362-390
        v = np.ascontiguousarray(vector, dtype=np.float32)
        check(self._l.wv_index_add(self._h, int(id), _fptr(v), v.size))

    def add_batch(self, ids: Sequence[int], vectors) -> None:  # flat/index.go:289-308
        if len(ids) != len(vectors):
            raise WeaviateError(_lib.WV_ERR_INSERT, "ids and vectors sizes does not match")
        if len(ids) == 0:
            raise WeaviateError(_lib.WV_ERR_INSERT, "insertBatch called with empty lists")
        if isinstance(vectors, np.ndarray) and vectors.ndim == 2:
            v = np.ascontiguousarray(vectors, dtype=np.float32)
            i = np.ascontiguousarray(ids, dtype=np.uint64)
            check(self._l.wv_index_add_batch(self._h, _uptr(i), _fptr(v), v.shape[0], v.shape[1]))
            return
        # ragged input: the reference loops Add and stops at the first error
        for id_, vec in zip(ids, vectors):
            self.add(id_, vec)

    def delete(self, *ids: int) -> None:  # flat/index.go:392-411
        a = np.ascontiguousarray(ids, dtype=np.uint64)
        check(self._l.wv_index_delete(self._h, _uptr(a), a.size))

    def load_segments(self, paths: Sequence[str], validate_checksum: bool = True) -> dict:
        """Restore from the vectors bucket's LSM segments, oldest first
        (initBuckets + PostStartup, flat/index.go:236-282, 867-1033); see
        wv_index_load_segments in include/wv_knn.h."""
        arr = (C.c_char_p * max(len(paths), 1))(*[str(p).encode() for p in paths])
        out = (C.c_int64 * 3)()
        check(self._l.wv_index_load_segments(self._h, arr, len(paths), int(bool(validate_checksum)), out))
        return {"loaded": out[0], "tombstoned": out[1], "nodes": out[2]}

    def contains_doc(self, id: int) -> bool:  # flat/index.go:1035-1055
        return bool(self._l.wv_index_contains_doc(self._h, int(id)))

    def already_indexed(self) -> int:  # flat/index.go:1156-1158
        return int(self._l.wv_index_already_indexed(self._h))

    @property
    def dims(self) -> int:
        return int(self._l.wv_index_dims(self._h))

    # -- search path ------------------------------------------------------
    # -- rest of db.VectorIndex (vector_index.go:25-54) -----------------------
    def iterate(self, fn) -> None:
        """flat.Iterate (flat/index.go:1057-1079): fn(id) -> bool, ascending ids."""
        cb = _lib.ITERATE_FN(lambda i, _u: 1 if fn(int(i)) else 0)
        check(self._l.wv_index_iterate(self._h, C.cast(cb, C.c_void_p), None))

    def query_vector_distances(self, query, ids, per_id_status: bool = False):
        """flat.QueryVectorDistancer(query).DistanceFunc over ids
        (flat/index.go:1160-1240).  per_id_status: -> (dists, rc[]) instead of
        raising on the first missing id."""
        q = np.ascontiguousarray(query, dtype=np.float32).ravel()
        i = np.ascontiguousarray(ids, dtype=np.uint64).ravel()
        out = np.zeros(i.size, np.float32)
        rc = np.zeros(i.size, np.int32) if per_id_status else None
        check(self._l.wv_index_query_distances(self._h, _fptr(q), q.size, i.ctypes.data_as(C.POINTER(C.c_uint64)),
                                               i.size, _fptr(out), _iptr(rc) if rc is not None else None))
        return (out, rc) if per_id_status else out

    def query_vector_distancer(self, query):
        """-> DistanceFunc(id) like common.QueryVectorDistancer."""
        return lambda doc_id: float(self.query_vector_distances(query, [doc_id])[0])

    def preload(self, id: int, vector) -> None:  # flat/index.go:844-865
        v = np.ascontiguousarray(vector, dtype=np.float32).ravel()
        check(self._l.wv_index_preload(self._h, int(id), _fptr(v), v.size))

    def update_user_config(self, **updated) -> None:
        """flat.UpdateUserConfig (flat/index.go:763-776), after
        ValidateUserConfigUpdate against the current config."""
        new = dict(self._cfg_args, **updated)
        validate_user_config_update(self._cfg_args, new)
        cfg = make_config(**new)
        check(self._l.wv_index_update_user_config(self._h, C.byref(cfg)))
        self._cfg_args = new
        self.rescore_limit = int(new["rescore_limit"])

    # upgradableIndexer of the flat index itself (flat/index.go:1251-1261)
    def should_upgrade(self) -> tuple:
        return False, 0

    def upgrade(self, callback=None) -> None:
        if callback is not None:
            callback()

    def upgraded(self) -> bool:
        return False

    def compression_stats(self) -> dict:  # flat/index.go:1246-1249
        buf = C.create_string_buffer(32)
        ratio = C.c_double(0)
        check(self._l.wv_index_compression_stats(self._h, buf, 32, C.byref(ratio)))
        return {"type": buf.value.decode(), "ratio": ratio.value}

    def search_by_vector_batch(self, queries, k: int, allow: Optional[AllowList] = None):
        """SearchByVector for each row of `queries` (flat/index.go:423-448).
        Returns (ids[nq,k] uint64, dists[nq,k] float32, counts[nq] int32)."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        nq, d = q.shape
        kk = max(int(k), 1)
        ids = np.zeros((nq, kk), dtype=np.uint64)
        dists = np.zeros((nq, kk), dtype=np.float32)
        counts = np.zeros(nq, dtype=np.int32)
        ap, na, mode, _keep = _allow_args(allow)
        check(self._l.wv_index_search_by_vector_batch(self._h, _fptr(q), nq, d, int(k), ap, na, mode, _uptr(ids),
                                                      _fptr(dists), _iptr(counts)))
        return ids, dists, counts

    def search_by_vector_batch_multi_allow(self, queries, k: int, allows, bitmap: bool = False):
        """SearchByVector for each row of `queries`, row i under its own allow
        list allows[i] (None = unfiltered): one batched call
        (wv_index_search_by_vector_batch_multi_allow, or with bitmap=True the
        lists as dense doc-id bitmaps, ..._multi_allow_bitmap), results equal
        to per-row search_by_vector_batch calls.
        Returns (ids[nq,k] uint64, dists[nq,k] float32, counts[nq] int32)."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        nq, d = q.shape
        allows = list(allows)
        if len(allows) != nq:
            raise WeaviateError(_lib.WV_ERR_INVALID, f"{len(allows)} allow lists for {nq} queries")
        kk = max(int(k), 1)
        ids = np.zeros((nq, kk), dtype=np.uint64)
        dists = np.zeros((nq, kk), dtype=np.float32)
        counts = np.zeros(nq, dtype=np.int32)
        modes = np.array([0 if a is None else 1 for a in allows], dtype=np.int32)
        if bitmap:
            top = max([int(a.ids.max()) + 1 for a in allows if a is not None and a.ids.size] + [1])
            words = (top + 31) // 32
            bits = np.zeros((nq, words), dtype=np.uint32)
            for i, a in enumerate(allows):
                if a is not None and a.ids.size:
                    v = np.asarray(a.ids, dtype=np.uint64)
                    np.bitwise_or.at(bits[i], (v >> 5).astype(np.int64), (np.uint32(1) << (v & 31).astype(np.uint32)))
            check(self._l.wv_index_search_by_vector_batch_multi_allow_bitmap(
                self._h, _fptr(q), nq, d, int(k), bits.ctypes.data_as(C.c_void_p), words, _iptr(modes), _uptr(ids),
                _fptr(dists), _iptr(counts)))
            return ids, dists, counts
        parts = [np.asarray(a.ids, dtype=np.uint64) for a in allows if a is not None]
        aids = np.ascontiguousarray(np.concatenate(parts) if parts else np.zeros(1, np.uint64), dtype=np.uint64)
        off = np.zeros(nq + 1, dtype=np.int64)
        off[1:] = np.cumsum([0 if a is None else a.ids.size for a in allows])
        check(self._l.wv_index_search_by_vector_batch_multi_allow(
            self._h, _fptr(q), nq, d, int(k), _uptr(aids), off.ctypes.data_as(C.c_void_p), _iptr(modes), _uptr(ids),
            _fptr(dists), _iptr(counts)))
        return ids, dists, counts

    def search_by_vector(self, vector, k: int, allow: Optional[AllowList] = None):
        """flat.SearchByVector: (ids, dists) ascending, len <= k.  One query per
        call, safe to call from many threads at once: concurrent calls are
        coalesced into batched launches by the C side's micro-batcher
        (wv_index_search_by_vector)."""
        v = np.ascontiguousarray(vector, dtype=np.float32).ravel()
        kk = max(int(k), 1)
        ids = np.zeros(kk, dtype=np.uint64)
        dists = np.zeros(kk, dtype=np.float32)
        n = C.c_int32(0)
        ap, na, mode, _keep = _allow_args(allow)
        check(self._l.wv_index_search_by_vector(self._h, _fptr(v), v.size, int(k), ap, na, mode, _uptr(ids),
                                                _fptr(dists), C.byref(n)))
        return ids[:n.value].copy(), dists[:n.value].copy()

    def batcher_stats(self) -> dict:
        out = (C.c_int64 * 3)()
        check(self._l.wv_index_batcher_stats(self._h, out))
        return {"calls": out[0], "launches": out[1], "max_batch": out[2]}

    def search_by_vector_distance(self, vector, target_distance: float, max_limit: int,
                                  allow: Optional[AllowList] = None):
        """flat.SearchByVectorDistance (flat/index.go:699-761)."""
        v = np.ascontiguousarray(vector, dtype=np.float32)
        ids = np.zeros(100, dtype=np.uint64)
        dists = np.zeros(100, dtype=np.float32)
        n = np.zeros(1, dtype=np.int32)
        ap, na, mode, _keep = _allow_args(allow)
        check(self._l.wv_index_search_by_vector_distance(self._h, _fptr(v), v.size, float(target_distance),
                                                         int(max_limit), ap, na, mode, _uptr(ids), _fptr(dists),
                                                         _iptr(n)))
        return ids[: n[0]].copy(), dists[: n[0]].copy()


# ---------------------------------------------------------------------------
# distancer.Provider mirror (distancer/provider.go:14-24), batched on the GPU
# ---------------------------------------------------------------------------
def single_dist_batch(distance: str, a, b, variant: str = "auto", device: int = 0) -> np.ndarray:
    """Provider.SingleDist(a[i], b[i]) for every row pair, exact reference order."""
    lib = _lib.load()
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    if a.ndim == 1:
        a, b = a[None, :], b[None, :]
    if a.shape != b.shape:
        raise WeaviateError(_lib.WV_ERR_VECTOR_LENGTH,
                            f"{a.shape[-1]} vs {b.shape[-1]}: vector lengths don't match")
    out = np.zeros(a.shape[0], dtype=np.float32)
    check(lib.wv_distance_batch(device, DISTANCES[distance], VARIANTS[variant], _fptr(a), _fptr(b), a.shape[0],
                                a.shape[1], _fptr(out)))
    return out


def hamming_bitwise_batch(a, b, device: int = 0) -> np.ndarray:
    """distancer.HammingBitwise over rows of uint64 words."""
    lib = _lib.load()
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    if a.ndim == 1:
        a, b = a[None, :], b[None, :]
    if a.shape != b.shape:
        raise WeaviateError(_lib.WV_ERR_VECTOR_LENGTH, "both vectors should have the same len")
    out = np.zeros(a.shape[0], dtype=np.float32)
    check(lib.wv_hamming_bitwise_batch(device, _uptr(a), _uptr(b), a.shape[0], a.shape[1], _fptr(out)))
    return out


def bq_encode_batch(vecs, device: int = 0) -> np.ndarray:
    """BinaryQuantizer.Encode over rows."""
    lib = _lib.load()
    v = np.ascontiguousarray(vecs, dtype=np.float32)
    if v.ndim == 1:
        v = v[None, :]
    words = (v.shape[1] + 63) // 64
    out = np.zeros((v.shape[0], words), dtype=np.uint64)
    check(lib.wv_bq_encode_batch(device, _fptr(v), v.shape[0], v.shape[1], _uptr(out)))
    return out


def normalize_batch(vecs, device: int = 0) -> np.ndarray:
    """distancer.Normalize over rows."""
    lib = _lib.load()
    v = np.ascontiguousarray(vecs, dtype=np.float32)
    if v.ndim == 1:
        v = v[None, :]
    out = np.zeros_like(v)
    check(lib.wv_normalize_batch(device, _fptr(v), v.shape[0], v.shape[1], _fptr(out)))
    return out


def lsm_segment_header(path: str, validate_checksum: bool = True) -> dict:
    """segmentindex.ParseHeader (+ ValidateChecksum for v1) of one segment file."""
    out = (C.c_int64 * 6)()
    check(_lib.load().wv_lsm_segment_header(str(path).encode(), int(bool(validate_checksum)), out))
    return dict(zip(("level", "version", "secondary_indices", "strategy", "index_start", "size"), list(out)))


def lsm_segment_scan(path: str, validate_checksum: bool = True) -> dict:
    """Walk a replace-strategy segment's nodes (ParseReplaceNode,
    lsmkv/segment_serialization.go:106-166): offsets, tombstones, BE uint64 keys."""
    lib = _lib.load()
    n = C.c_int64(0)
    bpath = str(path).encode()
    check(lib.wv_lsm_segment_scan(bpath, int(bool(validate_checksum)), None, None, None, None, 0, C.byref(n)))
    m = n.value
    start = np.zeros(m, np.int64)
    end = np.zeros(m, np.int64)
    tomb = np.zeros(m, np.uint8)
    keys = np.zeros(m, np.uint64)
    check(lib.wv_lsm_segment_scan(bpath, int(bool(validate_checksum)),
                                  start.ctypes.data_as(C.POINTER(C.c_int64)), end.ctypes.data_as(C.POINTER(C.c_int64)),
                                  tomb.ctypes.data_as(C.POINTER(C.c_uint8)), _uptr(keys), m, C.byref(n)))
    return {"start": start, "end": end, "tombstone": tomb.astype(bool), "key_id": keys}
