"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of oracle/liboracle.so (the CPU
restatement of the reference's flat-index hot path, oracle/oracle.c) and of
oracle/_ref/libref.so (the reference's own distance kernels compiled from
/root/reference).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref.so")

L2, DOT, COSINE, HAMMING = 0, 1, 2, 3
AVX256, AVX512 = 1, 2
METRIC = {"l2-squared": L2, "dot": DOT, "cosine": COSINE, "cosine-dot": COSINE, "hamming": HAMMING}

pf = C.POINTER(C.c_float)
pu = C.POINTER(C.c_uint64)
pi = C.POINTER(C.c_int)
pb = C.POINTER(C.c_uint8)

_o = None
_r = None


def lib() -> C.CDLL:
    global _o
    if _o is None:
        if not os.path.exists(ORACLE_SO):
            import subprocess
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        o = C.CDLL(ORACLE_SO)
        for n in ["or_l2_256", "or_l2_512", "or_dot_256", "or_dot_512", "or_hamming_f32"]:
            getattr(o, n).restype = C.c_float
            getattr(o, n).argtypes = [pf, pf, C.c_long]
        o.or_hamming_bitwise.restype = C.c_float
        o.or_hamming_bitwise.argtypes = [pu, pu, C.c_long]
        o.or_normalize.argtypes = [pf, pf, C.c_long]
        o.or_single_dist.restype = C.c_float
        o.or_single_dist.argtypes = [C.c_int, C.c_int, pf, pf, C.c_long]
        o.or_flat_search.restype = C.c_int
        o.or_flat_search.argtypes = [C.c_int, C.c_int, pf, pb, C.c_long, C.c_long, pf, C.c_long, C.c_int, pb,
                                     C.c_int, pu, pf, pi]
        o.or_bq_encode.argtypes = [pf, C.c_long, pu]
        o.or_flat_search_bq.restype = C.c_int
        o.or_flat_search_bq.argtypes = [C.c_int, C.c_int, pf, pb, pb, pu, C.c_long, C.c_long, pf, C.c_long, C.c_int,
                                        C.c_int, pb, C.c_int, pu, pf, pi]
        o.or_filter_by_distance.restype = C.c_int
        o.or_filter_by_distance.argtypes = [pu, pf, C.c_int, C.c_float, pu, pf]
        o.or_gen_matrix.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_long, C.c_long, pf]
        o.or_gen_dists.restype = C.c_int
        o.or_gen_dists.argtypes = [C.c_int, C.c_uint64, C.c_long, C.c_long, C.c_int, C.c_int, pf, C.c_long, C.c_int,
                                   pf]
        o.or_heap_scan.restype = C.c_int
        o.or_heap_scan.argtypes = [pf, C.c_long, C.c_int, pu, pf]
        o.or_bq_search_gen.restype = C.c_int
        o.or_bq_search_gen.argtypes = [C.c_int, C.c_uint64, C.c_long, C.c_long, C.c_int, C.c_int, pf, C.c_long,
                                       C.c_int, C.c_int, C.c_int, pu, pf, pi]
        o.or_rq_search_gen.restype = C.c_int
        o.or_rq_search_gen.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_long, C.c_long, C.c_int, C.c_int, pf,
                                       C.c_long, C.c_int, C.c_int, C.c_int, pu, pf, pi]
        o.or_gen_value.restype = C.c_float
        o.or_gen_value.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64]
        o.bl_set_ref_kernels.argtypes = [C.c_void_p] * 4
        o.bl_set_ref_hamming.argtypes = [C.c_void_p]
        o.bl_flat_search_batch.restype = C.c_int
        o.bl_flat_search_batch.argtypes = [C.c_int, C.c_int, C.c_int, pf, C.c_long, C.c_long, pf, C.c_long, C.c_int,
                                           C.c_int, pu, pf, pi]
        pl = C.POINTER(C.c_long)
        o.or_pcg_stream.argtypes = [C.c_uint64, C.c_uint64, C.c_int, pu]
        o.or_random_subset.argtypes = [C.c_uint64, C.c_long, C.c_int, pl]
        o.or_kmeans_fit.restype = C.c_int
        o.or_kmeans_fit.argtypes = [pf, C.c_long, C.c_long, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int, C.c_int,
                                    C.c_float, C.c_int, pf]
        o.or_pq_encode.argtypes = [pf, C.c_int, C.c_int, C.c_int, C.c_int, pf, pb]
        vp = C.c_void_p
        o.or_rq_new.restype = vp
        o.or_rq_new.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint64]
        o.or_rq_free.argtypes = [vp]
        o.or_rq_out_dim.restype = C.c_int
        o.or_rq_out_dim.argtypes = [vp]
        p16 = C.POINTER(C.c_uint16)
        o.or_rq_tables.argtypes = [vp, p16, p16, pf, pf]
        o.or_fwht64.argtypes = [pf]
        o.or_fwht256.argtypes = [pf]
        o.or_rq_rotate.argtypes = [vp, pf, C.c_long, pf]
        o.or_rq8_encode.argtypes = [vp, C.c_int, pf, C.c_long, pb]
        o.or_rq8_distance.restype = C.c_float
        o.or_rq8_distance.argtypes = [vp, pb, pb]
        o.or_brq_encode.argtypes = [vp, pf, C.c_long, pu]
        o.or_brq_encode_query.argtypes = [vp, pf, C.c_long, pf, pf, pi, pu]
        o.or_brq_distance.restype = C.c_float
        o.or_brq_distance.argtypes = [vp, C.c_float, C.c_float, C.c_int, pu, pu]
        o.or_flat_search_rq.restype = C.c_int
        o.or_flat_search_rq.argtypes = [vp, C.c_int, pf, pb, vp, C.c_long, C.c_long, pf, C.c_long, C.c_int, C.c_int,
                                        pb, C.c_int, pu, pf, pi]
        o.or_rq_query_distances.argtypes = [vp, C.c_int, vp, C.c_long, pf, C.c_long, pf]
        o.or_pq_lut.argtypes = [C.c_int, pf, C.c_int, C.c_int, C.c_int, pf, pf]
        o.or_pq_adc.restype = C.c_float
        o.or_pq_adc.argtypes = [C.c_int, pf, C.c_int, C.c_int, pb]
        o.or_pq_flat_search.restype = C.c_int
        o.or_pq_flat_search.argtypes = [C.c_int, C.c_int, pf, C.c_int, C.c_int, C.c_int, pb, pf, pb, C.c_long, pf,
                                        C.c_int, C.c_int, C.c_int, pu, pf, pi]
        o.bl_pq_search_batch.restype = C.c_int
        o.bl_pq_search_batch.argtypes = [C.c_int, pf, C.c_int, C.c_int, C.c_int, pb, C.c_long, pf, C.c_long, C.c_int,
                                         C.c_int, pu, pf, pi]
        o.bl_flat_search_bq_batch.restype = C.c_int
        o.bl_flat_search_bq_batch.argtypes = [C.c_int, C.c_int, C.c_int, pf, pu, C.c_long, C.c_long, pf, C.c_long,
                                              C.c_int, C.c_int, C.c_int, pu, pf, pi]
        o.or_sq_fit.argtypes = [pf, C.c_long, C.c_long, pf]
        o.or_sq_encode.argtypes = [C.c_float, C.c_float, pf, C.c_long, pb]
        o.or_sq_distance.restype = C.c_float
        o.or_sq_distance.argtypes = [C.c_int, C.c_float, C.c_float, C.c_long, pb, pb]
        o.or_hnsw_flat_search.restype = C.c_int
        o.or_hnsw_flat_search.argtypes = [pf, pf, pb, C.c_long, C.c_int, C.c_int, C.c_int, C.c_int, pu, pf, pi]
        _o = o
    return _o


def ref_lib() -> Optional[C.CDLL]:
    """The reference's compiled kernels, if built (None otherwise)."""
    global _r
    if _r is None and os.path.exists(REF_SO):
        _r = C.CDLL(REF_SO)
    return _r


def host_has_avx512() -> bool:
    try:
        flags = open("/proc/cpuinfo").read()
    except OSError:
        return False
    return " avx512f" in flags and " avx512dq" in flags and " avx512vl" in flags


def f(a):
    return a.ctypes.data_as(pf)


def single_dist(metric: int, variant: int, a: np.ndarray, b: np.ndarray) -> float:
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    return lib().or_single_dist(metric, variant, f(a), f(b), a.size)


def ref_kernel(name: str, a: np.ndarray, b: np.ndarray) -> float:
    """Call one of the reference's compiled kernels (l2_256, dot_512, ...)."""
    r = ref_lib()
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    res = C.c_float()
    n = C.c_long(a.size)
    getattr(r, name)(f(a), f(b), C.byref(res), C.byref(n))
    return res.value


def normalize(v: np.ndarray) -> np.ndarray:
    v = np.ascontiguousarray(v, dtype=np.float32)
    out = np.zeros_like(v)
    lib().or_normalize(f(v), f(out), v.size)
    return out


def bq_encode(v: np.ndarray) -> np.ndarray:
    v = np.ascontiguousarray(v, dtype=np.float32)
    out = np.zeros((v.size + 63) // 64, dtype=np.uint64)
    lib().or_bq_encode(f(v), v.size, out.ctypes.data_as(pu))
    return out


def hamming_bitwise(a: np.ndarray, b: np.ndarray) -> float:
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    return lib().or_hamming_bitwise(a.ctypes.data_as(pu), b.ctypes.data_as(pu), a.size)


class OracleFlat:
    """Oracle flat index: id-indexed store, vectors normalised at Add for cosine
    (flat/index.go:371), scanned in ascending id order."""

    def __init__(self, metric: int, variant: int, d: int, nslots: int):
        self.metric, self.variant, self.d = metric, variant, d
        self.store = np.zeros((nslots, d), dtype=np.float32)
        self.present = np.zeros(nslots, dtype=np.uint8)

    def add_batch(self, ids, vecs):
        vecs = np.asarray(vecs, dtype=np.float32)
        for i, v in zip(ids, vecs):
            self.store[int(i)] = normalize(v) if self.metric == COSINE else v
            self.present[int(i)] = 1

    def delete(self, ids):
        for i in ids:
            self.present[int(i)] = 0

    def search(self, query, k, allow=None):
        """-> (rc, ids, dists); allow: iterable of ids or None."""
        q = np.ascontiguousarray(query, dtype=np.float32)
        ids = np.zeros(max(k, 1), dtype=np.uint64)
        dd = np.zeros(max(k, 1), dtype=np.float32)
        n = C.c_int(0)
        allow_bm = None
        allow_empty = 0
        if allow is not None:
            allow_bm = np.zeros(len(self.present), dtype=np.uint8)
            a = [int(x) for x in allow if int(x) < len(self.present)]
            allow_bm[a] = 1
            allow_empty = 1 if len(list(allow)) == 0 else 0
        rc = lib().or_flat_search(self.metric, self.variant, f(self.store), self.present.ctypes.data_as(pb),
                                  len(self.present), self.d, f(q), q.size, k,
                                  allow_bm.ctypes.data_as(pb) if allow_bm is not None else None, allow_empty,
                                  ids.ctypes.data_as(pu), f(dd), C.byref(n))
        return rc, ids[: n.value].copy(), dd[: n.value].copy()


class OracleFlatBQ(OracleFlat):
    """Oracle flat index with BQ compression (flat/index.go:460-532): codes of the
    stored (normalised) rows, R-heap by hamming, rescoring in pop order."""

    def __init__(self, metric: int, variant: int, d: int, nslots: int, rescore_limit: int = -1):
        super().__init__(metric, variant, d, nslots)
        self.rescore_limit = rescore_limit
        self.codes = np.zeros((nslots, (d + 63) // 64), dtype=np.uint64)

    def add_batch(self, ids, vecs):
        super().add_batch(ids, vecs)
        for i in ids:
            self.codes[int(i)] = bq_encode(self.store[int(i)])

    def search(self, query, k, allow=None):
        q = np.ascontiguousarray(query, dtype=np.float32)
        ids = np.zeros(max(k, 1), dtype=np.uint64)
        dd = np.zeros(max(k, 1), dtype=np.float32)
        n = C.c_int(0)
        allow_bm = None
        allow_empty = 0
        if allow is not None:
            allow_bm = np.zeros(len(self.present), dtype=np.uint8)
            a = [int(x) for x in allow if int(x) < len(self.present)]
            allow_bm[a] = 1
            allow_empty = 1 if len(list(allow)) == 0 else 0
        rc = lib().or_flat_search_bq(self.metric, self.variant, f(self.store), self.present.ctypes.data_as(pb),
                                     self.present.ctypes.data_as(pb), self.codes.ctypes.data_as(pu),
                                     len(self.present), self.d, f(q), q.size, k, self.rescore_limit,
                                     allow_bm.ctypes.data_as(pb) if allow_bm is not None else None, allow_empty,
                                     ids.ctypes.data_as(pu), f(dd), C.byref(n))
        return rc, ids[: n.value].copy(), dd[: n.value].copy()


def cpu_baseline_bq(metric: int, variant: int, store: np.ndarray, codes: np.ndarray, queries: np.ndarray, k: int,
                    rescore_limit: int, nthreads: int, use_ref: bool):
    """Multi-threaded CPU BQ flat search (oracle/baseline.c): hamming R-heap over
    the codes, pop, fp32 rescoring, k-heap.  store/queries normalised for cosine."""
    o = lib()
    if use_ref:
        r = ref_lib()
        if r is None:
            raise RuntimeError("oracle/_ref/libref.so not built")
        o.bl_set_ref_kernels(C.cast(r.l2_256, C.c_void_p), C.cast(r.l2_512, C.c_void_p),
                             C.cast(r.dot_256, C.c_void_p), C.cast(r.dot_512, C.c_void_p))
        o.bl_set_ref_hamming(C.cast(r.hamming_bitwise_256, C.c_void_p))
    store = np.ascontiguousarray(store, dtype=np.float32)
    codes = np.ascontiguousarray(codes, dtype=np.uint64)
    queries = np.ascontiguousarray(queries, dtype=np.float32)
    nq = queries.shape[0]
    ids = np.zeros((nq, k), dtype=np.uint64)
    dd = np.zeros((nq, k), dtype=np.float32)
    cnt = np.zeros(nq, dtype=np.int32)
    rc = o.bl_flat_search_bq_batch(metric, variant, 1 if use_ref else 0, f(store), codes.ctypes.data_as(pu),
                                   store.shape[0], store.shape[1], f(queries), nq, k, rescore_limit, nthreads,
                                   ids.ctypes.data_as(pu), f(dd), cnt.ctypes.data_as(pi))
    if rc != 0:
        raise RuntimeError("baseline failed")
    return ids, dd, cnt


# ---- product quantizer (oracle/pq.c) ----
def pcg_stream(s1: int, s2: int, cnt: int) -> np.ndarray:
    out = np.zeros(cnt, dtype=np.uint64)
    lib().or_pcg_stream(s1, s2, cnt, out.ctypes.data_as(pu))
    return out


def random_subset(seed: int, n: int, k: int) -> np.ndarray:
    out = np.zeros(k, dtype=np.int64)
    lib().or_random_subset(seed, n, k, out.ctypes.data_as(C.POINTER(C.c_long)))
    return out


def pq_fit(data: np.ndarray, m: int, ks: int, seed: int, variant: int = AVX256, iterations: int = 10,
           delta: float = 0.01, brute_force: bool = False, nthreads: int = 1) -> np.ndarray:
    """ProductQuantizer.Fit with the KMeans encoder; segment s seeded seed+s
    (the segments are independent problems: nthreads fit them concurrently,
    as the reference's Fit does).  Returns centers [m][ks][ds]."""
    data = np.ascontiguousarray(data, dtype=np.float32)
    n, d = data.shape
    ds = d // m
    out = np.zeros((m, ks, ds), dtype=np.float32)

    def one(s):
        return lib().or_kmeans_fit(f(data), n, d, s, ds, ks, (seed + s) & (2**64 - 1), variant, iterations, delta,
                                   1 if brute_force else 0, f(out[s]))
    if nthreads > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(nthreads) as ex:
            rcs = list(ex.map(one, range(m)))
    else:
        rcs = [one(s) for s in range(m)]
    if min(rcs) < 0:
        raise ValueError("not enough data to fit k-means")
    return out


def pq_encode(centers: np.ndarray, vec: np.ndarray, variant: int = AVX256) -> np.ndarray:
    m, ks, ds = centers.shape
    c = np.ascontiguousarray(centers, dtype=np.float32)
    v = np.ascontiguousarray(vec, dtype=np.float32)
    out = np.zeros(m, dtype=np.uint8)
    lib().or_pq_encode(f(c), m, ks, ds, variant, f(v), out.ctypes.data_as(pb))
    return out


def pq_distance(metric: int, centers: np.ndarray, query: np.ndarray, code: np.ndarray) -> float:
    m, ks, ds = centers.shape
    c = np.ascontiguousarray(centers, dtype=np.float32)
    lut = np.zeros((m, ks), dtype=np.float32)
    lib().or_pq_lut(metric, f(c), m, ks, ds, f(np.ascontiguousarray(query, dtype=np.float32)), f(lut))
    return lib().or_pq_adc(metric, f(lut), m, ks, np.ascontiguousarray(code, dtype=np.uint8).ctypes.data_as(pb))


def pq_flat_search(metric: int, variant: int, centers: np.ndarray, codes: np.ndarray, store: np.ndarray,
                   present: np.ndarray, query: np.ndarray, k: int, limit: int, rescore: bool):
    """hnsw.flatSearch (one worker) over PQ codes (+ h.rescore).  query/store
    normalised already for cosine."""
    m, ks, ds = centers.shape
    ids = np.zeros(max(k, limit, 1) + 1, dtype=np.uint64)
    dd = np.zeros(max(k, limit, 1) + 1, dtype=np.float32)
    n = C.c_int(0)
    lib().or_pq_flat_search(metric, variant, f(np.ascontiguousarray(centers, np.float32)), m, ks, ds,
                            np.ascontiguousarray(codes, np.uint8).ctypes.data_as(pb),
                            f(np.ascontiguousarray(store, np.float32)),
                            np.ascontiguousarray(present, np.uint8).ctypes.data_as(pb), len(present),
                            f(np.ascontiguousarray(query, np.float32)), k, limit, 1 if rescore else 0,
                            ids.ctypes.data_as(pu), f(dd), C.byref(n))
    return ids[: n.value].copy(), dd[: n.value].copy()


def cpu_baseline_pq(metric: int, centers: np.ndarray, codes: np.ndarray, queries: np.ndarray, k: int, nthreads: int):
    """Threaded CPU PQ flat search (oracle/baseline.c): LUT + ADC + heap per query."""
    m, ks, ds = centers.shape
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    queries = np.ascontiguousarray(queries, dtype=np.float32)
    nq = queries.shape[0]
    ids = np.zeros((nq, k), dtype=np.uint64)
    dd = np.zeros((nq, k), dtype=np.float32)
    cnt = np.zeros(nq, dtype=np.int32)
    lib().bl_pq_search_batch(metric, f(np.ascontiguousarray(centers, np.float32)), m, ks, ds, codes.ctypes.data_as(pb),
                             codes.shape[0], f(queries), nq, k, nthreads, ids.ctypes.data_as(pu), f(dd),
                             cnt.ctypes.data_as(pi))
    return ids, dd, cnt


DEFAULT_FAST_ROTATION_SEED = 0x535AB5105169B1DF  # compressionhelpers/fast_rotation.go:27


class RQ:
    """Rotational quantizer restatement (oracle/rq.c): bits 8 = RotationalQuantizer
    (rotational_quantization.go), bits 1 = BinaryRotationalQuantizer
    (binary_rotational_quantization.go), with flat's seed and rounds."""

    def __init__(self, bits: int, metric: int, dims: int, seed: int = DEFAULT_FAST_ROTATION_SEED):
        self.bits, self.metric, self.dims = bits, metric, dims
        self.h = lib().or_rq_new(bits, metric, dims, seed)
        if not self.h:
            raise ValueError("unsupported rq configuration")
        self.D = lib().or_rq_out_dim(self.h)
        self.W = self.D // 64
        self.code_len = (16 + self.D) if bits == 8 else (1 + self.W)  # bytes / u64 words

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_rq_free(self.h)
            self.h = None

    def tables(self):
        sI = np.zeros((3, self.D // 2), np.uint16)
        sJ = np.zeros((3, self.D // 2), np.uint16)
        sg = np.zeros((3, self.D), np.float32)
        rd = np.zeros(self.D, np.float32)
        p16 = C.POINTER(C.c_uint16)
        lib().or_rq_tables(self.h, sI.ctypes.data_as(p16), sJ.ctypes.data_as(p16), f(sg), f(rd))
        return sI, sJ, sg, rd

    def rotate(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.float32)
        out = np.zeros(self.D, np.float32)
        lib().or_rq_rotate(self.h, f(x), x.size, f(out))
        return out

    def encode(self, x: np.ndarray, variant: int = AVX256) -> np.ndarray:
        """rq-8: RQCode bytes [16 + D]; rq-1: RQOneBitCode words [1 + D/64]"""
        x = np.ascontiguousarray(x, np.float32)
        if self.bits == 8:
            out = np.zeros(self.code_len, np.uint8)
            lib().or_rq8_encode(self.h, variant, f(x), x.size, out.ctypes.data_as(pb))
        else:
            out = np.zeros(self.code_len, np.uint64)
            lib().or_brq_encode(self.h, f(x), x.size, out.ctypes.data_as(pu))
        return out

    def encode_query(self, x: np.ndarray):
        """rq-1 encodeQuery -> (step, squared norm, dim, planes [5][W])"""
        x = np.ascontiguousarray(x, np.float32)
        planes = np.zeros((5, self.W), np.uint64)
        st, sq, dim = C.c_float(0), C.c_float(0), C.c_int(0)
        lib().or_brq_encode_query(self.h, f(x), x.size, C.byref(st), C.byref(sq), C.byref(dim),
                                  planes.ctypes.data_as(pu))
        return st.value, sq.value, dim.value, planes

    def distance(self, cx: np.ndarray, query) -> float:
        """rq-8: DistanceBetweenCompressedVectors(cx, cy=query code);
        rq-1: BinaryRQDistancer.Distance(cx) with query = encode_query(...)"""
        if self.bits == 8:
            return lib().or_rq8_distance(self.h, np.ascontiguousarray(cx, np.uint8).ctypes.data_as(pb),
                                         np.ascontiguousarray(query, np.uint8).ctypes.data_as(pb))
        st, sq, dim, planes = query
        return lib().or_brq_distance(self.h, st, sq, dim, np.ascontiguousarray(planes, np.uint64).ctypes.data_as(pu),
                                     np.ascontiguousarray(cx, np.uint64).ctypes.data_as(pu))


class OracleFlatRQ(OracleFlat):
    """Oracle flat index with rq-8 / rq-1 compression (flat/index.go:338-360 creates
    the quantizer at the first Add; :460-532 searches)."""

    def __init__(self, bits: int, metric: int, variant: int, d: int, nslots: int, rescore_limit: int = -1):
        super().__init__(metric, variant, d, nslots)
        self.rescore_limit = rescore_limit
        self.rq = RQ(bits, metric, d)
        dt = np.uint8 if bits == 8 else np.uint64
        self.codes = np.zeros((nslots, self.rq.code_len), dtype=dt)

    def add_batch(self, ids, vecs):
        super().add_batch(ids, vecs)
        for i in ids:
            self.codes[int(i)] = self.rq.encode(self.store[int(i)], self.variant)

    def query_distances(self, query) -> np.ndarray:
        q = np.ascontiguousarray(query, dtype=np.float32)
        out = np.zeros(len(self.present), np.float32)
        lib().or_rq_query_distances(self.rq.h, self.variant, self.codes.ctypes.data, len(self.present), f(q), q.size,
                                    f(out))
        return out

    def search(self, query, k, allow=None):
        q = np.ascontiguousarray(query, dtype=np.float32)
        ids = np.zeros(max(k, 1), dtype=np.uint64)
        dd = np.zeros(max(k, 1), dtype=np.float32)
        n = C.c_int(0)
        allow_bm = None
        allow_empty = 0
        if allow is not None:
            allow_bm = np.zeros(len(self.present), dtype=np.uint8)
            a = [int(x) for x in allow if int(x) < len(self.present)]
            allow_bm[a] = 1
            allow_empty = 1 if len(list(allow)) == 0 else 0
        rc = lib().or_flat_search_rq(self.rq.h, self.variant, f(self.store), self.present.ctypes.data_as(pb),
                                     self.codes.ctypes.data, len(self.present), self.d, f(q), q.size, k,
                                     self.rescore_limit, allow_bm.ctypes.data_as(pb) if allow_bm is not None else None,
                                     allow_empty, ids.ctypes.data_as(pu), f(dd), C.byref(n))
        return rc, ids[: n.value].copy(), dd[: n.value].copy()


def gen_matrix(kind: int, seed: int, row0: int, rows: int, d: int) -> np.ndarray:
    out = np.zeros((rows, d), dtype=np.float32)
    lib().or_gen_matrix(kind, seed, row0, rows, d, f(out))
    return out


def cpu_baseline(metric: int, variant: int, store: np.ndarray, queries: np.ndarray, k: int, nthreads: int,
                 use_ref: bool):
    """Multi-threaded CPU scan (oracle/baseline.c).  queries must be
    normalised already for cosine.  Returns (ids, dists, counts)."""
    o = lib()
    if use_ref:
        r = ref_lib()
        if r is None:
            raise RuntimeError("oracle/_ref/libref.so not built")
        o.bl_set_ref_kernels(C.cast(r.l2_256, C.c_void_p), C.cast(r.l2_512, C.c_void_p),
                             C.cast(r.dot_256, C.c_void_p), C.cast(r.dot_512, C.c_void_p))
    store = np.ascontiguousarray(store, dtype=np.float32)
    queries = np.ascontiguousarray(queries, dtype=np.float32)
    nq = queries.shape[0]
    ids = np.zeros((nq, k), dtype=np.uint64)
    dd = np.zeros((nq, k), dtype=np.float32)
    cnt = np.zeros(nq, dtype=np.int32)
    rc = o.bl_flat_search_batch(metric, variant, 1 if use_ref else 0, f(store), store.shape[0], store.shape[1],
                                f(queries), nq, k, nthreads, ids.ctypes.data_as(pu), f(dd), cnt.ctypes.data_as(pi))
    if rc != 0:
        raise RuntimeError("baseline failed")
    return ids, dd, cnt


# ---------------------------------------------------------------------------
# full-size oracles over the regenerated corpus (oracle/scale.c)
# ---------------------------------------------------------------------------
def gen_dists(kind: int, seed: int, n: int, d: int, metric: int, variant: int, queries: np.ndarray,
              nthreads: int = 16) -> np.ndarray:
    """SingleDist of each prepared query (normalised for cosine) to rows [0, n)
    of the generated corpus, rows prepared as flat.Add does.  [nq][n] float32."""
    q = np.ascontiguousarray(queries, dtype=np.float32)
    out = np.empty((q.shape[0], n), dtype=np.float32)
    lib().or_gen_dists(kind, seed, n, d, metric, variant, f(q), q.shape[0], nthreads, f(out))
    return out


def heap_scan(dists: np.ndarray, k: int):
    """The reference heap (insertToHeap in id order + extractHeap) over one
    query's precomputed distances of rows [0, n)."""
    dd = np.ascontiguousarray(dists, dtype=np.float32)
    ids = np.zeros(k, np.uint64)
    od = np.zeros(k, np.float32)
    m = lib().or_heap_scan(f(dd), dd.size, k, ids.ctypes.data_as(pu), f(od))
    return ids[:m], od[:m]


def bq_search_gen(kind: int, seed: int, n: int, d: int, metric: int, variant: int, queries: np.ndarray, k: int,
                  rescore_limit: int, nthreads: int = 16):
    """searchByVectorQuantized of raw queries over the generated corpus."""
    q = np.ascontiguousarray(queries, dtype=np.float32)
    nq = q.shape[0]
    ids = np.zeros((nq, k), np.uint64)
    dd = np.zeros((nq, k), np.float32)
    cnt = np.zeros(nq, np.int32)
    rc = lib().or_bq_search_gen(kind, seed, n, d, metric, variant, f(q), nq, k, rescore_limit, nthreads,
                                ids.ctypes.data_as(pu), f(dd), cnt.ctypes.data_as(pi))
    if rc != 0:
        raise RuntimeError("bq_search_gen failed")
    return ids, dd, cnt


def rq_search_gen(bits: int, kind: int, seed: int, n: int, d: int, metric: int, variant: int, queries: np.ndarray,
                  k: int, rescore_limit: int, nthreads: int = 16):
    """flat rq-8 / rq-1 searchByVectorQuantized of raw queries over the
    generated corpus (codes of every row built on the host, oracle/scale.c)."""
    q = np.ascontiguousarray(queries, dtype=np.float32)
    nq = q.shape[0]
    ids = np.zeros((nq, k), np.uint64)
    dd = np.zeros((nq, k), np.float32)
    cnt = np.zeros(nq, np.int32)
    rc = lib().or_rq_search_gen(bits, kind, seed, n, d, metric, variant, f(q), nq, k, rescore_limit, nthreads,
                                ids.ctypes.data_as(pu), f(dd), cnt.ctypes.data_as(pi))
    if rc != 0:
        raise RuntimeError("rq_search_gen failed")
    return ids, dd, cnt


# ---- scalar quantizer (oracle/sq.c) + generic hnsw.flatSearch ----------------
class SQ:
    """compressionhelpers.ScalarQuantizer restated (scalar_quantization.go)."""

    def __init__(self, data=None, a: Optional[float] = None, b: Optional[float] = None, d: Optional[int] = None):
        if data is not None:
            x = np.ascontiguousarray(data, dtype=np.float32)
            ab = np.zeros(2, np.float32)
            lib().or_sq_fit(f(x), x.shape[0], x.shape[1], f(ab))
            self.a, self.b, self.d = float(ab[0]), float(ab[1]), x.shape[1]
        else:
            self.a, self.b, self.d = float(np.float32(a)), float(np.float32(b)), int(d)

    def encode(self, v) -> np.ndarray:
        x = np.ascontiguousarray(v, dtype=np.float32).ravel()
        out = np.zeros(x.size + 8, np.uint8)
        lib().or_sq_encode(self.a, self.b, f(x), x.size, out.ctypes.data_as(pb))
        return out

    def distance(self, metric: int, cx: np.ndarray, cy: np.ndarray) -> float:
        return float(lib().or_sq_distance(metric, self.a, self.b, self.d, np.ascontiguousarray(cx).ctypes.data_as(pb),
                                          np.ascontiguousarray(cy).ctypes.data_as(pb)))


def hnsw_flat_search(cdist: np.ndarray, edist: np.ndarray, present: np.ndarray, k: int, limit: int, rescore: bool,
                     trim: int):
    """hnsw.flatSearch (one worker) + h.rescore over precomputed compressor
    distances cdist[slot] and rescoring distances edist[slot] -> (ids, dists)."""
    cd = np.ascontiguousarray(cdist, dtype=np.float32)
    ed = np.ascontiguousarray(edist, dtype=np.float32)
    pr = np.ascontiguousarray(present, dtype=np.uint8)
    ids = np.zeros(max(k, 1), np.uint64)
    dd = np.zeros(max(k, 1), np.float32)
    n = C.c_int(0)
    lib().or_hnsw_flat_search(f(cd), f(ed), pr.ctypes.data_as(pb), cd.size, int(k), int(limit), int(bool(rescore)),
                              int(trim), ids.ctypes.data_as(pu), f(dd), C.byref(n))
    return ids[:n.value].copy(), dd[:n.value].copy()


def search_time_ef(k: int, ef: int = -1, ef_min: int = 100, ef_max: int = 500, ef_factor: int = 8) -> int:
    """hnsw searchTimeEF / autoEfFromK (hnsw/search.go:44-76)."""
    if ef < 1:
        e = k * ef_factor
        e = ef_max if e > ef_max else ef_min if e < ef_min else e
        return max(e, k)
    return max(ef, k)
