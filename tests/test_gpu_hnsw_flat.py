"""GPU parity for hnsw.flatSearch + h.rescore over HNSW's compressor
distancers (hnsw/flat_search.go:28-141, hnsw/search.go:1047-1110,
compressionhelpers BQ / SQ / RQ / PQ): wv_index_hnsw_flat_search against the
oracle's generic restatement (oracle/sq.c or_hnsw_flat_search) fed with the
oracle's own compressor and SingleDist distances, bit-exact ids and distances.
The SQ quantizer (scalar_quantization.go) is also checked code by code.
MI355X only (marker gpu)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VARIANTS = {"avx256": 1, "avx512": 2}


def gen(oracle, kind, seed, rows, d):
    return oracle.gen_matrix(kind, seed, 0, rows, d)


def bits_equal(a, b, msg=""):
    np.testing.assert_array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32),
                                  err_msg=msg)


def store_of(oracle, metric, data):
    return np.stack([oracle.normalize(x) for x in data]) if metric == oracle.COSINE else data.copy()


def make(wv, oracle, comp, metric, variant, data, rescore_limit=-1, sq_limit=0):
    n, d = data.shape
    kw = dict(distance=metric, variant=variant, rescore_limit=rescore_limit)
    if comp == "bq":
        kw["bq"] = True
    elif comp == "sq":
        kw["sq"] = True
    elif comp in ("rq8", "rq1"):
        kw["rq"] = {"bits": 8 if comp == "rq8" else 1}
    elif comp == "pq":
        kw["pq"] = {"segments": d // 4, "centroids": 32, "trainingLimit": 100000, "rescore": True}
    idx = wv.FlatIndex(**kw)
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    if comp == "sq":
        idx.sq_fit(sq_limit)
    elif comp == "pq":
        idx.pq_fit(seed=9)
    return idx


def compressor_distances(oracle, comp, metric, variant, idx, data, q):
    """cdist[slot] of the query (oracle), for every slot."""
    m = oracle.METRIC[metric]
    store = store_of(oracle, m, data)
    qn = oracle.normalize(q) if m == oracle.COSINE else q
    n, d = data.shape
    if comp == "bq":
        cq = oracle.bq_encode(qn)
        return np.array([oracle.hamming_bitwise(cq, oracle.bq_encode(x)) for x in store], np.float32)
    if comp == "sq":
        info = idx.sq_info()
        sq = oracle.SQ(a=info["a"], b=info["b"], d=d)
        cq = sq.encode(qn)
        return np.array([sq.distance(m, cq, sq.encode(x)) for x in store], np.float32)
    if comp in ("rq8", "rq1"):
        orc = oracle.OracleFlatRQ(8 if comp == "rq8" else 1, m, VARIANTS[variant], d, n)
        orc.add_batch(np.arange(n), data)
        return orc.query_distances(q)
    centers = idx.pq_centers()
    codes = np.stack([oracle.pq_encode(centers, x, VARIANTS[variant]) for x in store])
    # PQDistancer: l2 -> L2 steps, dot / cosine -> dot steps + Wrap (pq.c or_pq_lut / or_pq_adc)
    return np.array([oracle.pq_distance(m, centers, qn, c) for c in codes], np.float32)


def exact_distances(oracle, metric, variant, data, q):
    m = oracle.METRIC[metric]
    store = store_of(oracle, m, data)
    qn = oracle.normalize(q) if m == oracle.COSINE else q
    return np.array([oracle.single_dist(m, VARIANTS[variant], x, qn) for x in store], np.float32)


def expected(oracle, comp, cd, ed, present, k, rescore_limit, ef=-1, rescore_on=True):
    sqrq = comp in ("sq", "rq8", "rq1")
    rescore = rescore_on and not (sqrq and rescore_limit == 0)
    limit = oracle.search_time_ef(k, ef) if rescore else k
    trim = rescore_limit if (sqrq and rescore_limit >= k) else 0
    return oracle.hnsw_flat_search(cd, ed, present, k, limit, rescore, trim)


@pytest.mark.parametrize("comp", ["bq", "sq", "rq8", "rq1", "pq"])
@pytest.mark.parametrize("metric,variant,kind", [("cosine", "avx256", 0), ("l2-squared", "avx512", 1),
                                                 ("dot", "avx256", 0)])
def test_hnsw_flat_search_equals_oracle(wv, oracle, comp, metric, variant, kind):
    n, d, k = 3000, 64, 10
    data = gen(oracle, kind, 41, n, d)
    queries = gen(oracle, kind, 42, 6, d)
    rl = 20 if comp in ("sq", "rq8", "rq1") else -1
    idx = make(wv, oracle, comp, metric, variant, data, rescore_limit=rl)
    present = np.ones(n, np.uint8)
    for ef in (-1, 16):
        idx.set_option("ef", ef)
        ids, dists, counts = idx.hnsw_flat_search(queries, k)
        for qi, q in enumerate(queries):
            cd = compressor_distances(oracle, comp, metric, variant, idx, data, q)
            ed = exact_distances(oracle, metric, variant, data, q)
            ei, ed_ = expected(oracle, comp, cd, ed, present, k, rl, ef)
            assert counts[qi] == len(ei), (comp, metric, ef, qi)
            np.testing.assert_array_equal(ids[qi, :counts[qi]], ei, err_msg=f"{comp} {metric} ef{ef} q{qi}")
            bits_equal(dists[qi, :counts[qi]], ed_, f"{comp} {metric} ef{ef} q{qi}")
    idx.close()


@pytest.mark.parametrize("comp", ["sq", "rq8", "bq"])
def test_hnsw_flat_rescore_switches_and_allow_list(wv, oracle, comp):
    """doNotRescore (limit = k, compressor distances returned), SQ/RQ rescore
    limit 0 (no rescoring) and trimming (rescore_limit >= k), with an allow
    list (the reason hnsw runs its flat search) and deleted ids."""
    n, d, k = 2500, 48, 8
    data = gen(oracle, 1, 51, n, d)  # integer data: ties in every distance
    queries = gen(oracle, 1, 52, 4, d)
    rng = np.random.default_rng(0)
    allow = np.sort(rng.choice(n, 700, replace=False)).astype(np.uint64)
    for rl, resc in ((12, 1), (0, 1), (-1, 0), (300, 1)):
        idx = make(wv, oracle, comp, "l2-squared", "avx256", data, rescore_limit=rl)
        idx.delete(int(allow[3]), int(allow[10]))
        idx.set_option("hnsw_rescore", resc)
        present = np.zeros(n, np.uint8)
        present[allow.astype(np.int64)] = 1
        present[int(allow[3])] = present[int(allow[10])] = 0
        ids, dists, counts = idx.hnsw_flat_search(queries, k, allow=wv.AllowList(allow.tolist()))
        for qi, q in enumerate(queries):
            cd = compressor_distances(oracle, comp, "l2-squared", "avx256", idx, data, q)
            ed = exact_distances(oracle, "l2-squared", "avx256", data, q)
            ei, ed_ = expected(oracle, comp, cd, ed, present, k, rl, -1, bool(resc))
            np.testing.assert_array_equal(ids[qi, :counts[qi]], ei, err_msg=f"{comp} rl{rl} r{resc} q{qi}")
            bits_equal(dists[qi, :counts[qi]], ed_, f"{comp} rl{rl} r{resc} q{qi}")
        idx.close()


@pytest.mark.parametrize("metric", ["l2-squared", "cosine", "dot"])
@pytest.mark.parametrize("d", [4, 33, 150, 768])
def test_sq_fit_and_codes_bit_exact(wv, oracle, metric, d):
    """NewScalarQuantizer over the first training_limit rows in id order, then
    Encode of every row: (a, b) and every code byte (incl. the big-endian
    tail) equal the oracle's; RestoreScalarQuantizer re-encodes identically."""
    n = 900
    data = gen(oracle, 0, 61, n, d) * np.float32(1.7)
    data[7] = 0
    idx = wv.FlatIndex(distance=metric, variant="avx256", sq=True)
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    idx.sq_fit(500)
    m = oracle.METRIC[metric]
    store = store_of(oracle, m, data)
    sq = oracle.SQ(store[:500])
    info = idx.sq_info()
    assert info["ready"] and info["code_bytes"] == d + 8
    bits_equal([info["a"], info["b"]], [sq.a, sq.b], "a, b")
    np.testing.assert_array_equal(idx.sq_codes(n), np.stack([sq.encode(x) for x in store]))
    # later Adds are encoded on insert; a restored quantizer encodes the same way
    extra = gen(oracle, 0, 62, 50, d)
    idx.add_batch(np.arange(n, n + 50, dtype=np.uint64), extra)
    np.testing.assert_array_equal(idx.sq_codes(n + 50)[n:], np.stack([sq.encode(x) for x in store_of(oracle, m, extra)]))
    idx2 = wv.FlatIndex(distance=metric, variant="avx256", sq=True)
    idx2.add_batch(np.arange(n, dtype=np.uint64), data)
    idx2.sq_restore(info["a"], info["b"])
    np.testing.assert_array_equal(idx2.sq_codes(n), idx.sq_codes(n))
    idx.close()
    idx2.close()


def test_sq_errors(wv, oracle):
    idx = wv.FlatIndex(distance="l2-squared", sq=True)
    with pytest.raises(wv.WeaviateError, match="cannot be executed before inserting some data"):
        idx.sq_fit()
    idx.add_batch(np.arange(10, dtype=np.uint64), gen(oracle, 0, 1, 10, 8))
    with pytest.raises(wv.WeaviateError, match="invalid range value while restoring SQ settings"):
        idx.sq_restore(0.0, 1.0)
    with pytest.raises(wv.WeaviateError, match="quantizer not initialized"):
        idx.hnsw_flat_search(gen(oracle, 0, 2, 1, 8), 3)
    idx.sq_fit()
    with pytest.raises(wv.WeaviateError, match="vector lengths don't match: 17 vs 16"):
        idx.hnsw_flat_search(gen(oracle, 0, 2, 1, 9), 3)
    idx.close()
    h = wv.FlatIndex(distance="hamming", sq=True)
    h.add_batch(np.arange(10, dtype=np.uint64), gen(oracle, 0, 1, 10, 8))
    h.sq_fit()
    with pytest.raises(wv.WeaviateError, match="Distance not supported yet hamming"):
        h.hnsw_flat_search(gen(oracle, 0, 2, 1, 8), 3)
    h.close()
