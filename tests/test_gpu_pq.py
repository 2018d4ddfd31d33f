"""GPU parity of the product quantizer and the PQ brute-force search vs the
oracle (oracle/pq.c): k-means codebooks, codes, ADC distances and search
results bit-exact for the same PCG seed.  MI355X only (marker gpu)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VARIANTS = {"avx256": 1, "avx512": 2}


def gen(oracle, kind, seed, rows, d):
    return oracle.gen_matrix(kind, seed, 0, rows, d)


def stored_rows(oracle, metric, data):
    if metric == oracle.COSINE:
        return np.stack([oracle.normalize(x) for x in data])
    return data.copy()


@pytest.mark.parametrize("metric,kind,n,d,m,ks,limit,variant", [
    ("l2-squared", 0, 3000, 32, 8, 64, 100000, "avx256"),   # ds = 4 (scalar SingleDist path)
    ("cosine", 0, 4000, 64, 8, 256, 100000, "avx256"),      # ds = 8 (SIMD path), ks = 256
    ("dot", 0, 2500, 60, 15, 32, 2000, "avx512"),           # ds = 4, training limit < n
    ("l2-squared", 1, 2000, 24, 6, 16, 100000, "avx256"),   # integer data: duplicate points / ties
    ("cosine", 0, 1500, 96, 4, 64, 100000, "avx512"),       # ds = 24
])
def test_pq_fit_codes_distance_match_oracle(wv, oracle, metric, kind, n, d, m, ks, limit, variant):
    data = gen(oracle, kind, 61, n, d)
    idx = wv.FlatIndex(distance=metric, variant=variant,
                       pq={"segments": m, "centroids": ks, "trainingLimit": limit, "rescore": True})
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    idx.pq_fit(seed=1234)
    assert idx.compressed()
    got = idx.pq_centers()
    om = oracle.METRIC[metric]
    store = stored_rows(oracle, om, data)
    exp = oracle.pq_fit(store[:min(n, limit)], m, ks, seed=1234, variant=VARIANTS[variant])
    np.testing.assert_array_equal(got.view(np.uint32), exp.view(np.uint32))
    codes = idx.pq_codes(n)
    ecodes = np.stack([oracle.pq_encode(exp, x, VARIANTS[variant]) for x in store])
    np.testing.assert_array_equal(codes, ecodes)
    q = gen(oracle, kind, 62, 1, d)[0]
    gd = idx.pq_distance(q, codes[:500])
    ed = np.array([oracle.pq_distance(om, exp, q, c) for c in codes[:500]], np.float32)
    np.testing.assert_array_equal(gd.view(np.uint32), ed.view(np.uint32))
    idx.close()


@pytest.mark.parametrize("metric,kind,rescore,k,rl", [
    ("l2-squared", 0, True, 10, 64),
    ("cosine", 0, True, 10, 100),
    ("dot", 0, False, 10, -1),
    ("l2-squared", 1, True, 7, 40),     # integer data: ADC ties -> heap order
    ("l2-squared", 1, False, 20, -1),
    ("cosine", 0, True, 10, 40),        # worker heap limit 40: the candidate path with rescoring
])
# cand 1: block minima + candidate blocks + exact ADC of their rows (k_pq_cand; ties flagged
# to the replay), cand 0: the full ADC matrix + replay; adc 2: k_pq_adc2 (odd list: one
# single-query block), adc 1: k_pq_adc
@pytest.mark.parametrize("adc,nq,cand", [(2, 16, 1), (2, 15, 1), (2, 16, 0), (1, 16, 0)])
def test_pq_search_matches_oracle(wv, oracle, metric, kind, rescore, k, rl, adc, nq, cand):
    n, d, m, ks = 5000, 32, 8, 32
    data = gen(oracle, kind, 71, n, d)
    idx = wv.FlatIndex(distance=metric, variant="avx256", rescore_limit=rl,
                       pq={"segments": m, "centroids": ks, "rescore": rescore})
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    idx.pq_fit(seed=77)
    idx.set_option("pq_adc", adc)
    idx.set_option("pq_cand", cand)
    centers = idx.pq_centers()
    codes = idx.pq_codes(n)
    om = oracle.METRIC[metric]
    store = stored_rows(oracle, om, data)
    present = np.ones(n, np.uint8)
    queries = gen(oracle, kind, 72, nq, d)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    for qi in range(len(queries)):
        qv = oracle.normalize(queries[qi]) if om == oracle.COSINE else queries[qi]
        oi, od = oracle.pq_flat_search(om, 1, centers, codes, store, present, qv, k, max(rl, k), rescore)
        np.testing.assert_array_equal(ids[qi, :counts[qi]], oi, err_msg=f"q{qi}")
        np.testing.assert_array_equal(dists[qi, :counts[qi]].view(np.uint32), od.view(np.uint32), err_msg=f"q{qi}")
    idx.close()


def test_pq_add_after_fit_and_set_centers(wv, oracle):
    n, d, m, ks = 2000, 16, 4, 16
    data = gen(oracle, 0, 81, n, d)
    a = wv.FlatIndex(distance="l2-squared", pq={"segments": m, "centroids": ks})
    a.add_batch(np.arange(n, dtype=np.uint64), data)
    a.pq_fit(seed=5)
    more = gen(oracle, 0, 82, 300, d)
    a.add_batch(np.arange(n, n + 300, dtype=np.uint64), more)  # encoded on Add
    c = a.pq_centers()
    exp = np.stack([oracle.pq_encode(c, x) for x in more])
    np.testing.assert_array_equal(a.pq_codes(n + 300)[n:], exp)
    b = wv.FlatIndex(distance="l2-squared", pq={"segments": m, "centroids": ks})
    b.add_batch(np.arange(n + 300, dtype=np.uint64), np.concatenate([data, more]))
    b.pq_set_centers(c)  # NewProductQuantizerWithEncoders
    np.testing.assert_array_equal(b.pq_codes(n + 300), a.pq_codes(n + 300))
    q = gen(oracle, 0, 83, 4, d)
    for x, y in zip(a.search_by_vector_batch(q, 10), b.search_by_vector_batch(q, 10)):
        np.testing.assert_array_equal(x, y)
    a.close()
    b.close()


def test_pq_errors(wv, oracle):
    data = gen(oracle, 0, 91, 100, 30)
    idx = wv.FlatIndex(distance="l2-squared", pq={"segments": 7, "centroids": 16})
    idx.add_batch(np.arange(100, dtype=np.uint64), data)
    with pytest.raises(wv.WeaviateError, match="segments should be an integer divisor of dimensions"):
        idx.pq_fit()
    idx.close()
    idx = wv.FlatIndex(distance="l2-squared", pq={"segments": 5, "centroids": 300})
    idx.add_batch(np.arange(100, dtype=np.uint64), data)
    with pytest.raises(wv.WeaviateError, match="centroids should not be higher than 256"):
        idx.pq_fit()
    idx.close()
    idx = wv.FlatIndex(distance="l2-squared", pq={"segments": 5, "centroids": 256})
    idx.add_batch(np.arange(100, dtype=np.uint64), data)
    with pytest.raises(wv.WeaviateError, match="not enough data to fit k-means"):
        idx.pq_fit()
    # before Fit the index searches uncompressed
    ids, _ = idx.search_by_vector(data[3], 1)
    assert ids[0] == 3
    idx.close()


# k_pq_adc3 (ks = 256 only: queries on the lanes, 1024-row chunks, 64-query groups): a row
# count off the chunk size, m off the 16-segment group, two query groups (the second
# partial), deleted rows and an allow list (invalid rows), integer data (ADC ties); the
# same results as k_pq_adc2 and the oracle; k_pq_adc4 (pq_adc3 = 2, 16-byte LUT reads) too
@pytest.mark.parametrize("metric,kind,rescore,k,rl,allow", [
    ("l2-squared", 0, False, 10, -1, False),
    ("cosine", 0, True, 10, 40, False),
    ("dot", 0, False, 12, -1, True),
    ("l2-squared", 1, False, 20, -1, False),
])
def test_pq_adc3_matches_adc2_and_oracle(wv, oracle, metric, kind, rescore, k, rl, allow):
    n, d, m, ks, nq = 3171, 96, 24, 256, 70
    data = gen(oracle, kind, 171, n, d)
    idx = wv.FlatIndex(distance=metric, variant="avx256", rescore_limit=rl,
                       pq={"segments": m, "centroids": ks, "rescore": rescore})
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    idx.pq_fit(seed=17)
    gone = list(range(5, n, 97))
    idx.delete(*gone)
    centers = idx.pq_centers()
    codes = idx.pq_codes(n)
    om = oracle.METRIC[metric]
    store = stored_rows(oracle, om, data)
    present = np.ones(n, np.uint8)
    present[gone] = 0
    al = None
    if allow:
        keep = [i for i in range(n) if i % 3 != 1]
        al = wv.AllowList(keep)
        mask = np.zeros(n, np.uint8)
        mask[keep] = 1
        present &= mask
    queries = gen(oracle, kind, 172, nq, d)
    res = {}
    for adc3 in (1, 0, 2):
        idx.set_option("pq_adc3", adc3)
        res[adc3] = idx.search_by_vector_batch(queries, k, allow=al)
    for alt in (0, 2):
        for a, b in zip(res[1], res[alt]):
            np.testing.assert_array_equal(np.asarray(a), np.asarray(b), err_msg=f"pq_adc3={alt}")
    ids, dists, counts = res[1]
    for qi in list(range(0, nq, 7)) + [63, 64, nq - 1]:
        qv = oracle.normalize(queries[qi]) if om == oracle.COSINE else queries[qi]
        oi, od = oracle.pq_flat_search(om, 1, centers, codes, store, present, qv, k, max(rl, k), rescore)
        np.testing.assert_array_equal(ids[qi, :counts[qi]], oi, err_msg=f"q{qi}")
        np.testing.assert_array_equal(dists[qi, :counts[qi]].view(np.uint32), od.view(np.uint32), err_msg=f"q{qi}")
    idx.close()


# PQ block keys on the integer matrix cores (option pq8, l2-squared, 384 < d <= 1536):
# keys over the centred int8 reconstruction plane, candidate 32-row blocks, exact ADC of
# their rows (k_pq_cand8); must equal the LUT-minima route (pq8 = 0) and the oracle bit
# for bit -- with deleted rows, an allow list, integer data (ADC ties -> flagged ->
# replay), rows added after the fit (a dirty block range rebuilt at the next search) and
# a capacity growth (the plane reallocated)
@pytest.mark.parametrize("kind,n,d,m,ks,rescore,k,rl,allow", [
    (2, 9000, 960, 240, 256, False, 10, -1, False),   # the C5 shape (GIST-like U[0,1))
    (2, 6000, 400, 100, 64, True, 10, 100, True),     # rescoring: worker heap 100
    (1, 5000, 768, 192, 32, False, 20, -1, False),    # integer data: ADC ties
    (0, 7000, 1024, 128, 256, False, 5, -1, True),    # ds = 8
])
def test_pq8_keys_match_lut_route_and_oracle(wv, oracle, kind, n, d, m, ks, rescore, k, rl, allow):
    data = gen(oracle, kind, 181, n, d)
    idx = wv.FlatIndex(distance="l2-squared", variant="avx256", rescore_limit=rl,
                       pq={"segments": m, "centroids": ks, "rescore": rescore})
    idx.add_batch(np.arange(n - 500, dtype=np.uint64), data[: n - 500])
    idx.pq_fit(seed=19)
    gone = list(range(3, n - 500, 89))
    idx.delete(*gone)
    queries = gen(oracle, kind, 182, 70, d)
    idx.search_by_vector_batch(queries[:3], k)  # builds the plane
    idx.add_batch(np.arange(n - 500, n, dtype=np.uint64), data[n - 500:])  # encoded on Add: dirty blocks
    idx.add_batch(np.arange(40, 48, dtype=np.uint64), data[n - 8:])  # upserts inside built blocks
    store = data.copy()
    store[40:48] = data[n - 8:]
    present = np.ones(n, np.uint8)
    present[gone] = 0
    al = None
    if allow:
        keep = [i for i in range(n) if i % 4 != 1]
        al = wv.AllowList(keep)
        mask = np.zeros(n, np.uint8)
        mask[keep] = 1
        present &= mask
    res = {}
    for opt in (1, 0):
        idx.set_option("pq8", opt)
        res[opt] = idx.search_by_vector_batch(queries, k, allow=al)
        if opt == 1:
            assert idx.stats()["last_route"] == 8  # WV_ROUTE_PQ_INT8
    for a, b in zip(res[1], res[0]):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b))
    centers = idx.pq_centers()
    codes = idx.pq_codes(n)
    ids, dists, counts = res[1]
    for qi in range(0, len(queries), 6):
        oi, od = oracle.pq_flat_search(oracle.L2, 1, centers, codes, store, present, queries[qi], k, max(rl, k),
                                       rescore)
        np.testing.assert_array_equal(ids[qi, :counts[qi]], oi, err_msg=f"q{qi}")
        np.testing.assert_array_equal(dists[qi, :counts[qi]].view(np.uint32), od.view(np.uint32), err_msg=f"q{qi}")
    # growth: the plane follows the index capacity
    idx.set_option("pq8", 1)
    idx.reserve(4 * n)
    for a, b in zip(idx.search_by_vector_batch(queries, k, allow=al), res[0]):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b))
    idx.close()
