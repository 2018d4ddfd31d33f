"""CPU: the scalar-quantizer oracle (oracle/sq.c) pinned to the reference's own
tests (compressionhelpers/scalar_quantization_test.go), and the generic
hnsw.flatSearch restatement pinned to the PQ one (oracle/pq.c)."""
import numpy as np
import pytest


def test_sq_encode_known_answer(oracle):  # scalar_quantization_test.go:31-43 Test_NoRaceSQEncode
    sq = oracle.SQ(np.array([[1, 0, 0, 0], [1, 1, 1, 5]], np.float32))
    code = sq.encode(np.array([0.5, 1, 0, 2], np.float32))
    assert list(code[:4]) == [25, 51, 0, 102]
    # the 8-byte tail: big-endian sum and sum of squares of the codes
    assert int.from_bytes(code[4:8].tobytes(), "big") == 25 + 51 + 102
    assert int.from_bytes(code[8:12].tobytes(), "big") == 25 ** 2 + 51 ** 2 + 102 ** 2


@pytest.mark.parametrize("metric", ["l2-squared", "cosine", "dot"])
def test_sq_distance_close_to_float(oracle, metric):  # :45-61 Test_NoRaceSQDistance
    m = oracle.METRIC[metric]
    sq = oracle.SQ(np.array([[1, 0, 0, 0], [1, 1, 1, 5]], np.float32))
    v1 = np.array([0.217, 0.435, 0, 0.348], np.float32)
    v2 = np.array([0.241, 0.202, 0.257, 0.300], np.float32)
    dist = sq.distance(m, sq.encode(v1), sq.encode(v2))
    expected = oracle.single_dist(m, oracle.AVX256, v1, v2)
    assert abs(expected - dist) < 0.0112


@pytest.mark.parametrize("metric", ["l2-squared", "cosine", "dot"])
def test_sq_recall_and_stats(oracle, metric):  # :63-121 Test_NoRaceRandomSQDistanceFloatToByte
    m = oracle.METRIC[metric]
    rng = np.random.default_rng(5)
    data = rng.standard_normal((100, 150)).astype(np.float32)
    queries = rng.standard_normal((10, 150)).astype(np.float32)
    data = np.stack([oracle.normalize(x) for x in data])
    queries = np.stack([oracle.normalize(x) for x in queries])
    sq = oracle.SQ(data)
    codes = [sq.encode(x) for x in data]
    hits = 0
    for q in queries:
        exact = np.array([oracle.single_dist(m, oracle.AVX256, q, x) for x in data])
        truth = set(np.argsort(exact, kind="stable")[:10].tolist())
        cq = sq.encode(q)
        approx = np.array([sq.distance(m, cq, c) for c in codes])
        hits += len(truth & set(np.argsort(approx, kind="stable")[:10].tolist()))
    assert hits / 100 >= 0.95
    assert sq.a >= -1 and sq.a >= sq.b and sq.b <= 1


def test_sq_hamming_unsupported(oracle):  # :45-57: "Distance not supported yet"
    sq = oracle.SQ(np.array([[1, 0], [0, 1]], np.float32))
    c = sq.encode(np.array([0.5, 0.5], np.float32))
    assert np.isnan(sq.distance(oracle.HAMMING, c, c))


@pytest.mark.parametrize("rescore,limit", [(False, 5), (True, 5), (True, 40)])
def test_generic_flat_search_equals_pq_restatement(oracle, rescore, limit):
    """or_hnsw_flat_search over PQ distances == or_pq_flat_search (both
    restate hnsw/flat_search.go:28-141 + search.go:1047-1110)."""
    rng = np.random.default_rng(3)
    n, d, m, k = 600, 16, 4, 5
    data = np.round(rng.standard_normal((n, d)) * 2).astype(np.float32) / 2  # ties in both distances
    centers = oracle.pq_fit(data, m, 16, seed=4)
    codes = np.stack([oracle.pq_encode(centers, x) for x in data])
    present = np.ones(n, np.uint8)
    present[::7] = 0
    for qi in range(6):
        q = data[rng.integers(n)] + np.float32(0.25) * qi
        exp = oracle.pq_flat_search(oracle.L2, oracle.AVX256, centers, codes, data, present, q, k, limit, rescore)
        cd = np.array([oracle.pq_distance(oracle.L2, centers, q, c) for c in codes], np.float32)
        ed = np.array([oracle.single_dist(oracle.L2, oracle.AVX256, x, q) for x in data], np.float32)
        got = oracle.hnsw_flat_search(cd, ed, present, k, limit if rescore else k, rescore, 0)
        np.testing.assert_array_equal(got[0], exp[0])
        np.testing.assert_array_equal(got[1].view(np.uint32), exp[1].view(np.uint32))


def test_search_time_ef():  # hnsw/search.go:44-76
    import oracle as orc
    assert orc.search_time_ef(10) == 100        # 80 -> efMin
    assert orc.search_time_ef(20) == 160
    assert orc.search_time_ef(100) == 500       # 800 -> efMax
    assert orc.search_time_ef(600) == 600       # k > efMax
    assert orc.search_time_ef(10, ef=64) == 64
    assert orc.search_time_ef(100, ef=64) == 100
