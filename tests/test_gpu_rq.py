"""GPU parity for flat's rotational quantizers ("rq-8", "rq-1";
flat/quantizer.go:85-99): codes, quantized scan distances and
searchByVectorQuantized results of the HIP path against the oracle
(oracle/rq.c), bit-exact.  MI355X only (marker gpu)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VARIANTS = {"avx256": 1, "avx512": 2}


def gen(oracle, kind, seed, rows, d, row0=0):
    return oracle.gen_matrix(kind, seed, row0, rows, d)


def bits_equal(a, b, msg=""):
    np.testing.assert_array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32),
                                  err_msg=msg)


def build(wv, oracle, bits, metric, variant, data, rescore=-1, ids=None):
    n, d = data.shape
    ids = np.arange(n, dtype=np.uint64) if ids is None else ids
    idx = wv.FlatIndex(distance=metric, variant=variant, rq={"bits": bits}, rescore_limit=rescore)
    idx.add_batch(ids, data)
    orc = oracle.OracleFlatRQ(bits, oracle.METRIC[metric], VARIANTS[variant], d, int(ids.max()) + 1, rescore)
    orc.add_batch(ids, data)
    return idx, orc


@pytest.mark.parametrize("bits", [8, 1])
@pytest.mark.parametrize("metric,variant,d", [("cosine", "avx256", 768), ("l2-squared", "avx512", 128),
                                              ("dot", "avx256", 200), ("cosine", "avx512", 960),
                                              ("l2-squared", "avx256", 33), ("dot", "avx512", 1536)])
def test_rq_codes_bit_exact(wv, oracle, bits, metric, variant, d):
    n = 700
    data = gen(oracle, 0, 3, n, d) * np.float32(2.5)
    data[5] = 0  # zero vector: ZeroRQCode / zero rq-1 code
    data[6] = 1  # constant row
    idx, orc = build(wv, oracle, bits, metric, variant, data)
    info = idx.rq_info()
    assert info["bits"] == bits and info["created"] and info["output_dim"] == orc.rq.D
    got = idx.rq_codes(n)
    np.testing.assert_array_equal(got, orc.codes, err_msg=f"rq-{bits} codes")
    idx.close()


@pytest.mark.parametrize("bits", [8, 1])
@pytest.mark.parametrize("metric", ["cosine", "l2-squared", "dot"])
def test_rq_scan_distances_bit_exact(wv, oracle, bits, metric):
    n, d = 1500, 384
    data = gen(oracle, 0, 7, n, d)
    queries = gen(oracle, 0, 8, 40, d)
    queries[3] = 0  # zero query (rq-1: RQMultiBitCode{})
    idx, orc = build(wv, oracle, bits, metric, "avx256", data)
    got = idx.rq_distances(queries, n)
    for q in range(len(queries)):
        bits_equal(got[q], orc.query_distances(queries[q]), f"rq-{bits} {metric} q{q}")
    idx.close()


@pytest.mark.parametrize("bits", [8, 1])
@pytest.mark.parametrize("metric,kind,n,d,k,rescore", [
    ("cosine", 0, 5000, 768, 10, -1),
    ("l2-squared", 0, 3000, 128, 10, 100),
    ("dot", 0, 2500, 256, 7, 40),
    ("l2-squared", 1, 4000, 64, 20, -1),   # integer data: quantized ties
    ("cosine", 2, 1000, 960, 1, 200),
])
def test_rq_search_matches_oracle(wv, oracle, bits, metric, kind, n, d, k, rescore):
    data = gen(oracle, kind, 11, n, d)
    queries = gen(oracle, kind, 12, 24, d)
    idx, orc = build(wv, oracle, bits, metric, "avx256", data, rescore)
    assert idx.compressed()
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    for q in range(len(queries)):
        rc, oi, od = orc.search(queries[q], k)
        assert rc == 0 and counts[q] == len(oi), f"q{q}"
        np.testing.assert_array_equal(ids[q, :counts[q]], oi, err_msg=f"rq-{bits} {metric} q{q} ids")
        bits_equal(dists[q, :counts[q]], od, f"rq-{bits} {metric} q{q} dists")
    idx.close()


@pytest.mark.parametrize("bits", [8, 1])
def test_rq_duplicates_allow_delete_upsert(wv, oracle, bits):
    """All-equal rows tie on every quantized distance: the R-heap's tie order
    decides; plus deletes, upserts and allow lists."""
    n, d, k = 3000, 96, 10
    data = gen(oracle, 0, 21, n, d)
    data[1000:1600] = data[999]  # 601 identical rows
    idx, orc = build(wv, oracle, bits, "cosine", "avx512", data, 64)
    dele = np.arange(0, n, 7, dtype=np.uint64)
    idx.delete(*dele)
    orc.delete(dele)
    up = gen(oracle, 0, 22, 50, d)
    upids = np.arange(100, 150, dtype=np.uint64)
    idx.add_batch(upids, up)
    orc.add_batch(upids, up)
    queries = np.concatenate([gen(oracle, 0, 23, 6, d), data[999:1000]])
    allow = np.arange(50, 2500, 3, dtype=np.uint64)
    for q in range(len(queries)):
        gi, gd = idx.search_by_vector(queries[q], k)
        rc, oi, od = orc.search(queries[q], k)
        np.testing.assert_array_equal(gi, oi, err_msg=f"q{q}")
        bits_equal(gd, od, f"q{q}")
        gi, gd = idx.search_by_vector(queries[q], k, allow=wv.AllowList(allow))
        rc, oi, od = orc.search(queries[q], k, allow=allow)
        np.testing.assert_array_equal(gi, oi, err_msg=f"allow q{q}")
        bits_equal(gd, od, f"allow q{q}")
        gi, gd = idx.search_by_vector(queries[q], k, allow=wv.AllowList([]))
        assert len(gi) == 0
    idx.close()


def test_rq_large_batch_groups(wv, oracle):
    """More queries than one 32-query group and a ragged last group."""
    n, d, k = 20000, 128, 10
    data = gen(oracle, 0, 41, n, d)
    queries = gen(oracle, 0, 42, 77, d)
    for bits in (8, 1):
        idx, orc = build(wv, oracle, bits, "l2-squared", "avx256", data, 30)
        ids, dists, counts = idx.search_by_vector_batch(queries, k)
        for q in range(0, len(queries), 5):
            rc, oi, od = orc.search(queries[q], k)
            np.testing.assert_array_equal(ids[q, :counts[q]], oi, err_msg=f"rq-{bits} q{q}")
            bits_equal(dists[q, :counts[q]], od)
        idx.close()


def test_rq_errors(wv, oracle):
    with pytest.raises(wv.WeaviateError, match="Distance not supported"):
        wv.FlatIndex(distance="hamming", rq={"bits": 8})
    idx = wv.FlatIndex(distance="cosine", rq={"bits": 1})
    assert not idx.compressed()  # quantizer created at the first Add
    with pytest.raises(wv.WeaviateError, match="quantizer not initialized"):
        idx.rq_codes(0)
    idx.add_batch(np.arange(10, dtype=np.uint64), gen(oracle, 0, 1, 10, 100))
    assert idx.compressed()
    with pytest.raises(wv.WeaviateError, match="vector lengths don't match"):
        idx.search_by_vector(np.zeros(99, np.float32), 3)
    idx.close()


@pytest.mark.parametrize("metric,kind,n,d,k,rescore,nq", [
    ("cosine", 0, 40000, 768, 10, 200, 300),   # the bench's shape, smaller corpus
    ("l2-squared", 0, 9000, 128, 10, 63, 70),   # R + 1 = 64: the 64-entry list is too short, RT 4
    ("dot", 0, 7000, 320, 5, -1, 33),           # odd chunk count (D = 320, NC = 5)
    ("l2-squared", 1, 12000, 64, 20, 100, 40),  # integer data: quantized ties -> replayed queries
    ("cosine", 0, 3000, 1024, 3, 500, 20),      # D = 1024 (NC 16), R + 2 > 448: RT 16
])
@pytest.mark.parametrize("bits", [8, 1])
def test_rq_mfma_route_equals_replay_and_oracle(wv, oracle, bits, metric, kind, n, d, k, rescore, nq):
    """rq-8 / rq-1 on the integer MFMA (k_rq8_keys -> k_rq8_sel -> k_rq8_cand,
    flagged queries replayed) against the distance-matrix route (rq_mfma 0)
    over every query, and the oracle on a sample, bit for bit."""
    data = gen(oracle, kind, 51, n, d)
    queries = gen(oracle, kind, 52, nq, d)
    queries[1] = data[17]  # a stored vector: distance ties with itself only
    queries[2] = 0  # zero query (rq-1: RQMultiBitCode{}, dot 0)
    idx, orc = build(wv, oracle, bits, metric, "avx256", data, rescore)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    st = idx.stats()
    assert st["last_route"] == 10  # WV_ROUTE_RQ8_INT8
    idx.set_option("rq_mfma", 0)
    ids0, dists0, counts0 = idx.search_by_vector_batch(queries, k)
    assert idx.stats()["last_route"] != 10
    np.testing.assert_array_equal(counts, counts0)
    np.testing.assert_array_equal(ids, ids0)
    bits_equal(dists, dists0, "mfma vs replay route")
    for q in range(0, nq, max(1, nq // 6)):
        rc, oi, od = orc.search(queries[q], k)
        np.testing.assert_array_equal(ids[q, :counts[q]], oi, err_msg=f"q{q}")
        bits_equal(dists[q, :counts[q]], od, f"q{q}")
    idx.close()


@pytest.mark.parametrize("bits", [8, 1])
def test_rq_mfma_route_ties_deletes_allow(wv, oracle, bits):
    """Identical rows tie on the quantized distance: those queries are flagged
    and replayed; deletes and allow lists mask rows inside the key pass."""
    n, d, k = 6000, 192, 10
    data = gen(oracle, 0, 61, n, d)
    data[2000:2300] = data[1999]
    idx, orc = build(wv, oracle, bits, "l2-squared", "avx256", data, 50)
    dele = np.arange(3, n, 11, dtype=np.uint64)
    idx.delete(*dele)
    orc.delete(dele)
    queries = np.concatenate([gen(oracle, 0, 62, 40, d), data[1999:2000], data[4000:4001]])
    before = idx.stats()["replayed_queries"]
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    assert idx.stats()["last_route"] == 10
    assert idx.stats()["replayed_queries"] - before >= 1  # the duplicate-row query
    for q in range(len(queries)):
        rc, oi, od = orc.search(queries[q], k)
        np.testing.assert_array_equal(ids[q, :counts[q]], oi, err_msg=f"q{q}")
        bits_equal(dists[q, :counts[q]], od, f"q{q}")
    allow = np.arange(100, 5000, 2, dtype=np.uint64)
    for q in (0, 40, 41):
        gi, gd = idx.search_by_vector(queries[q], k, allow=wv.AllowList(allow))
        rc, oi, od = orc.search(queries[q], k, allow=allow)
        np.testing.assert_array_equal(gi, oi, err_msg=f"allow q{q}")
        bits_equal(gd, od, f"allow q{q}")
    idx.close()
