"""GPU parity: the HIP flat index vs the oracle (CPU restatement of
flat/index.go + priorityqueue + distancer), bit-exact ids and distances.

Runs on an MI355X only (marker gpu).  Sizes keep the oracle to seconds.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VARIANTS = {"avx256": 1, "avx512": 2}


def gen(oracle, kind, seed, rows, d, row0=0):
    return oracle.gen_matrix(kind, seed, row0, rows, d)


def assert_same(oracle_res, ids, dists, ctx=""):
    rc, oids, od = oracle_res
    assert rc == 0
    assert len(ids) == len(oids), f"{ctx}: count {len(ids)} vs {len(oids)}"
    np.testing.assert_array_equal(ids, oids, err_msg=f"{ctx}: ids")
    # bit-exact distances
    np.testing.assert_array_equal(np.asarray(dists, np.float32).view(np.uint32),
                                  np.asarray(od, np.float32).view(np.uint32), err_msg=f"{ctx}: dists")


def build_pair(wv, oracle, metric_name, variant, data, ids=None, dims=0, options=None):
    n, d = data.shape
    ids = np.arange(n, dtype=np.uint64) if ids is None else ids
    idx = wv.FlatIndex(distance=metric_name, variant=variant, dims=dims)
    for key, val in (options or {}).items():
        idx.set_option(key, val)
    idx.add_batch(ids, data)
    orc = oracle.OracleFlat(oracle.METRIC[metric_name], VARIANTS[variant], d, int(ids.max()) + 1)
    orc.add_batch(ids, data)
    return idx, orc


@pytest.mark.parametrize("variant", ["avx256", "avx512"])
@pytest.mark.parametrize("metric", ["l2-squared", "dot", "cosine"])
def test_distance_batch_bit_exact(wv, oracle, metric, variant):
    rng = np.random.default_rng(1)
    for d in [1, 3, 7, 8, 9, 31, 32, 33, 100, 127, 128, 129, 200, 255, 256, 300, 768, 960, 1536]:
        a = rng.standard_normal((64, d)).astype(np.float32)
        b = rng.standard_normal((64, d)).astype(np.float32) * np.float32(3.0)
        got = wv.single_dist_batch(metric, a, b, variant=variant)
        exp = np.array([oracle.single_dist(oracle.METRIC[metric], VARIANTS[variant], a[i], b[i])
                        for i in range(64)], dtype=np.float32)
        np.testing.assert_array_equal(got.view(np.uint32), exp.view(np.uint32), err_msg=f"d={d}")


def test_normalize_bit_exact(wv, oracle):
    rng = np.random.default_rng(2)
    for d in [1, 5, 128, 768, 1536]:
        v = (rng.standard_normal((50, d)) * 10).astype(np.float32)
        v[0] = 0
        got = wv.normalize_batch(v)
        exp = np.stack([oracle.normalize(x) for x in v])
        np.testing.assert_array_equal(got.view(np.uint32), exp.view(np.uint32))


def test_hamming_and_bq_exact(wv, oracle):
    rng = np.random.default_rng(3)
    for d in [1, 63, 64, 65, 128, 1536]:
        v = rng.standard_normal((40, d)).astype(np.float32)
        codes = wv.bq_encode_batch(v)
        exp = np.stack([oracle.bq_encode(x) for x in v])
        np.testing.assert_array_equal(codes, exp)
        h = wv.hamming_bitwise_batch(codes[:20], codes[20:])
        eh = np.array([oracle.hamming_bitwise(codes[i], codes[20 + i]) for i in range(20)], np.float32)
        np.testing.assert_array_equal(h, eh)


@pytest.mark.parametrize("variant", ["avx256", "avx512"])
@pytest.mark.parametrize("metric,kind,n,d,k", [
    ("l2-squared", 0, 20000, 128, 10),   # C1-shaped (scaled): U(-1,1)
    ("cosine", 0, 6000, 768, 10),        # C3-shaped (scaled)
    ("dot", 0, 8000, 96, 7),
    ("l2-squared", 1, 6000, 128, 10),    # SIFT-shaped integer data: ties -> replay
    ("cosine", 0, 3000, 33, 24),         # ragged dims, max fast-path k
])
def test_search_matches_oracle(wv, oracle, metric, kind, n, d, k, variant):
    data = gen(oracle, kind, 11, n, d)
    queries = gen(oracle, kind, 12, 48, d)
    idx, orc = build_pair(wv, oracle, metric, variant, data)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    for qi in range(len(queries)):
        res = orc.search(queries[qi], k)
        assert_same(res, ids[qi, :counts[qi]], dists[qi, :counts[qi]], ctx=f"q{qi}")
    idx.close()


def test_forced_replay_equals_fast_path(wv, oracle):
    data = gen(oracle, 0, 21, 5000, 64)
    queries = gen(oracle, 0, 22, 32, 64)
    idx, orc = build_pair(wv, oracle, "l2-squared", "avx256", data)
    ids1, d1, c1 = idx.search_by_vector_batch(queries, 10)
    idx.set_option("force_replay", 1)
    ids2, d2, c2 = idx.search_by_vector_batch(queries, 10)
    np.testing.assert_array_equal(ids1, ids2)
    np.testing.assert_array_equal(d1.view(np.uint32), d2.view(np.uint32))
    assert idx.stats()["replayed_queries"] >= 32


def test_ties_duplicates_heap_order(wv, oracle):
    """Many exactly duplicated vectors: result order must follow the reference
    heap layout, not (dist, id)."""
    base = gen(oracle, 1, 31, 50, 8)
    data = np.concatenate([base] * 40)  # 2000 rows, each vector 40 times
    queries = gen(oracle, 1, 32, 16, 8)
    for k in [1, 5, 10, 17]:
        idx, orc = build_pair(wv, oracle, "l2-squared", "avx256", data)
        ids, dists, counts = idx.search_by_vector_batch(queries, k)
        for qi in range(len(queries)):
            assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"k{k} q{qi}")
        idx.close()


def test_large_k_replay_path(wv, oracle):
    data = gen(oracle, 0, 41, 4000, 48)
    queries = gen(oracle, 0, 42, 8, 48)
    idx, orc = build_pair(wv, oracle, "cosine", "avx256", data)
    ids, dists, counts = idx.search_by_vector_batch(queries, 100)
    for qi in range(len(queries)):
        assert_same(orc.search(queries[qi], 100), ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"q{qi}")
    # k in the thousands: the replay heap needs more than the default 64 KiB LDS
    for k in (3000, 6000):
        ids, dists, counts = idx.search_by_vector_batch(queries[:3], k)
        for qi in range(3):
            assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"k{k} q{qi}")
    # beyond the LDS heap: a clear error, not a launch failure
    with pytest.raises(wv.WeaviateError, match="exceeds the exact replay heap limit"):
        idx.search_by_vector_batch(queries[:1], 20000)


def test_allow_list_delete_upsert(wv, oracle):
    data = gen(oracle, 0, 51, 3000, 40)
    queries = gen(oracle, 0, 52, 8, 40)
    idx, orc = build_pair(wv, oracle, "dot", "avx256", data)
    # upsert some ids, delete others
    new = gen(oracle, 0, 53, 100, 40)
    up_ids = np.arange(500, 600, dtype=np.uint64)
    idx.add_batch(up_ids, new)
    orc.add_batch(up_ids, new)
    dels = list(range(0, 3000, 7))
    idx.delete(*dels)
    orc.delete(dels)
    allow = list(range(100, 2500, 3))
    al = wv.AllowList(allow)
    ids, dists, counts = idx.search_by_vector_batch(queries, 10, allow=al)
    for qi in range(len(queries)):
        assert_same(orc.search(queries[qi], 10, allow=allow), ids[qi, :counts[qi]], dists[qi, :counts[qi]],
                    f"q{qi}")
    # empty allow list -> empty result, no error (flat/index.go:590-594)
    ids, d_ = idx.search_by_vector(queries[0], 10, allow=wv.AllowList([]))
    assert len(ids) == 0
    assert idx.already_indexed() == 3100
    assert not idx.contains_doc(7) and idx.contains_doc(8)


def test_sparse_ids_and_small_corpus(wv, oracle):
    data = gen(oracle, 0, 61, 5, 16)
    ids = np.array([3, 1000, 17, 4096, 9], dtype=np.uint64)
    idx, orc = build_pair(wv, oracle, "l2-squared", "avx256", data, ids=ids)
    q = gen(oracle, 0, 62, 4, 16)
    for k in [1, 3, 5, 10]:
        got_ids, got_d, cnt = idx.search_by_vector_batch(q, k)
        for qi in range(4):
            assert_same(orc.search(q[qi], k), got_ids[qi, :cnt[qi]], got_d[qi, :cnt[qi]], f"k{k}")


def test_errors_and_edge_cases(wv):
    idx = wv.FlatIndex(distance="l2-squared", root_path="/tmp/x")
    with pytest.raises(wv.WeaviateError, match="cannot insert vector of dimension 0"):
        idx.add(1, np.zeros(0, np.float32))
    # empty index: no error, empty result
    ids, d = idx.search_by_vector(np.ones(3, np.float32), 5)
    assert len(ids) == 0
    idx.add(1, np.array([3, 4, 5], np.float32))
    with pytest.raises(wv.WeaviateError, match=r"insert called with a vector of the wrong size: 2\. Saved length: 3, path: /tmp/x"):
        idx.add(2, np.array([1, 2], np.float32))
    with pytest.raises(wv.WeaviateError, match="vector lengths don't match"):
        idx.search_by_vector(np.ones(4, np.float32), 5)
    with pytest.raises(wv.WeaviateError, match="insertBatch called with empty lists"):
        idx.add_batch([], [])
    with pytest.raises(wv.WeaviateError, match="ids and vectors sizes does not match"):
        idx.add_batch([1, 2], [np.ones(3, np.float32)])
    ids, d = idx.search_by_vector(np.array([1.5, 2, 2.5], np.float32), 5)
    assert list(ids) == [1] and d[0] == np.float32(12.5)  # distancer/l2_test.go known answer
    # 1-d vectors (flat/index_test.go TestEdgeCases)
    one = wv.FlatIndex(distance="cosine")
    one.add(0, np.array([1.0], np.float32))
    one.add(1, np.array([-2.0], np.float32))
    ids, d = one.search_by_vector(np.array([5.0], np.float32), 2)
    assert list(ids) == [0, 1] and d[0] == 0 and d[1] == 2


def test_search_by_vector_distance(wv, oracle):
    data = gen(oracle, 0, 71, 2000, 24)
    idx, orc = build_pair(wv, oracle, "cosine", "avx256", data)
    q = gen(oracle, 0, 72, 1, 24)[0]
    rc, oids, od = orc.search(q, 100)
    target = float(od[30])
    ids, d = idx.search_by_vector_distance(q, target, 10000)
    exp = [(i, x) for i, x in zip(oids, od) if x <= target or abs(float(x) - target) <= 1e-6]
    assert list(ids) == [e[0] for e in exp][: len(ids)]
    assert len(ids) == 31


@pytest.mark.parametrize("kernel", [0, 3, 6, 7])
@pytest.mark.parametrize("metric,kind,n,d,k", [("cosine", 0, 9000, 768, 10), ("l2-squared", 0, 7000, 96, 24),
                                               ("dot", 1, 5000, 64, 5), ("cosine", 0, 3000, 2048, 10)])
def test_select_kernel_variants(wv, oracle, kernel, metric, kind, n, d, k):
    """Every select path (0 auto, 3 the f32 MFMA select, 6 the GEMV select,
    7 block keys; d = 2048 has no block-key planes: 7 and 0 take the f32
    select) against the oracle on every query."""
    data = gen(oracle, kind, 81, n, d)
    queries = gen(oracle, kind, 82, 300, d)   # > 2 query blocks, ragged last block
    idx, orc = build_pair(wv, oracle, metric, "avx256", data)
    idx.set_option("kernel", kernel)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    for qi in range(len(queries)):
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"q{qi}")
    idx.close()


def test_removed_select_kernels_rejected(wv, oracle):
    """The round-1 select kernels (1, 2: f32 tiles; 4, 5: bf16x3) were removed:
    the option refuses them, and their bf16x3 planes option is gone."""
    idx = wv.FlatIndex(distance="cosine")
    for kernel in (1, 2, 4, 5, 8):
        with pytest.raises(wv.WeaviateError, match="kernel must be"):
            idx.set_option("kernel", kernel)
    with pytest.raises(wv.WeaviateError):
        idx.set_option("bf3_planes", 1)
    idx.close()


@pytest.mark.parametrize("metric,kind,n,d,k,nq", [
    ("cosine", 0, 30000, 768, 10, 1), ("cosine", 0, 30000, 768, 10, 8), ("l2-squared", 0, 20000, 100, 24, 3),
    ("dot", 2, 12000, 40, 5, 5), ("l2-squared", 1, 8000, 2500, 10, 6), ("cosine", 0, 5000, 1536, 32 - 8, 2),
    ("cosine", 0, 3000, 3500, 10, 4), ("cosine", 0, 3000, 6500, 10, 4)])  # above 6144: no planes, the GEMV by default
def test_gemv_small_batches(wv, oracle, metric, kind, n, d, k, nq):
    """Small batches: the default route and the HBM-streaming GEMV (k_gemv_select).

    Measured on C3 (profiles/r04_small_batch_c3.jsonl, tools/small_batch.py):
    with block-key planes the padded int8 key pass beats the GEMV at every
    B = 1..256 (B = 1: 3.39 vs 5.11 ms), so small batches keep the block-key
    route wherever planes exist (d <= 6144 since round 5) and take the GEMV only without them;
    `kernel = 6` forces the GEMV.  Both routes are asserted and oracle-checked.
    """
    data = gen(oracle, kind, 91, n, d)
    queries = gen(oracle, kind, 92, nq, d)
    idx, orc = build_pair(wv, oracle, metric, "avx256", data)
    idx.delete(*range(3, n, 17))
    orc.delete(list(range(3, n, 17)))
    planes = d <= 6144  # bf16 / int8 planes up to 1536, int8-only planes up to 6144
    for forced in (False, True):
        idx.set_option("kernel", 6 if forced else 0)
        expect = "gemv" if forced or not planes else ("qs_bf16", "qs_w4", "qs_int8", "q8_gemv")
        before = idx.stats()["replayed_queries"]
        ids, dists, counts = idx.search_by_vector_batch(queries, k)
        route = wv._lib.ROUTES[idx.stats()["last_route"]]
        assert route in (expect if isinstance(expect, tuple) else (expect,)), (forced, route)
        for qi in range(nq):
            assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"q{qi}")
        if kind == 0 and route == "gemv":  # continuous data: the fp32 error bound proves every query
            assert idx.stats()["replayed_queries"] == before
        allow = list(range(5, n, 3))
        ids, dists, counts = idx.search_by_vector_batch(queries, k, allow=wv.AllowList(allow))
        for qi in range(nq):
            assert_same(orc.search(queries[qi], k, allow=allow), ids[qi, :counts[qi]], dists[qi, :counts[qi]],
                        f"a{qi}")
    idx.close()


# ---------------------------------------------------------------------------
# BQ-compressed flat search (flat/index.go:460-532)
# ---------------------------------------------------------------------------
def build_bq_pair(wv, oracle, metric_name, variant, data, rescore_limit, ids=None):
    n, d = data.shape
    ids = np.arange(n, dtype=np.uint64) if ids is None else ids
    idx = wv.FlatIndex(distance=metric_name, variant=variant, bq=True, rescore_limit=rescore_limit)
    idx.add_batch(ids, data)
    orc = oracle.OracleFlatBQ(oracle.METRIC[metric_name], VARIANTS[variant], d, int(ids.max()) + 1, rescore_limit)
    orc.add_batch(ids, data)
    return idx, orc


@pytest.mark.parametrize("metric,kind,n,d,k,rescore", [
    ("cosine", 0, 20000, 1536, 10, 200),   # C4-shaped (scaled)
    ("cosine", 0, 5000, 768, 10, -1),      # default rescore limit -> k
    ("l2-squared", 0, 7000, 128, 10, 100),
    ("dot", 0, 3000, 100, 5, 37),          # ragged words
    ("cosine", 1, 3000, 64, 10, 50),       # all-positive data: every code is 0, hamming ties everywhere
    ("l2-squared", 2, 2500, 200, 20, 20),  # rescore == k
    ("cosine", 0, 600, 65, 10, 1000),      # rescore limit > corpus
    ("l2-squared", 0, 1500, 2500, 10, 30),  # 40 words: generic (non-LDS) kernels
    ("cosine", 0, 9000, 1000, 10, 64),     # 16 words
])
def test_bq_search_matches_oracle(wv, oracle, metric, kind, n, d, k, rescore):
    data = gen(oracle, kind, 11, n, d)
    queries = gen(oracle, kind, 12, 24, d)
    idx, orc = build_bq_pair(wv, oracle, metric, "avx256", data, rescore)
    assert idx.compressed()
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    for q in range(len(queries)):
        assert_same(orc.search(queries[q], k), ids[q, :counts[q]], dists[q, :counts[q]], f"bq {metric} q{q}")
    idx.close()


def test_bq_allow_delete_upsert_variant(wv, oracle):
    n, d, k = 4000, 96, 10
    data = gen(oracle, 0, 21, n, d)
    idx, orc = build_bq_pair(wv, oracle, "cosine", "avx512", data, 64)
    dele = np.arange(0, n, 7, dtype=np.uint64)
    idx.delete(*dele)
    orc.delete(dele)
    up = gen(oracle, 0, 22, 50, d)
    upids = np.arange(100, 150, dtype=np.uint64)
    idx.add_batch(upids, up)
    orc.add_batch(upids, up)
    queries = gen(oracle, 0, 23, 8, d)
    allow = np.arange(50, 3000, 3, dtype=np.uint64)
    for q in range(len(queries)):
        gi, gd = idx.search_by_vector(queries[q], k)
        assert_same(orc.search(queries[q], k), gi, gd, f"q{q}")
        gi, gd = idx.search_by_vector(queries[q], k, allow=wv.AllowList(allow))
        assert_same(orc.search(queries[q], k, allow=allow), gi, gd, f"allow q{q}")
        gi, gd = idx.search_by_vector(queries[q], k, allow=wv.AllowList([]))
        assert len(gi) == 0
    idx.close()


def test_bq_errors(wv, oracle):
    data = gen(oracle, 0, 31, 300, 128)
    idx, _ = build_bq_pair(wv, oracle, "l2-squared", "avx256", data, -1)
    with pytest.raises(wv.WeaviateError, match="both vectors should have the same len"):
        idx.search_by_vector(np.zeros(200, np.float32), 5)
    with pytest.raises(wv.WeaviateError, match="vector lengths don't match"):
        idx.search_by_vector(np.zeros(100, np.float32), 5)  # same word count, rescoring length check
    idx.close()


def test_bq_generic_kernels_equal_lds_kernels(wv, oracle):
    data = gen(oracle, 0, 51, 6000, 512)
    queries = gen(oracle, 0, 52, 300, 512)
    idx = wv.FlatIndex(distance="cosine", bq=True, rescore_limit=40)
    idx.add_batch(np.arange(6000, dtype=np.uint64), data)
    a = idx.search_by_vector_batch(queries, 10)
    idx.set_option("bq_kernel", 1)
    b = idx.search_by_vector_batch(queries, 10)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    idx.close()


@pytest.mark.parametrize("metric,kind,d", [("cosine", 0, 768), ("l2-squared", 0, 128), ("dot", 0, 300),
                                           ("l2-squared", 2, 2048)])
def test_f32_select_error_within_proof_bound(wv, oracle, metric, kind, d):
    """The approximate distances of the f32 MFMA select kernel (candidates A,
    kernel 3: the fallback above 1536 dims) stay within the eps the
    exactness proof uses."""
    n = 20000
    data = gen(oracle, kind, 91, n, d)
    queries = gen(oracle, kind, 92, 256, d)
    idx = wv.FlatIndex(distance=metric, variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    idx.set_option("kernel", 3)
    idx.search_by_vector_batch(queries, 10)
    A, E, I, eps = idx.debug_candidates(len(queries))
    ok = I != 0xFFFFFFFF
    err = np.abs(A[ok].astype(np.float64) - E[ok].astype(np.float64))
    bound = np.broadcast_to(eps[:, None], A.shape)[ok]
    ratio = (err / bound).max()
    print(f"f32 select max |A-E| / eps = {ratio:.4f}")
    assert (err <= bound).all(), f"max err/eps = {ratio}"
    idx.close()


@pytest.mark.parametrize("k", [1, 10, 50, 63, 64, 100, 191, 200])
def test_block_key_replay_parallel_and_single_wave(wv, oracle, k):
    """Integer data (exact ties everywhere): most queries go to the heap replay.
    replay_par=3 (2, the default, for k < 64): pooled k_rp_bounds / k_rp_exact /
    k_rp_heap, also with a one-block and a 300-block pool (queries that do not
    fit fall back to the on-the-fly scan);
    replay_par=1, k < 64: k_blk_replay_par; else / replay_par=0: the one-wave
    k_blk_replay.  All equal the reference heap, including queries with
    non-finite values (every block visited)."""
    n, d = 60000, 24
    data = gen(oracle, 1, 91, n, d)
    queries = gen(oracle, 1, 92, 40, d)
    queries[3, 5] = np.nan
    queries[7, 0] = np.inf
    res = []
    for par, pool in ((3, 0), (3, 1), (3, 300), (2, 0), (1, 0), (0, 0)):
        idx, orc = build_pair(wv, oracle, "l2-squared", "avx256", data)
        idx.set_option("replay_par", par)
        if pool:
            idx.set_option("rp_pool", pool)
        before = idx.stats()["replayed_queries"]
        res.append(idx.search_by_vector_batch(queries, k))
        assert idx.stats()["replayed_queries"] - before >= 2  # at least the non-finite queries
    for qi in range(len(queries)):
        exp = orc.search(queries[qi], k)
        for ids, dists, counts in res:
            assert_same(exp, ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"k{k} q{qi}")


@pytest.mark.parametrize("metric", ["cosine", "l2-squared", "dot"])
def test_pooled_replay_float_data(wv, oracle, metric):
    """Random float data: forced replay of every query through the pooled
    k_rp_* kernels (the C3 path of a flagged query) equals the oracle."""
    n, d, k = 50000, 96, 10
    data = gen(oracle, 0, 93, n, d)
    queries = gen(oracle, 0, 94, 24, d)
    idx, orc = build_pair(wv, oracle, metric, "avx256", data)
    idx.set_option("replay_par", 2)
    idx.set_option("qs_force_flag", 1)
    before = idx.stats()["replayed_queries"]
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    assert idx.stats()["replayed_queries"] - before == len(queries)
    for qi in range(len(queries)):
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"{metric} q{qi}")


@pytest.mark.parametrize("metric,variant,d,k", [("l2-squared", "avx256", 128, 100), ("cosine", "avx256", 37, 10),
                                               ("dot", "avx256", 200, 100), ("l2-squared", "avx256", 5, 10),
                                               ("cosine", "avx512", 100, 24), ("l2-squared", "avx512", 160, 100),
                                               ("dot", "avx256", 771, 10)])
def test_one_wave_replay_float_data(wv, oracle, metric, variant, d, k):
    """Random float data, every query forced through the one-wave k_blk_replay
    (replay_par 0): the 8-lanes-per-row exact distances (AVX2 order, and the
    AVX-512 order below 128 dims; 32-, 8-element and scalar tails) and the
    lane-per-row form (AVX-512 from 128 dims) equal the oracle bit for bit."""
    n = 20000
    data = gen(oracle, 0, 97, n, d)
    queries = gen(oracle, 0, 98, 16, d)
    idx, orc = build_pair(wv, oracle, metric, variant, data)
    idx.set_option("replay_par", 0)
    idx.set_option("qs_force_flag", 1)
    before = idx.stats()["replayed_queries"]
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    assert idx.stats()["replayed_queries"] - before == len(queries)
    for qi in range(len(queries)):
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"{metric} d{d} q{qi}")


@pytest.mark.parametrize("metric,variant,d,k", [("cosine", "avx256", 768, 10), ("l2-squared", "avx256", 130, 24),
                                               ("dot", "avx512", 96, 10), ("cosine", "avx512", 200, 100)])
def test_exact_row_filter_equals_unfiltered(wv, oracle, metric, variant, d, k):
    """exact_filter 1 (k_blk_exact skips rows whose bf16-plane bound reaches
    the cap) returns what exact_filter 0 (every candidate row exact) and the
    oracle return, bit for bit."""
    n = 30000
    data = gen(oracle, 0, 99, n, d)
    queries = gen(oracle, 0, 100, 200, d)
    res = []
    for filt in (0, 1):
        idx, orc = build_pair(wv, oracle, metric, variant, data)
        idx.set_option("exact_filter", filt)
        res.append(idx.search_by_vector_batch(queries, k))
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
    for qi in range(0, len(queries), 20):
        ids, dists, counts = res[1]
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"{metric} q{qi}")


@pytest.mark.parametrize("metric,kind,variant,n,d,k", [("l2-squared", 1, "avx256", 40000, 128, 100),   # C2-like ties
                                                      ("cosine", 0, "avx512", 30000, 200, 10),
                                                      ("dot", 0, "avx256", 20000, 500, 24),
                                                      ("l2-squared", 1, "avx256", 30000, 24, 200)])  # R = 8 lists
def test_block_major_exact_equals_oracle(wv, oracle, metric, kind, variant, n, d, k):
    """exact_bm=1: candidate lists inverted per 32-row block (k_inv_*), each
    block's rows staged once (k_exact_bm), k_blk_exact reads the distances.
    Results (fast path, proof flags and replays) equal the oracle and the
    per-query path bit for bit."""
    data = gen(oracle, kind, 95, n, d)
    queries = gen(oracle, kind, 96, 300, d)
    res = []
    for bm in (0, 1):
        idx, orc = build_pair(wv, oracle, metric, variant, data)
        idx.set_option("exact_bm", bm)
        res.append(idx.search_by_vector_batch(queries, k))
    for qi in range(len(queries)):
        exp = orc.search(queries[qi], k)
        for ids, dists, counts in res:
            assert_same(exp, ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"{metric} k{k} q{qi}")


@pytest.mark.parametrize("metric,kind,variant,n,d,k,options", [
    ("cosine", 0, "avx256", 20000, 1024, 10, None),     # voyage-3 width
    ("l2-squared", 0, "avx512", 12000, 1536, 10, None),
    ("l2-squared", 1, "avx256", 12000, 1024, 100, None),  # integer data: ties -> the keyed replay
    ("dot", 0, "avx256", 9000, 800, 24, None),           # dpb 1024: zero-padded columns
    ("cosine", 0, "avx256", 8000, 1030, 10, None),       # dpb 1536: 506 zero columns
    ("cosine", 0, "avx512", 15000, 1536, 100, None),
    ("l2-squared", 2, "avx256", 10000, 1100, 10, None),  # dpb 1536
])
def test_block_keys_above_768_dims(wv, oracle, metric, kind, variant, n, d, k, options):
    """768 < d <= 1536: k_qs_blockkey_w4 (one wave per SIMD, 128-query
    workgroups, two column halves per ring step) feeds the same selection /
    exact / replay pipeline.  Bit-exact against the oracle for every query,
    and its block keys within the proof's eps of the exact block minima."""
    data = gen(oracle, kind, 61, n, d)
    queries = gen(oracle, kind, 62, 160, d)
    idx, orc = build_pair(wv, oracle, metric, variant, data, options=options)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    for qi in range(len(queries)):
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], ctx=f"q{qi}")
    sample = [0, 57, 128, 159]
    qs = queries[sample]
    if metric == "cosine":
        qs = np.stack([oracle.normalize(x) for x in qs])
    D = oracle.gen_dists(kind, 61, n, d, oracle.METRIC[metric], VARIANTS[variant], qs, 8)
    worst = 0.0
    for i, q in enumerate(sample):
        A, eps = idx.debug_blockkeys(q)  # raises unless the block-key path ran
        bmin = D[i][: (n // 32) * 32].reshape(-1, 32).min(axis=1).astype(np.float64)
        err = np.abs(A[: bmin.size].astype(np.float64) - bmin)
        worst = max(worst, float(err.max() / eps))
        assert (err <= eps).all(), f"q{q}: block-key error {err.max()} > eps {eps}"
    print(f"d={d}: max |A_block - min E| / eps = {worst:.4f}")
    idx.close()


@pytest.mark.parametrize("metric,kind,n,d,k,nq", [
    ("l2-squared", 0, 20000, 128, 10, 100),   # C1-shaped: bf16 block keys
    ("cosine", 0, 12000, 768, 10, 64),        # int8 block keys
    ("l2-squared", 1, 9000, 128, 100, 50),    # integer ties: the heap replay inside the graph
])
def test_search_device_graph_replay(wv, oracle, metric, kind, n, d, k, nq):
    """A repeated identical wv_index_search_device call on a caller stream is
    captured into a hipGraph on its second occurrence and replayed after; the
    replays must equal the uncaptured path, count their queries in the stats,
    and stop applying once the corpus changes (Add / Delete / options)."""
    torch = pytest.importorskip("torch")
    from weaviate_amd import _lib
    lib = _lib.load()
    data = gen(oracle, kind, 95, n, d)
    queries = gen(oracle, kind, 96, nq, d)
    idx, _ = build_pair(wv, oracle, metric, "avx256", data)
    orc = oracle.OracleFlat(oracle.METRIC[metric], VARIANTS["avx256"], d, n + 8)  # room for the added rows
    orc.add_batch(np.arange(n, dtype=np.uint64), data)
    qd = torch.from_numpy(queries).cuda()
    oi = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    od = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    on = torch.empty(nq, dtype=torch.int32, device="cuda")
    stream = torch.cuda.Stream()

    def run():
        oi.fill_(-1)
        od.fill_(-1)
        on.fill_(-1)
        torch.cuda.synchronize()
        _lib.check(lib.wv_index_search_device(idx._h, qd.data_ptr(), nq, d, k, 0, oi.data_ptr(), od.data_ptr(),
                                              on.data_ptr(), None, stream.cuda_stream))
        stream.synchronize()
        return oi.cpu().numpy().copy(), od.cpu().numpy().copy(), on.cpu().numpy().copy()

    def check(res, tag):
        ids, dists, counts = res
        for qi in range(0, nq, max(1, nq // 16)):
            assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]].astype(np.uint64),
                        dists[qi, :counts[qi]], f"{tag} q{qi}")

    idx.set_option("graph", 0)
    ref = run()
    check(ref, "plain")
    idx.set_option("graph", 1)
    q0 = idx.stats()["queries"]
    for rep in range(4):  # 1: uncaptured, 2: captured, 3-4: replays
        got = run()
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(a, b, err_msg=f"rep {rep}")
    assert idx.stats()["queries"] - q0 == 4 * nq
    # a caller that reuses one query buffer (a cgo shim's pinned buffer): new
    # contents at the same address replay the captured graph on the new queries
    queries2 = gen(oracle, kind, 97, nq, d)
    for rep in range(2):
        qd.copy_(torch.from_numpy(queries2))
        got2 = run()
        for qi in range(0, nq, max(1, nq // 16)):
            assert_same(orc.search(queries2[qi], k), got2[0][qi, :got2[2][qi]].astype(np.uint64),
                        got2[1][qi, :got2[2][qi]], f"rewritten buffer rep {rep} q{qi}")
        qd.copy_(torch.from_numpy(queries))
        got = run()
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(a, b, err_msg=f"restored buffer rep {rep}")
    # the corpus changes: near-copies of the first queries become their nearest rows
    extra = (queries[:8] + np.float32(1e-3)).astype(np.float32)
    new_ids = np.arange(n, n + 8, dtype=np.uint64)
    idx.add_batch(new_ids, extra)
    orc.add_batch(new_ids, extra)
    got = run()
    check(got, "after add")
    assert set(range(n, n + 8)) & set(got[0][:8].ravel().tolist())
    idx.delete(*range(n, n + 8))
    orc.delete(list(range(n, n + 8)))
    for rep in range(3):
        got = run()
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(a, b, err_msg=f"after delete rep {rep}")
    idx.close()


@pytest.mark.parametrize("metric,kind,n,d,k", [
    ("l2-squared", 0, 40000, 128, 500),    # bf16 keys, 960-block lists (no block-major pass)
    ("cosine", 0, 40000, 768, 500),        # int8 keys
    ("l2-squared", 1, 30000, 128, 900),    # integer data: ties -> the heap replay at k = 900
    ("dot", 0, 20000, 2048, 600),          # int8-only planes
])
def test_large_k_stays_on_block_keys(wv, oracle, metric, kind, n, d, k):
    """448 <= k < 960: the block-key path with 960-block candidate lists
    (qs_R = 16) instead of the all-rows replay; every query against the oracle."""
    data = gen(oracle, kind, 97, n, d)
    queries = gen(oracle, kind, 98, 24, d)
    idx, orc = build_pair(wv, oracle, metric, "avx256", data)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    route = wv._lib.ROUTES[idx.stats()["last_route"]]
    assert route in ("qs_bf16", "qs_w4", "qs_int8", "q8_gemv"), route
    for qi in range(len(queries)):
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"q{qi}")
    idx.close()
