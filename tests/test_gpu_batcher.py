"""GPU: the micro-batcher behind wv_index_search_by_vector.  Many threads each
search one query (as goroutines call flat.SearchByVector,
shard_read.go:415-424); every caller must get exactly the rows a batched
search (and the oracle) gives for its query, errors stay with their caller,
and concurrent calls share launches."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("metric,bq,n,d", [("cosine", False, 20000, 128), ("l2-squared", True, 8000, 256)])
def test_concurrent_single_queries_equal_batch(wv, oracle, metric, bq, n, d):
    data = oracle.gen_matrix(0, 61, 0, n, d)
    queries = oracle.gen_matrix(0, 62, 0, 96, d)
    kw = {"bq": True, "rescore_limit": 40} if bq else {}
    idx = wv.FlatIndex(distance=metric, variant="avx256", **kw)
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    idx.set_option("batch_window_us", 3000)
    allow = wv.AllowList(range(0, n, 3))
    ks = [10 if i % 3 else 7 for i in range(len(queries))]
    exp = {}
    for k in set(ks):
        ids, dists, counts = idx.search_by_vector_batch(queries, k)
        for q in range(len(queries)):
            if ks[q] == k:
                exp[q] = (ids[q, :counts[q]], dists[q, :counts[q]])
    ids_a, d_a, c_a = idx.search_by_vector_batch(queries[:8], 10, allow=allow)

    def one(i):
        if i < 8:
            return ("allow", i, idx.search_by_vector(queries[i], 10, allow=allow))
        if i == 8:
            try:
                idx.search_by_vector(np.ones(d + 1, np.float32), 10)
            except wv.WeaviateError as e:
                return ("err", i, str(e))
            return ("err", i, None)
        return ("plain", i, idx.search_by_vector(queries[i], ks[i]))

    with ThreadPoolExecutor(32) as ex:
        res = list(ex.map(one, range(len(queries))))
    for kind, i, r in res:
        if kind == "err":
            # the error the one-query call gives: ErrVectorLength, or for BQ the
            # hamming word-count check (distancer/hamming.go:63-68)
            assert r is not None and ("vector lengths don't match" in r or "should have the same len" in r)
            continue
        if kind == "allow":
            ei, ed = ids_a[i, :c_a[i]], d_a[i, :c_a[i]]
        else:
            ei, ed = exp[i]
        np.testing.assert_array_equal(r[0], ei, err_msg=f"{kind} q{i}")
        np.testing.assert_array_equal(r[1].view(np.uint32), ed.view(np.uint32), err_msg=f"{kind} q{i}")
    # the oracle agrees on a sample (the batched rows are oracle-checked elsewhere)
    M = oracle.METRIC[metric]
    orc = (oracle.OracleFlatBQ(M, 1, d, n, 40) if bq else oracle.OracleFlat(M, 1, d, n))
    orc.add_batch(np.arange(n, dtype=np.uint64), data)
    for kind, i, r in res[9:15]:
        rc, oi, od = orc.search(queries[i], ks[i])
        np.testing.assert_array_equal(r[0], oi)
    st = idx.batcher_stats()
    assert st["calls"] == len(queries)
    assert st["launches"] < st["calls"] and st["max_batch"] > 1, st
    idx.close()


def test_batcher_mixed_groups_isolate_errors(wv, oracle):
    """Mostly unfiltered callers, a few with their own lists and one with a
    malformed list (n_allow > 0, no ids) and one bad dimension, all sharing a
    window: the malformed caller fails alone before enqueueing, the bad
    dimension's launch is retried per caller, and every other caller gets the
    rows of its own one-query call (unfiltered callers never take
    the per-query-bitmap path)."""
    import ctypes as C
    n, d, k = 20000, 96, 10
    data = oracle.gen_matrix(1, 63, 0, n, d)
    queries = oracle.gen_matrix(1, 64, 0, 64, d)
    idx = wv.FlatIndex(distance="l2-squared", variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    idx.set_option("batch_window_us", 5000)
    rng = np.random.default_rng(2)
    lists = {i: wv.AllowList(rng.choice(n, 400, replace=False).tolist()) for i in range(0, 64, 16)}
    exp = {i: idx.search_by_vector_batch(queries[i:i + 1], k, allow=lists.get(i)) for i in range(64)}
    lib = wv.load()

    def one(i):
        if i == 5:  # malformed list: fails alone
            out_i = np.zeros(k, np.uint64)
            out_d = np.zeros(k, np.float32)
            cnt = C.c_int32(0)
            q = np.ascontiguousarray(queries[i])
            rc = lib.wv_index_search_by_vector(idx._h, q.ctypes.data_as(C.POINTER(C.c_float)), d, k, None, 7, 1,
                                               out_i.ctypes.data_as(C.POINTER(C.c_uint64)),
                                               out_d.ctypes.data_as(C.POINTER(C.c_float)), C.byref(cnt))
            return ("bad", i, rc)
        if i == 6:
            try:
                idx.search_by_vector(np.ones(d + 3, np.float32), k)
            except wv.WeaviateError as e:
                return ("err", i, str(e))
            return ("err", i, None)
        return ("ok", i, idx.search_by_vector(queries[i], k, allow=lists.get(i)))

    with ThreadPoolExecutor(64) as ex:
        res = list(ex.map(one, range(64)))
    for kind, i, r in res:
        if kind == "bad":
            assert r == wv._lib.WV_ERR_INVALID
        elif kind == "err":
            assert r is not None and "vector lengths don't match" in r
        else:
            ei, ed, ec = exp[i]
            np.testing.assert_array_equal(r[0], ei[0, :ec[0]], err_msg=f"q{i}")
            np.testing.assert_array_equal(r[1].view(np.uint32), ed[0, :ec[0]].view(np.uint32), err_msg=f"q{i}")
    idx.close()
