"""GPU: the multi-shard index (wv_multi, multi.hip) over compressed shards and
under allow lists -- configs[3]'s BQ search, the quantized searches (trained
PQ, SQ, rq-8 / rq-1), per-shard allow lists (shard_read.go:401-413 -> flat
SearchByVector(..., allowList)), per-query lists and SearchByVectorDistance
across shards (shard_read.go:439, merged by index.go:2067-2071).  The shards
share the one GPU of the box (local transport).  Every result must equal one
flat index over the whole corpus (ids, distance bits, tie order) and, where
the oracle restates the path, the oracle's reference heap."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _assert_equal(got, exp, tag=""):
    gi, gd, gn = got
    ei, ed, en = exp
    np.testing.assert_array_equal(gn, en, err_msg=f"{tag} counts")
    for i in range(len(gn)):
        np.testing.assert_array_equal(gi[i, :gn[i]], ei[i, :en[i]], err_msg=f"{tag} q{i} ids")
        np.testing.assert_array_equal(gd[i, :gn[i]].view(np.uint32), ed[i, :en[i]].view(np.uint32),
                                      err_msg=f"{tag} q{i} dists")


def _multi(shards, per, **kw):
    from weaviate_amd.multi import MultiFlatIndex
    return MultiFlatIndex(devices=[0] * shards, id_stride=per, transport="local", variant="avx256", **kw)


# par: every shard holds >= R block minima (32-row blocks on the integer MFMA
# route, 7..24 code words; 256-row blocks below), so the R-th smallest bound of
# the shards before r is finite and the parallel R-heap resolves every query;
# smaller shards bound nothing and take the serial chain (same result)
@pytest.mark.parametrize("shards,metric,kind,n,d,k,rl,par", [(3, "cosine", 0, 156000, 1536, 10, 40, True),  # C4's width
                                                            (4, "l2-squared", 0, 80000, 256, 10, 16, True),
                                                            (2, "cosine", 0, 16000, 1536, 10, 200, False),
                                                            (3, "l2-squared", 1, 9000, 96, 10, 200, False),
                                                            (5, "dot", 0, 10000, 128, 7, 40, False),
                                                            (8, "cosine", 1, 16000, 256, 10, 200, False)])
def test_multi_bq_equals_single_index_and_oracle(wv, oracle, shards, metric, kind, n, d, k, rl, par):
    data = oracle.gen_matrix(kind, 61, 0, n, d)
    queries = oracle.gen_matrix(kind, 62, 0, 96, d)
    per = (n + shards - 1) // shards
    m = _multi(shards, per, distance=metric, dims=d, bq=True, rescore_limit=rl)
    m.add_batch(np.arange(n, dtype=np.uint64), data)
    got = m.search_by_vector_batch(queries, k)
    st = m.stats()
    if par:
        assert st["last_overflowed"] == 0 and st["chain_hops"] == 0  # the parallel R-heap
    single = wv.FlatIndex(distance=metric, bq=True, rescore_limit=rl, variant="avx256")
    single.add_batch(np.arange(n, dtype=np.uint64), data)
    _assert_equal(got, single.search_by_vector_batch(queries, k), "single")
    orc = oracle.OracleFlatBQ(oracle.METRIC[metric], 1, d, n, rl)
    orc.add_batch(np.arange(n), data)
    for i in range(0, len(queries), 9):
        rc, ei, ed = orc.search(queries[i], k)
        assert rc == 0 and got[2][i] == len(ei)
        np.testing.assert_array_equal(got[0][i, :got[2][i]], ei, err_msg=f"q{i} vs oracle")
        np.testing.assert_array_equal(got[1][i, :got[2][i]].view(np.uint32), ed.view(np.uint32))
    # the serial chain (what an overflowed record takes): same result
    m.set_option("chain", 1)
    got2 = m.search_by_vector_batch(queries, k)
    assert m.stats()["chain_hops"] >= st["chain_hops"] + shards
    _assert_equal(got2, got, "chain")
    single.close()
    m.close()


@pytest.mark.parametrize("comp,shards,metric,kind,per,d,k,rl,rescore", [
    ("pq", 3, "l2-squared", 0, 4000, 32, 10, -1, False),   # worker heap = k
    ("pq", 2, "cosine", 0, 5000, 64, 10, 60, True),        # rescoring: the owners' exact distances
    ("pq", 4, "l2-squared", 1, 2500, 24, 7, 40, True),     # integer data: ADC ties
    ("sq", 3, "l2-squared", 0, 4000, 48, 10, 20, True),    # SQ: ef limit, trim to the rescore limit
    ("rq8", 3, "cosine", 0, 4000, 64, 10, 30, True),       # flat rq-8: searchByVectorQuantized
    ("rq1", 2, "l2-squared", 1, 5000, 64, 10, 40, True),   # flat rq-1, integer data
])
def test_multi_quant_equals_single_index(wv, oracle, comp, shards, metric, kind, per, d, k, rl, rescore):
    n = per * shards
    data = oracle.gen_matrix(kind, 71, 0, n, d)
    queries = oracle.gen_matrix(kind, 72, 0, 80, d)
    kw = dict(distance=metric, rescore_limit=rl)
    if comp == "pq":
        kw["pq"] = {"segments": d // 4, "centroids": 32, "trainingLimit": 100000, "rescore": rescore}
    elif comp == "sq":
        kw["sq"] = True
    else:
        kw["rq"] = {"bits": 8 if comp == "rq8" else 1}
    single = wv.FlatIndex(variant="avx256", **kw)
    single.add_batch(np.arange(n, dtype=np.uint64), data)
    m = _multi(shards, per, dims=d, **kw)
    m.add_batch(np.arange(n, dtype=np.uint64), data)
    if comp == "pq":
        single.pq_fit(seed=5)
        m.pq_fit(seed=5)  # the first trainingLimit rows gathered from the shards in id order
        for s in m.shards:
            np.testing.assert_array_equal(s.pq_centers().view(np.uint32), single.pq_centers().view(np.uint32))
    elif comp == "sq":
        single.sq_fit(2000)
        info = single.sq_info()
        for s in m.shards:
            s.sq_restore(info["a"], info["b"])
    exp = single.search_by_vector_batch(queries, k)
    _assert_equal(m.search_by_vector_batch(queries, k), exp, comp)
    m.set_option("chain", 1)
    _assert_equal(m.search_by_vector_batch(queries, k), exp, comp + " chain")
    assert m.stats()["chain_hops"] >= shards
    single.close()
    m.close()


def _allow_cases(n, per, rng):
    return {
        "10pct": np.sort(rng.choice(n, n // 10, replace=False)),
        "sparse": np.sort(rng.choice(n, 150, replace=False)),
        "one_shard": np.arange(per + 3, 2 * per - 5, 2),
        "empty_shards": np.arange(0, per // 2),
    }


@pytest.mark.parametrize("comp,shards,metric,kind,n,d,k", [("none", 4, "cosine", 0, 16000, 768, 10),
                                                          ("none", 3, "l2-squared", 1, 9000, 64, 10),
                                                          ("bq", 3, "cosine", 1, 9000, 256, 10),
                                                          ("rq8", 2, "dot", 0, 8000, 64, 10)])
def test_multi_allow_lists_equal_single_index(wv, oracle, comp, shards, metric, kind, n, d, k):
    """One allow list per batch: each shard searches under its part of it."""
    data = oracle.gen_matrix(kind, 81, 0, n, d)
    queries = oracle.gen_matrix(kind, 82, 0, 64, d)
    per = (n + shards - 1) // shards
    kw = dict(distance=metric)
    if comp == "bq":
        kw.update(bq=True, rescore_limit=100)
    elif comp == "rq8":
        kw.update(rq={"bits": 8}, rescore_limit=50)
    m = _multi(shards, per, dims=d, **kw)
    m.add_batch(np.arange(n, dtype=np.uint64), data)
    single = wv.FlatIndex(variant="avx256", **kw)
    single.add_batch(np.arange(n, dtype=np.uint64), data)
    rng = np.random.default_rng(5)
    for name, ids in _allow_cases(n, per, rng).items():
        allow = wv.AllowList(ids.tolist())
        _assert_equal(m.search_by_vector_batch(queries, k, allow=allow),
                      single.search_by_vector_batch(queries, k, allow=allow), name)
    # the empty list finds nothing; unfiltered afterwards: the shards' own present bitmaps are back
    got = m.search_by_vector_batch(queries, k, allow=wv.AllowList([]))
    assert (got[2] == 0).all()
    _assert_equal(m.search_by_vector_batch(queries, k), single.search_by_vector_batch(queries, k), "after")
    if comp == "none":
        orc = oracle.OracleFlat(oracle.METRIC[metric], 1, d, n)
        orc.add_batch(np.arange(n), data)
        ids = _allow_cases(n, per, np.random.default_rng(5))["10pct"]
        got = m.search_by_vector_batch(queries, k, allow=wv.AllowList(ids.tolist()))
        for i in range(0, len(queries), 13):
            rc, ei, ed = orc.search(queries[i], k, allow=ids)
            assert rc == 0 and got[2][i] == len(ei)
            np.testing.assert_array_equal(got[0][i, :got[2][i]], ei, err_msg=f"q{i} vs oracle")
    single.close()
    m.close()


def test_multi_per_query_allow_lists_and_device_call(wv, oracle):
    n, d, k, shards = 12000, 128, 10, 3
    per = n // shards
    data = oracle.gen_matrix(1, 83, 0, n, d)
    queries = oracle.gen_matrix(1, 84, 0, 40, d)
    m = _multi(shards, per, distance="l2-squared", dims=d)
    m.add_batch(np.arange(n, dtype=np.uint64), data)
    single = wv.FlatIndex(distance="l2-squared", variant="avx256")
    single.add_batch(np.arange(n, dtype=np.uint64), data)
    rng = np.random.default_rng(9)
    pool = [None, wv.AllowList(rng.choice(n, 500, replace=False).tolist()),
            wv.AllowList(rng.choice(n, 3000, replace=False).tolist()), wv.AllowList([]),
            wv.AllowList(np.arange(2 * per, n).tolist())]
    allows = [pool[i % len(pool)] for i in range(len(queries))]
    _assert_equal(m.search_by_vector_batch_multi_allow(queries, k, allows),
                  single.search_by_vector_batch_multi_allow(queries, k, allows), "multi_allow")
    # the device form on a caller stream
    dev = torch.device("cuda", 0)
    q = torch.from_numpy(queries).to(dev)
    oi = torch.empty((len(queries), k), dtype=torch.int64, device=dev)
    od = torch.empty((len(queries), k), dtype=torch.float32, device=dev)
    on = torch.empty(len(queries), dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        m.search_device(q.data_ptr(), len(queries), d, k, oi.data_ptr(), od.data_ptr(), on.data_ptr(), s.cuda_stream,
                        allow=pool[2])
    s.synchronize()
    _assert_equal((oi.cpu().numpy().view(np.uint64), od.cpu().numpy(), on.cpu().numpy()),
                  single.search_by_vector_batch(queries, k, allow=pool[2]), "device")
    single.close()
    m.close()


@pytest.mark.parametrize("metric,kind,comp", [("l2-squared", 1, "none"), ("cosine", 0, "none"), ("cosine", 0, "bq")])
def test_multi_search_by_vector_distance(wv, oracle, metric, kind, comp):
    n, d, shards = 9000, 64, 3
    per = n // shards
    data = oracle.gen_matrix(kind, 85, 0, n, d)
    queries = oracle.gen_matrix(kind, 86, 0, 12, d)
    kw = dict(distance=metric)
    if comp == "bq":
        kw.update(bq=True, rescore_limit=150)
    m = _multi(shards, per, dims=d, **kw)
    m.add_batch(np.arange(n, dtype=np.uint64), data)
    single = wv.FlatIndex(variant="avx256", **kw)
    single.add_batch(np.arange(n, dtype=np.uint64), data)
    allow = wv.AllowList(np.arange(100, n, 3).tolist())
    for i, qv in enumerate(queries):
        ids, dd, _ = single.search_by_vector_batch(qv[None, :], 100)
        target = float(dd[0, 40])  # about 40 rows within reach
        for a in (None, allow):
            ge = single.search_by_vector_distance(qv, target, 1000, allow=a)
            gm = m.search_by_vector_distance(qv, target, 1000, allow=a)
            np.testing.assert_array_equal(gm[0], ge[0], err_msg=f"q{i}")
            np.testing.assert_array_equal(gm[1].view(np.uint32), ge[1].view(np.uint32))
    single.close()
    m.close()


def test_multi_add_batch_validates_before_inserting(wv, oracle):
    """A failed AddBatch leaves no shard partially updated."""
    n, d, shards = 3000, 32, 3
    per = n // shards
    m = _multi(shards, per, distance="l2-squared", dims=d)
    data = oracle.gen_matrix(0, 87, 0, n, d)
    m.add_batch(np.arange(0, n, 2, dtype=np.uint64), data[::2])
    before = [s.already_indexed() for s in m.shards]
    with pytest.raises(wv.WeaviateError):
        m.add_batch(np.array([1, per + 1], dtype=np.uint64), np.zeros((2, d + 1), np.float32))
    assert [s.already_indexed() for s in m.shards] == before
    m.close()
