"""GPU: per-query allow lists in one batch
(wv_index_search_by_vector_batch_multi_allow).  Weaviate's concurrent callers
each bring their own filter (shard_read.go:415-424 -> flat/index.go:423-448,
helpers.AllowList per call); the batch must give every query exactly what a
one-query search under its own list gives (and the oracle), with one
block-key launch for the whole batch: keys over the lists' union, the exact
pass and the replays over each query's own bitmap."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _allow_lists(wv, n, nq, k, seed):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(nq):
        kind = i % 9
        if kind == 0:
            out.append(None)
        elif kind == 1:  # sparse, some ids past the store
            out.append(wv.AllowList(rng.integers(0, n + 500, 40)))
        elif kind == 2:  # dense half
            out.append(wv.AllowList(np.flatnonzero(rng.random(n) < 0.5)))
        elif kind == 3:  # one contiguous span
            a = int(rng.integers(0, n - 3000))
            out.append(wv.AllowList(range(a, a + 3000)))
        elif kind == 4:  # empty: no results (flat/index.go:590-594)
            out.append(wv.AllowList())
        elif kind == 5:
            out.append(wv.AllowList(range(i % 7, n, 7)))
        elif kind == 6:  # fewer rows than k
            out.append(wv.AllowList(rng.integers(0, n, max(1, k // 2))))
        elif kind == 7:  # a handful of neighbouring blocks
            a = int(rng.integers(0, n - 200))
            out.append(wv.AllowList(range(a, a + k + 3)))
        else:  # every other block of 32 rows
            out.append(wv.AllowList([j for j in range(n) if (j >> 5) % 2 == i % 2]))
    return out


@pytest.mark.parametrize("metric,n,d,k,nq", [
    ("cosine", 20000, 128, 10, 54),
    ("l2-squared", 30000, 96, 32, 45),
    ("dot", 12000, 256, 5, 36),
    ("cosine", 20000, 768, 10, 300),
])
def test_multi_allow_equals_one_query_calls(wv, oracle, metric, n, d, k, nq):
    data = oracle.gen_matrix(0, 71, 0, n, d)
    queries = oracle.gen_matrix(0, 72, 0, nq, d)
    idx = wv.FlatIndex(distance=metric, variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    deleted = list(range(5, n, 97))
    idx.delete(*deleted)
    allows = _allow_lists(wv, n, nq, k, seed=n + d)
    # every list in the shared launch (no sparse list searched alone, the
    # unresolved ones replayed inside it)
    idx.set_option("pqa_split_max", 0)
    idx.set_option("pqa_alone", 0)
    b0 = idx.stats()["batches"]
    ids, dists, counts = idx.search_by_vector_batch_multi_allow(queries, k, allows)
    st = idx.stats()
    assert st["batches"] - b0 == 1, "the batch must share one launch"
    assert wv._lib.ROUTES[st["last_route"]].startswith(("qs_", "q8_")), st
    # default: the sparsest lists alone, the rest shared, the unresolved ones
    # searched alone afterwards -- the same rows
    idx.set_option("pqa_split_max", 64)
    idx.set_option("pqa_alone", 1)
    ids2, dists2, counts2 = idx.search_by_vector_batch_multi_allow(queries, k, allows)
    np.testing.assert_array_equal(counts2, counts)
    for i in range(nq):
        np.testing.assert_array_equal(ids2[i, :counts[i]], ids[i, :counts[i]], err_msg=f"q{i}")
        np.testing.assert_array_equal(dists2[i, :counts[i]].view(np.uint32), dists[i, :counts[i]].view(np.uint32))
    for i in range(nq):
        ei, ed, ec = idx.search_by_vector_batch(queries[i:i + 1], k, allow=allows[i])
        assert counts[i] == ec[0], f"q{i}"
        np.testing.assert_array_equal(ids[i, :counts[i]], ei[0, :ec[0]], err_msg=f"q{i}")
        np.testing.assert_array_equal(dists[i, :counts[i]].view(np.uint32), ed[0, :ec[0]].view(np.uint32),
                                      err_msg=f"q{i}")
        if i % 9 == 4:
            assert counts[i] == 0
    # the oracle on a sample of every list kind
    orc = oracle.OracleFlat(oracle.METRIC[metric], 1, d, n)
    orc.add_batch(np.arange(n, dtype=np.uint64), data)
    orc.delete(deleted)
    for i in range(min(nq, 18)):
        al = None if allows[i] is None else [int(x) for x in allows[i].ids]
        rc, oi, od = orc.search(queries[i], k, al)
        np.testing.assert_array_equal(ids[i, :counts[i]], oi, err_msg=f"q{i}")
        np.testing.assert_array_equal(dists[i, :counts[i]].view(np.uint32), od.view(np.uint32), err_msg=f"q{i}")
    idx.close()


def test_multi_allow_fallback_routes_and_errors(wv, oracle):
    """BQ has no shared-launch form: the batch is grouped by identical list and
    still equals the one-query calls; bad arguments are rejected."""
    n, d, k = 6000, 64, 8
    data = oracle.gen_matrix(0, 73, 0, n, d)
    queries = oracle.gen_matrix(0, 74, 0, 12, d)
    idx = wv.FlatIndex(distance="l2-squared", variant="avx256", bq=True, rescore_limit=40)
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    common = wv.AllowList(range(0, n, 2))
    allows = [None, common, wv.AllowList(range(100, 900)), common] * 3
    ids, dists, counts = idx.search_by_vector_batch_multi_allow(queries, k, allows)
    for i in range(len(queries)):
        ei, ed, ec = idx.search_by_vector_batch(queries[i:i + 1], k, allow=allows[i])
        assert counts[i] == ec[0]
        np.testing.assert_array_equal(ids[i, :counts[i]], ei[0, :ec[0]])
        np.testing.assert_array_equal(dists[i, :counts[i]].view(np.uint32), ed[0, :ec[0]].view(np.uint32))
    with pytest.raises(wv.WeaviateError):
        idx.search_by_vector_batch_multi_allow(queries, k, allows[:-1])
    with pytest.raises(wv.WeaviateError, match="vector lengths don't match|same len"):
        idx.search_by_vector_batch_multi_allow(np.ones((3, d + 1), np.float32), k, [None, common, None])
    idx.close()


def test_batcher_coalesces_distinct_allow_lists(wv, oracle):
    """concurrent callers with their own allow lists share launches and each
    gets its one-query result"""
    n, d, k = 20000, 128, 10
    data = oracle.gen_matrix(0, 75, 0, n, d)
    queries = oracle.gen_matrix(0, 76, 0, 64, d)
    idx = wv.FlatIndex(distance="cosine", variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    idx.set_option("batch_window_us", 3000)
    allows = _allow_lists(wv, n, len(queries), k, seed=5)
    exp = [idx.search_by_vector_batch(queries[i:i + 1], k, allow=allows[i]) for i in range(len(queries))]
    # three rounds in different orders: the callers' pooled bitmap rows are
    # reused by other callers (stale rows would give another caller's list)
    rng = np.random.default_rng(3)
    for rnd in range(3):
        order = rng.permutation(len(queries)) if rnd else np.arange(len(queries))
        with ThreadPoolExecutor(32) as ex:
            res = dict(zip(order, ex.map(lambda i: idx.search_by_vector(queries[i], k, allow=allows[i]), order)))
        for i in range(len(queries)):
            ri, rd = res[i]
            ei, ed, ec = exp[i]
            np.testing.assert_array_equal(ri, ei[0, :ec[0]], err_msg=f"round {rnd} q{i}")
            np.testing.assert_array_equal(rd.view(np.uint32), ed[0, :ec[0]].view(np.uint32), err_msg=f"round {rnd} q{i}")
    st = idx.batcher_stats()
    assert st["launches"] < st["calls"] and st["max_batch"] > 1, st
    idx.close()


@pytest.mark.parametrize("opts,k,nq", [({"pqa_budget_mb": 1}, 10, 200),     # bitmap budget: sub-batches (offsets q0 * k)
                                       ({"sel_lower": 1}, 10, 64),           # the select's lowered thresholds
                                       ({}, 1000, 24),                       # k > 959: 1984-block lists, R = 32
                                       ({"pqa_split_max": 0, "pqa_alone": 0}, 300, 40)])
def test_multi_allow_option_paths_equal_one_query_calls(wv, oracle, opts, k, nq):
    """The multi-allow paths ADVICE r5 listed as untested: the per-query bitmap
    budget's sub-batch recursion, sel_lower = 1, large k with per-query
    bitmaps; each against the one-query calls."""
    n, d = 30000, 128
    data = oracle.gen_matrix(1, 73, 0, n, d)  # integer data: ties, replays
    queries = oracle.gen_matrix(1, 74, 0, nq, d)
    idx = wv.FlatIndex(distance="l2-squared", variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    for kk, vv in opts.items():
        idx.set_option(kk, vv)
    allows = _allow_lists(wv, n, nq, min(k, 64), seed=7 + k)
    ids, dists, counts = idx.search_by_vector_batch_multi_allow(queries, k, allows)
    for i in range(nq):
        ei, ed, ec = idx.search_by_vector_batch(queries[i:i + 1], k, allow=allows[i])
        assert counts[i] == ec[0], f"q{i}"
        np.testing.assert_array_equal(ids[i, :counts[i]], ei[0, :ec[0]], err_msg=f"q{i}")
        np.testing.assert_array_equal(dists[i, :counts[i]].view(np.uint32), ed[0, :ec[0]].view(np.uint32),
                                      err_msg=f"q{i}")
    idx.close()


@pytest.mark.parametrize("id_base,opts,k,nq", [(0, {}, 10, 54),
                                               (1000013, {}, 10, 45),                       # unaligned shard base
                                               (64, {"pqa_split_max": 0, "pqa_alone": 0}, 32, 40),
                                               (0, {"pqa_budget_mb": 1}, 10, 120),           # sub-batches: via lists
                                               (0, {}, 300, 30)])
def test_multi_allow_bitmap_form_equals_id_lists(wv, oracle, id_base, opts, k, nq):
    """wv_index_search_by_vector_batch_multi_allow_bitmap: the same lists as
    dense doc-id bitmaps give the id-list call's rows (and the oracle's), on an
    index whose doc ids start at id_base (a shard): the bitmap words are read
    from id_base on with the bit shift id_base % 32."""
    n, d = 20000, 128
    data = oracle.gen_matrix(1, 81, 0, n, d)  # integer data: ties
    queries = oracle.gen_matrix(1, 82, 0, nq, d)
    idx = wv.FlatIndex(distance="l2-squared", variant="avx256", id_base=id_base)
    idx.add_batch(np.arange(id_base, id_base + n, dtype=np.uint64), data)
    idx.delete(*range(id_base + 3, id_base + n, 101))
    for kk, vv in opts.items():
        idx.set_option(kk, vv)
    base = _allow_lists(wv, n, nq, min(k, 64), seed=11 + k)
    allows = [None if a is None else wv.AllowList(a.ids.astype(np.uint64) + np.uint64(id_base)) for a in base]
    ids, dists, counts = idx.search_by_vector_batch_multi_allow(queries, k, allows)
    bi, bd, bc = idx.search_by_vector_batch_multi_allow(queries, k, allows, bitmap=True)
    np.testing.assert_array_equal(bc, counts)
    for i in range(nq):
        np.testing.assert_array_equal(bi[i, :counts[i]], ids[i, :counts[i]], err_msg=f"q{i}")
        np.testing.assert_array_equal(bd[i, :counts[i]].view(np.uint32), dists[i, :counts[i]].view(np.uint32),
                                      err_msg=f"q{i}")
    orc = oracle.OracleFlat(oracle.METRIC["l2-squared"], 1, d, n)
    orc.add_batch(np.arange(n, dtype=np.uint64), data)
    orc.delete(list(range(3, n, 101)))
    for i in range(min(nq, 12)):
        al = None if base[i] is None else [int(x) for x in base[i].ids]
        rc, oi, od = orc.search(queries[i], k, al)
        np.testing.assert_array_equal(bi[i, :bc[i]], oi.astype(np.uint64) + np.uint64(id_base), err_msg=f"q{i}")
        np.testing.assert_array_equal(bd[i, :bc[i]].view(np.uint32), od.view(np.uint32), err_msg=f"q{i}")
    idx.close()


@pytest.mark.parametrize("metric,kind,d,k,nq", [("cosine", 0, 768, 10, 300),
                                               ("dot", 1, 512, 10, 100),     # integer data: ties, replays
                                               ("cosine", 1, 640, 32, 64),
                                               ("dot", 0, 768, 1, 40)])
def test_multi_allow_per_query_keys_equal_union_keys(wv, oracle, metric, kind, d, k, nq):
    """Per-query masked int8 keys (k_q8_blockkey<.., MASK>, option pqa_keys = 1,
    the default for dot / cosine at 384 < d <= 768) against the union's keys
    with per-query thresholds (pqa_keys = 0), the one-query calls and the
    oracle: ids, distance bits and tie order."""
    n = 24000
    data = oracle.gen_matrix(kind, 91, 0, n, d)
    queries = oracle.gen_matrix(kind, 92, 0, nq, d)
    idx = wv.FlatIndex(distance=metric, variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    idx.delete(*range(9, n, 89))
    allows = _allow_lists(wv, n, nq, k, seed=d + k)
    ids, dists, counts = idx.search_by_vector_batch_multi_allow(queries, k, allows)
    assert wv._lib.ROUTES[idx.stats()["last_route"]] == "qs_int8", idx.stats()
    bi, bd, bc = idx.search_by_vector_batch_multi_allow(queries, k, allows, bitmap=True)
    idx.set_option("pqa_keys", 0)
    ui, ud, uc = idx.search_by_vector_batch_multi_allow(queries, k, allows)
    for other in ((bi, bd, bc), (ui, ud, uc)):
        np.testing.assert_array_equal(other[2], counts)
        for i in range(nq):
            np.testing.assert_array_equal(other[0][i, :counts[i]], ids[i, :counts[i]], err_msg=f"q{i}")
            np.testing.assert_array_equal(other[1][i, :counts[i]].view(np.uint32), dists[i, :counts[i]].view(np.uint32),
                                          err_msg=f"q{i}")
    for i in range(0, nq, max(1, nq // 24)):
        ei, ed, ec = idx.search_by_vector_batch(queries[i:i + 1], k, allow=allows[i])
        assert counts[i] == ec[0], f"q{i}"
        np.testing.assert_array_equal(ids[i, :counts[i]], ei[0, :ec[0]], err_msg=f"q{i}")
        np.testing.assert_array_equal(dists[i, :counts[i]].view(np.uint32), ed[0, :ec[0]].view(np.uint32))
    orc = oracle.OracleFlat(oracle.METRIC[metric], 1, d, n)
    orc.add_batch(np.arange(n, dtype=np.uint64), data)
    orc.delete(list(range(9, n, 89)))
    for i in range(min(nq, 12)):
        al = None if allows[i] is None else [int(x) for x in allows[i].ids]
        rc, oi, od = orc.search(queries[i], k, al)
        np.testing.assert_array_equal(ids[i, :counts[i]], oi, err_msg=f"q{i}")
        np.testing.assert_array_equal(dists[i, :counts[i]].view(np.uint32), od.view(np.uint32), err_msg=f"q{i}")
    idx.close()
