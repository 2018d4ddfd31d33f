"""The rest of the db.VectorIndex surface on a flat index
(adapters/repos/db/vector_index.go:25-54): Iterate, QueryVectorDistancer,
Preload, UpdateUserConfig, CompressionStats -- through the C-ABI, against the
oracle (SingleDist / HammingBitwise restatements)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_iterate_ascending_and_early_stop(wv, oracle):
    idx = wv.FlatIndex(distance="l2-squared", id_base=0)
    ids = np.array([9, 3, 40, 7, 1000, 5], np.uint64)
    idx.add_batch(ids, oracle.gen_matrix(0, 1, 0, len(ids), 16))
    idx.delete(7)
    seen = []
    idx.iterate(lambda i: seen.append(i) or True)
    assert seen == [3, 5, 9, 40, 1000]
    seen = []
    idx.iterate(lambda i: seen.append(i) or len(seen) < 2)  # fn returning false stops the cursor
    assert seen == [3, 5]
    idx.close()


@pytest.mark.parametrize("metric,variant", [("cosine", "avx256"), ("l2-squared", "avx512"), ("dot", "avx256"),
                                            ("hamming", "avx256")])
def test_query_vector_distancer_equals_single_dist(wv, oracle, metric, variant):
    n, d = 500, 45
    data = oracle.gen_matrix(0, 3, 0, n, d)
    idx = wv.FlatIndex(distance=metric, variant=variant)
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    q = oracle.gen_matrix(0, 4, 0, 1, d)[0]
    M = oracle.METRIC[metric]
    v = {"avx256": 1, "avx512": 2}[variant]
    qq = oracle.normalize(q) if M == oracle.COSINE else q
    ids = np.array([0, 17, 499, 3, 17], np.uint64)
    got = idx.query_vector_distances(q, ids)
    for i, g in zip(ids, got):
        row = oracle.normalize(data[i]) if M == oracle.COSINE else data[i]
        e = np.float32(oracle.single_dist(M, v, qq, row))
        assert np.float32(g).view(np.uint32) == e.view(np.uint32)
    dist = idx.query_vector_distancer(q)
    assert np.float32(dist(17)).view(np.uint32) == np.float32(got[1]).view(np.uint32)
    # missing ids: the empty bucket value makes SingleDist fail (distancer ErrVectorLength)
    with pytest.raises(wv.WeaviateError, match=f"{d} vs 0: vector lengths don't match"):
        idx.query_vector_distances(q, [n + 5])
    idx.delete(3)
    out, rc = idx.query_vector_distances(q, [3, 0], per_id_status=True)
    assert rc[0] != 0 and rc[1] == 0 and out[1] == got[0]
    with pytest.raises(wv.WeaviateError, match="vector lengths don't match"):
        idx.query_vector_distances(q[:-1], [0])
    idx.close()


def test_query_vector_distancer_bq_cache(wv, oracle):
    n, d = 300, 130
    data = oracle.gen_matrix(0, 5, 0, n, d)
    q = oracle.gen_matrix(0, 6, 0, 1, d)[0]
    ids = np.array([1, 2, 299], np.uint64)
    # BQ without the cache: fp32 SingleDist of the stored row (defaultDistFunc)
    idx = wv.FlatIndex(distance="cosine", bq=True)
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    got = idx.query_vector_distances(q, ids)
    qn = oracle.normalize(q)
    exp = [oracle.single_dist(oracle.COSINE, 1, qn, oracle.normalize(data[i])) for i in ids]
    np.testing.assert_array_equal(got.view(np.uint32), np.float32(exp).view(np.uint32))
    # with the cache: HammingBitwise(code, query code)
    idx.set_option("cache", 1)
    got = idx.query_vector_distances(q, ids)
    qc = oracle.bq_encode(qn)
    exp = [oracle.hamming_bitwise(oracle.bq_encode(oracle.normalize(data[i])), qc) for i in ids]
    np.testing.assert_array_equal(got, np.float32(exp))
    with pytest.raises(wv.WeaviateError, match="is larger than the cache size"):
        idx.query_vector_distances(q, [n + 100])
    idx.close()


def test_preload_compressed_only(wv, oracle):
    d = 64
    rows = oracle.gen_matrix(0, 7, 0, 4, d)
    plain = wv.FlatIndex(distance="l2-squared")
    plain.add(0, rows[0])
    plain.preload(1, rows[1])  # uncompressed: Preload does nothing
    assert not plain.contains_doc(1) and plain.already_indexed() == 1
    plain.close()
    bq = wv.FlatIndex(distance="l2-squared", bq=True, rescore_limit=10)
    bq.add(0, rows[0])
    bq.preload(1, rows[1])  # compressed: the code is stored, AlreadyIndexed unchanged
    assert bq.contains_doc(1) and bq.already_indexed() == 1
    ids, dists = bq.search_by_vector(rows[1], 1)
    assert ids[0] == 1
    bq.close()


def test_update_user_config_rescore_and_immutables(wv, oracle):
    n, d, k = 4000, 64, 5
    data = oracle.gen_matrix(0, 8, 0, n, d)
    queries = oracle.gen_matrix(0, 9, 0, 6, d)
    idx = wv.FlatIndex(distance="cosine", variant="avx256", bq=True, rescore_limit=k)
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    idx.update_user_config(rescore_limit=150)
    orc = oracle.OracleFlatBQ(oracle.COSINE, 1, d, n, 150)
    orc.add_batch(np.arange(n), data)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    for qi in range(len(queries)):
        rc, oi, od = orc.search(queries[qi], k)
        np.testing.assert_array_equal(ids[qi, :counts[qi]], oi)
        np.testing.assert_array_equal(dists[qi, :counts[qi]].view(np.uint32), od.view(np.uint32))
    with pytest.raises(wv.WeaviateError, match='distance is immutable: attempted change from "cosine" to "dot"'):
        idx.update_user_config(distance="dot")
    with pytest.raises(wv.WeaviateError, match='bq is immutable: attempted change from "true" to "false"'):
        idx.update_user_config(bq=False)
    assert idx.compression_stats() == {"type": "none", "ratio": 1.0}
    idx.close()
