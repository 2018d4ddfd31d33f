"""GPU: the block-key route for k >= 960 (1984- and 4032-block candidate
lists, k_blk_select<32/64> / k_blk_exact<32/64>).  The reference limits a
search only by QUERY_MAXIMUM_RESULTS (usecases/config/environment.go:625-633);
results must equal the oracle's heap (flat/index.go:578-688) bit for bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("metric,n,d,k", [
    ("cosine", 150000, 128, 1000),
    ("l2-squared", 150000, 768, 2000),
    ("dot", 120000, 96, 3000),
    ("cosine", 100000, 768, 1500),
])
def test_large_k_block_key_route_equals_oracle(wv, oracle, metric, n, d, k):
    data = oracle.gen_matrix(0, 81, 0, n, d)
    queries = oracle.gen_matrix(0, 82, 0, 20, d)
    idx = wv.FlatIndex(distance=metric, variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    deleted = list(range(3, n, 211))
    idx.delete(*deleted)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    st = idx.stats()
    assert wv._lib.ROUTES[st["last_route"]].startswith(("qs_", "q8_")), st
    orc = oracle.OracleFlat(oracle.METRIC[metric], 1, d, n)
    orc.add_batch(np.arange(n, dtype=np.uint64), data)
    orc.delete(deleted)
    for i in range(len(queries)):
        rc, oi, od = orc.search(queries[i], k)
        assert counts[i] == len(oi) == k
        np.testing.assert_array_equal(ids[i, :counts[i]], oi, err_msg=f"q{i}")
        np.testing.assert_array_equal(dists[i, :counts[i]].view(np.uint32), od.view(np.uint32), err_msg=f"q{i}")
    # an allow list and a batch of per-query lists at the same k
    allow = wv.AllowList(range(0, n, 2))
    ids_a, d_a, c_a = idx.search_by_vector_batch(queries[:4], k, allow=allow)
    ids_m, d_m, c_m = idx.search_by_vector_batch_multi_allow(queries[:4], k, [allow, None, allow, None])
    for i in range(4):
        rc, oi, od = orc.search(queries[i], k, [int(x) for x in allow.ids])
        np.testing.assert_array_equal(ids_a[i, :c_a[i]], oi, err_msg=f"allow q{i}")
        if i % 2 == 0:
            np.testing.assert_array_equal(ids_m[i, :c_m[i]], oi, err_msg=f"multi q{i}")
        else:
            np.testing.assert_array_equal(ids_m[i, :c_m[i]], ids[i, :counts[i]], err_msg=f"multi q{i}")
    idx.close()
