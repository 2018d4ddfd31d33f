"""GPU: int8 block keys above 3072 dims (k_q8_blockkey_cp with 4-6 column
parts of 1024 columns, 64-query workgroups).  The reference accepts any
dimension (flat/index.go:823-842); results must equal the oracle's heap
(flat/index.go:578-688) bit for bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("metric,n,d,k,nq", [
    ("cosine", 40000, 4096, 10, 70),
    ("l2-squared", 30000, 6144, 25, 40),
    ("dot", 30000, 5000, 10, 130),
    ("cosine", 20000, 3500, 100, 20),
    ("l2-squared", 25000, 4096, 1000, 12),
])
def test_wide_int8_keys_equal_oracle(wv, oracle, metric, n, d, k, nq):
    data = oracle.gen_matrix(0, 91, 0, n, d)
    queries = oracle.gen_matrix(0, 92, 0, nq, d)
    idx = wv.FlatIndex(distance=metric, variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    deleted = list(range(7, n, 173))
    idx.delete(*deleted)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    st = idx.stats()
    assert wv._lib.ROUTES[st["last_route"]] == "qs_int8", st
    orc = oracle.OracleFlat(oracle.METRIC[metric], 1, d, n)
    orc.add_batch(np.arange(n, dtype=np.uint64), data)
    orc.delete(deleted)
    for i in range(min(nq, 16)):
        rc, oi, od = orc.search(queries[i], k)
        assert counts[i] == len(oi) == k
        np.testing.assert_array_equal(ids[i, :counts[i]], oi, err_msg=f"q{i}")
        np.testing.assert_array_equal(dists[i, :counts[i]].view(np.uint32), od.view(np.uint32), err_msg=f"q{i}")
    # the rest of the batch against one-query calls (other query groups / spans)
    for i in range(16, nq, 9):
        ei, ed, ec = idx.search_by_vector_batch(queries[i:i + 1], k)
        np.testing.assert_array_equal(ids[i, :counts[i]], ei[0, :ec[0]], err_msg=f"q{i}")
    allow = wv.AllowList(range(1, n, 3))
    ia, da, ca = idx.search_by_vector_batch(queries[:3], k, allow=allow)
    for i in range(3):
        rc, oi, od = orc.search(queries[i], k, [int(x) for x in allow.ids])
        np.testing.assert_array_equal(ia[i, :ca[i]], oi, err_msg=f"allow q{i}")
    idx.close()
