"""The dynamic index (adapters/repos/db/vector/dynamic/index.go) wired to the
engine: forwarding to the inner flat index below the threshold, the
upgradableIndexer answers, and the out-of-scope HNSW upgrade.  CPU tests cover
the control flow (no index is created); the GPU test checks that a dynamic
index returns exactly the flat index's (= the oracle's) results."""
import numpy as np
import pytest


def test_upgraded_state_unsupported(wv):
    # New (:177-208): an upgraded dynamic index opens HNSW, which is out of scope
    with pytest.raises(wv.WeaviateError, match="hnsw is not served"):
        wv.DynamicIndex(upgraded=True, distance="cosine")


class _Fake:
    def __init__(self, indexed, threshold=10, upgraded=False):
        self.n, self.t, self.u = indexed, threshold, upgraded

    def should_upgrade(self):
        return True, self.t

    def upgraded(self):
        return self.u

    def already_indexed(self):
        return self.n


@pytest.mark.parametrize("indexed,upgraded,expect", [(5, False, False), (10, False, False), (11, False, True),
                                                     (11, True, False)])
def test_queue_upgrade_trigger(indexed, upgraded, expect):  # vector_index_queue.go:263-290
    from weaviate_amd.dynamic import should_trigger_upgrade
    assert should_trigger_upgrade(_Fake(indexed, 10, upgraded)) is expect


@pytest.mark.gpu
@pytest.mark.parametrize("metric", ["cosine", "l2-squared"])
def test_dynamic_forwards_to_flat(wv, oracle, metric):
    n, d, k = 3000, 64, 10
    data = oracle.gen_matrix(1 if metric == "l2-squared" else 0, 71, 0, n, d)
    queries = oracle.gen_matrix(1 if metric == "l2-squared" else 0, 72, 0, 20, d)
    dyn = wv.DynamicIndex(threshold=2500, distance=metric, variant="avx256")
    assert dyn.type() == "dynamic" and dyn.underlying_index() == "flat" and not dyn.is_upgraded()
    dyn.add_batch(np.arange(n, dtype=np.uint64), data)
    dyn.delete(5, 17)
    orc = oracle.OracleFlat(oracle.METRIC[metric], 1, d, n)
    orc.add_batch(np.arange(n), data)
    orc.delete([5, 17])
    ids, dists, counts = dyn.search_by_vector_batch(queries, k)
    for i in range(len(queries)):
        rc, ei, ed = orc.search(queries[i], k)
        np.testing.assert_array_equal(ids[i, :counts[i]], ei)
        np.testing.assert_array_equal(dists[i, :counts[i]].view(np.uint32), ed.view(np.uint32))
    si, sd = dyn.search_by_vector(queries[0], k)
    np.testing.assert_array_equal(si, ids[0, :counts[0]])
    assert dyn.should_upgrade() == (True, 2500) and not dyn.upgraded()
    from weaviate_amd.dynamic import should_trigger_upgrade
    assert should_trigger_upgrade(dyn)  # AlreadyIndexed 3000 > 2500
    called = []
    with pytest.raises(wv.WeaviateError, match="hnsw is not served"):
        dyn.upgrade(lambda: called.append(1))
    assert called == [1]  # the queue's resume callback still runs
    ids2, _, _ = dyn.search_by_vector_batch(queries, k)  # still serving from the flat index
    np.testing.assert_array_equal(ids2, ids)
    assert dyn.contains_doc(3) and not dyn.contains_doc(5)
    assert dyn.compression_stats()["type"] == "none"
    dyn.update_user_config(threshold=5000)
    assert dyn.should_upgrade() == (True, 5000) and not should_trigger_upgrade(dyn)
    dyn.shutdown()
