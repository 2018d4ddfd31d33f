"""GPU: restore a flat index from LSM segments of its vectors bucket
(wv_index_load_segments) and search it -- bit-exact against the oracle built
from the bucket's final state (oracle/lsm.py replay: newest wins, tombstones
delete).  Segments are written by the oracle's restated lsmkv writer."""
import numpy as np
import pytest

import lsm  # oracle/lsm.py (test infrastructure)

pytestmark = pytest.mark.gpu


def _segments(tmp_path, oracle, n, d, kind=0, normalized=False):
    """normalized: the bucket holds what flat.Add stored for cosine -- rows
    already through distancer.Normalize (flat/index.go:376-378)."""
    prep = (lambda m: np.stack([oracle.normalize(x) for x in m])) if normalized else (lambda m: m)
    base = prep(oracle.gen_matrix(kind, 31, 0, n, d))
    upd = prep(oracle.gen_matrix(kind, 32, 0, n // 5, d))
    ids = np.arange(n, dtype=np.uint64) * 3 + 5          # sparse ids
    up_ids = ids[::5][: len(upd)]
    dead = np.setdiff1d(ids[1::11], up_ids)  # one node per key within a segment
    revived = dead[::4]
    rv = prep(oracle.gen_matrix(kind, 33, 0, len(revived), d))
    blobs = [
        lsm.write_segment(lsm.vector_entries(ids[: n // 2], base[: n // 2]), version=0),
        lsm.write_segment(lsm.vector_entries(ids[n // 2:], base[n // 2:]), version=1, level=1),
        lsm.write_segment(sorted(lsm.vector_entries(up_ids, upd) + lsm.vector_entries(dead, None),
                                 key=lambda kv: kv[0])),
        lsm.write_segment(lsm.vector_entries(revived, rv)),
    ]
    paths = []
    for i, b in enumerate(blobs):
        p = tmp_path / f"segment-{i}.db"
        p.write_bytes(b)
        paths.append(str(p))
    state = lsm.replay_segments(blobs)
    live = sorted(k for k, v in state.items() if v is not None)
    return paths, state, np.array(live, np.uint64), np.stack([state[k] for k in live])


@pytest.mark.parametrize("metric,bq,n,d,k", [
    ("cosine", False, 6000, 96, 10),
    ("l2-squared", False, 4000, 128, 25),
    ("dot", True, 5000, 200, 10),
])
def test_load_segments_search_equals_oracle(wv, oracle, tmp_path, metric, bq, n, d, k):
    M = oracle.METRIC[metric]
    paths, state, live_ids, live_vecs = _segments(tmp_path, oracle, n, d, normalized=M == oracle.COSINE)
    kw = {"bq": True, "rescore_limit": 60} if bq else {}
    idx = wv.FlatIndex(distance=metric, variant="avx256", **kw)
    info = idx.load_segments(paths)
    n_dead = sum(v is None for v in state.values())
    assert info["loaded"] == len(live_ids) and info["tombstoned"] == n_dead
    assert idx.already_indexed() == len(live_ids) and idx.dims == d
    for key, v in list(state.items())[:50]:
        assert idx.contains_doc(key) == (v is not None)
    if bq:
        orc = oracle.OracleFlatBQ(M, 1, d, int(max(state)) + 1, 60)
    else:
        orc = oracle.OracleFlat(M, 1, d, int(max(state)) + 1)
    if M == oracle.COSINE:  # the oracle holds the bucket's bytes exactly (no second normalisation)
        orc.store[live_ids.astype(np.int64)] = live_vecs
        orc.present[live_ids.astype(np.int64)] = 1
    else:
        orc.add_batch(live_ids, live_vecs)
    queries = oracle.gen_matrix(0, 34, 0, 16, d)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    for q in range(len(queries)):
        rc, oids, od = orc.search(queries[q], k)
        assert rc == 0
        np.testing.assert_array_equal(ids[q, :counts[q]], oids, err_msg=f"q{q}")
        np.testing.assert_array_equal(dists[q, :counts[q]].view(np.uint32),
                                      np.asarray(od, np.float32).view(np.uint32), err_msg=f"q{q}")
    idx.close()


def test_load_segments_dimension_mismatch(wv, tmp_path):
    a = tmp_path / "a.db"
    a.write_bytes(lsm.write_segment(lsm.vector_entries([1, 2], np.ones((2, 8), np.float32))))
    b = tmp_path / "b.db"
    b.write_bytes(lsm.write_segment(lsm.vector_entries([3], np.ones((1, 9), np.float32))))
    idx = wv.FlatIndex(distance="l2-squared")
    with pytest.raises(wv.WeaviateError, match="insert called with a vector of the wrong size: 9. Saved length: 8"):
        idx.load_segments([str(a), str(b)])
    idx.close()
    idx = wv.FlatIndex(distance="l2-squared")
    idx.add(7, np.ones(8, np.float32))
    idx.load_segments([str(a)])
    assert idx.contains_doc(7) and idx.already_indexed() == 3
    idx.close()
