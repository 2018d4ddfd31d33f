"""GPU: the sharded-BQ C ABI (wv_index_bq_begin / _replay / _rescore /
wv_bq_final) driven like weaviate_amd.sharded.ShardedBQSearch, with the shards
as separate indexes on one GPU (the RCCL broadcasts/all-gather become local
tensor hand-overs).  Must equal the single BQ index and the oracle exactly."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shards,metric,kind,n,d,k,rl", [(3, "cosine", 0, 9000, 1536, 10, 200),
                                                        (2, "l2-squared", 0, 5000, 128, 10, 64),
                                                        (4, "cosine", 1, 4000, 96, 7, 30)])
def test_sharded_bq_chain_equals_single_index(wv, oracle, shards, metric, kind, n, d, k, rl):
    from weaviate_amd.sharded import GpuBQShardBackend
    dev = torch.device("cuda", 0)
    data = oracle.gen_matrix(kind, 31, 0, n, d)
    queries = oracle.gen_matrix(kind, 32, 0, 64, d)
    per = (n + shards - 1) // shards
    backs = []
    for r in range(shards):
        lo, hi = r * per, min(n, (r + 1) * per)
        idx = wv.FlatIndex(distance=metric, bq=True, rescore_limit=rl, id_base=lo, variant="avx256")
        idx.add_batch(np.arange(lo, hi, dtype=np.uint64), data[lo:hi])
        backs.append(GpuBQShardBackend(idx, 0))
    q = torch.from_numpy(queries).to(dev)
    for b in backs:
        b.bq_begin(q, k)
    state = None
    for r, b in enumerate(backs):
        state = b.bq_replay(state, r == shards - 1)
    ids, _, ln = state
    E_all = torch.stack([b.bq_rescore(ids, ln) for b in backs])
    oi, od, on = backs[0].bq_final(shards, per, ids, ln, E_all)
    torch.cuda.synchronize()
    oi, od, on = oi.cpu().numpy(), od.cpu().numpy(), on.cpu().numpy()
    single = wv.FlatIndex(distance=metric, bq=True, rescore_limit=rl, variant="avx256")
    single.add_batch(np.arange(n, dtype=np.uint64), data)
    si, sd, sn = single.search_by_vector_batch(queries, k)
    orc = oracle.OracleFlatBQ(oracle.METRIC[metric], 1, d, n, rl)
    orc.add_batch(np.arange(n), data)
    for i in range(len(queries)):
        np.testing.assert_array_equal(on[i], sn[i])
        np.testing.assert_array_equal(oi[i, :on[i]].astype(np.uint64), si[i, :sn[i]], err_msg=f"q{i}")
        np.testing.assert_array_equal(od[i, :on[i]].view(np.uint32), sd[i, :sn[i]].view(np.uint32))
        if i % 8 == 0:
            rc, ids, dd = orc.search(queries[i], k)
            np.testing.assert_array_equal(oi[i, :on[i]].astype(np.uint64), ids)
    for b in backs:
        b.index.close()
    single.close()
