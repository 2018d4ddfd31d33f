"""GPU: the multi-shard index of the C library (wv_multi, multi.hip) -- the
sharded exact search driven from one process with the library's own
transports.  Shards share the one GPU of the box (local transport), or one
shard runs over a real RCCL communicator (world 1).  Must equal the single
flat index over the whole corpus bit for bit (ids, distances, tie order) and
the oracle's reference heap (oracle/oracle.c)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _single(wv, metric, data, queries, k):
    single = wv.FlatIndex(distance=metric, variant="avx256")
    single.add_batch(np.arange(data.shape[0], dtype=np.uint64), data)
    out = single.search_by_vector_batch(queries, k)
    single.close()
    return out


def _assert_equal(got, exp, tag=""):
    gi, gd, gn = got
    ei, ed, en = exp
    np.testing.assert_array_equal(gn, en, err_msg=f"{tag} counts")
    for i in range(len(gn)):
        np.testing.assert_array_equal(gi[i, :gn[i]], ei[i, :en[i]], err_msg=f"{tag} q{i} ids")
        np.testing.assert_array_equal(gd[i, :gn[i]].view(np.uint32), ed[i, :en[i]].view(np.uint32),
                                      err_msg=f"{tag} q{i} dists")


def _multi(wv, metric, d, shards, per, transport="local"):
    from weaviate_amd.multi import MultiFlatIndex
    return MultiFlatIndex(distance=metric, dims=d, devices=[0] * shards, id_stride=per, transport=transport,
                          variant="avx256")


@pytest.mark.parametrize("shards,metric,kind,n,d,k", [(2, "cosine", 0, 12000, 768, 10),
                                                     (3, "l2-squared", 1, 6000, 64, 10),   # integer data: ties
                                                     (4, "dot", 0, 5000, 100, 24),
                                                     (8, "cosine", 0, 16000, 128, 10),
                                                     (8, "cosine", 0, 16000, 768, 10),
                                                     (5, "l2-squared", 1, 9000, 48, 1),
                                                     (2, "l2-squared", 1, 20000, 32, 100)])  # k >= 64: flag chain
def test_multi_equals_single_index_and_oracle(wv, oracle, shards, metric, kind, n, d, k):
    data = oracle.gen_matrix(kind, 43, 0, n, d)
    queries = oracle.gen_matrix(kind, 44, 0, 300, d)
    per = (n + shards - 1) // shards
    m = _multi(wv, metric, d, shards, per)
    m.add_batch(np.arange(n, dtype=np.uint64), data)
    got = m.search_by_vector_batch(queries, k)
    st = m.stats()
    _assert_equal(got, _single(wv, metric, data, queries, k), "single")
    if kind == 1 and k > 1:
        assert st["last_flagged"] > 0  # integer data: the cross-shard replay ran
    orc = oracle.OracleFlat(oracle.METRIC[metric], 1, d, n)
    orc.add_batch(np.arange(n), data)
    for i in range(0, len(queries), 7):
        rc, ei, ed = orc.search(queries[i], k)
        assert rc == 0 and got[2][i] == len(ei)
        np.testing.assert_array_equal(got[0][i, :got[2][i]], ei, err_msg=f"q{i} vs oracle")
        np.testing.assert_array_equal(got[1][i, :got[2][i]].view(np.uint32), ed.view(np.uint32))
    # a second batch on the same buffers and a different k
    _assert_equal(m.search_by_vector_batch(queries[:37], 5), _single(wv, metric, data, queries[:37], 5), "k5")
    m.close()


def test_multi_record_overflow_takes_the_chain(wv, oracle):
    """A record capacity of k forces every recorded replay to overflow: the
    overflowed queries go down the serial chain and the results stay exact."""
    n, d, k, shards = 6000, 64, 10, 3
    data = oracle.gen_matrix(1, 43, 0, n, d)
    queries = oracle.gen_matrix(1, 44, 0, 300, d)
    m = _multi(wv, "l2-squared", d, shards, n // shards)
    m.add_batch(np.arange(n, dtype=np.uint64), data)
    m.set_option("rec_cap", k)
    got = m.search_by_vector_batch(queries, k)
    st = m.stats()
    assert st["last_flagged"] > 0 and st["last_overflowed"] > 0 and st["chain_hops"] >= shards
    _assert_equal(got, _single(wv, "l2-squared", data, queries, k))
    m.close()


def test_multi_ranks_off_the_block_key_path(wv, oracle):
    """An empty shard and a shard holding a NaN row (off the block-key path:
    +inf keys, the one-shot local search, all-rows replays) beside block-key
    shards."""
    n, d, k, shards = 8000, 96, 10, 4
    per = n // shards
    data = oracle.gen_matrix(1, 43, 0, n, d)
    data[per + 17, 5] = np.nan  # shard 1
    keep = np.ones(n, bool)
    keep[2 * per:3 * per] = False  # shard 2 stays empty
    queries = oracle.gen_matrix(1, 44, 0, 64, d)
    m = _multi(wv, "l2-squared", d, shards, per)
    ids = np.arange(n, dtype=np.uint64)[keep]
    m.add_batch(ids, data[keep])
    got = m.search_by_vector_batch(queries, k)
    single = wv.FlatIndex(distance="l2-squared", variant="avx256")
    single.add_batch(ids, data[keep])
    exp = single.search_by_vector_batch(queries, k)
    single.close()
    _assert_equal(got, exp)
    m.close()


def test_multi_device_buffers_and_sim_timing(wv, oracle):
    """wv_multi_search_device on device buffers and a caller stream; option sim
    times every shard's stages alone and leaves the results unchanged."""
    n, d, k, shards = 16000, 768, 10, 8
    data = oracle.gen_matrix(0, 45, 0, n, d)
    queries = oracle.gen_matrix(0, 46, 0, 300, d)
    m = _multi(wv, "cosine", d, shards, n // shards)
    m.add_batch(np.arange(n, dtype=np.uint64), data)
    exp = _single(wv, "cosine", data, queries, k)
    dev = torch.device("cuda", 0)
    q = torch.from_numpy(queries).to(dev)
    oi = torch.empty((len(queries), k), dtype=torch.int64, device=dev)
    od = torch.empty((len(queries), k), dtype=torch.float32, device=dev)
    on = torch.empty(len(queries), dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)
    for sim in (0, 1):
        m.set_option("sim", sim)
        oi.fill_(-7)
        with torch.cuda.stream(s):
            m.search_device(q.data_ptr(), len(queries), d, k, oi.data_ptr(), od.data_ptr(), on.data_ptr(),
                            s.cuda_stream)
        s.synchronize()
        _assert_equal((oi.cpu().numpy().view(np.uint64), od.cpu().numpy(), on.cpu().numpy()), exp, f"sim{sim}")
    t = m.stage_ms()
    assert all(x > 0 for x in t["phase1"]) and all(x > 0 for x in t["phase2"])
    m.close()


def test_multi_rccl_world_one_equals_single(wv, oracle):
    """The RCCL transport (a communicator of one rank, the library's own)."""
    from weaviate_amd.multi import MultiFlatIndex
    n, d, k = 20000, 768, 10
    data = oracle.gen_matrix(0, 47, 0, n, d)
    queries = oracle.gen_matrix(0, 48, 0, 256, d)
    m = MultiFlatIndex(distance="cosine", dims=d, devices=[0], id_stride=n, transport="rccl", variant="avx256")
    m.add_batch(np.arange(n, dtype=np.uint64), data)
    _assert_equal(m.search_by_vector_batch(queries, k), _single(wv, "cosine", data, queries, k))
    assert m.stats()["transport"] == 1
    m.close()


def test_multi_add_routes_and_upserts(wv, oracle):
    """AddBatch routes every id to its shard; a re-add replaces the vector (upsert)
    on the owning shard; ids past the last range go to the last rank."""
    n, d, k, shards = 3000, 64, 10, 3
    data = oracle.gen_matrix(0, 49, 0, n + 500, d)
    queries = oracle.gen_matrix(0, 50, 0, 40, d)
    m = _multi(wv, "cosine", d, shards, 1000)
    m.add_batch(np.arange(n + 500, dtype=np.uint64), data)  # ids 3000..3499 -> rank 2
    upd = np.arange(0, n, 97, dtype=np.uint64)
    m.add_batch(upd, data[upd + 1])
    ref = data.copy()
    ref[upd] = data[upd + 1]
    assert [s.already_indexed() for s in m.shards] == [1000 + len(upd[upd < 1000]), 1000 + len(upd[(upd >= 1000) & (upd < 2000)]),
                                                       1500 + len(upd[upd >= 2000])]
    _assert_equal(m.search_by_vector_batch(queries, k), _single(wv, "cosine", ref, queries, k))
    m.close()
