"""GPU: the sharded exact-search protocol of weaviate_amd.sharded.ShardedFlatSearch
(mode-1 shard search -> gather -> wv_merge_shards -> cross-shard heap replay of
flagged queries) with the shards as separate indexes on one GPU; the RCCL
all-gather / broadcasts become local hand-overs.  Must equal the single index."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("stale", [False, True])
@pytest.mark.parametrize("shards,metric,kind,n,d,k", [(2, "cosine", 0, 12000, 768, 10),
                                                     (3, "l2-squared", 1, 6000, 64, 10),   # integer data: ties
                                                     (4, "dot", 0, 5000, 100, 24),
                                                     (2, "l2-squared", 1, 20000, 32, 100)])
def test_sharded_flat_protocol_equals_single_index(wv, oracle, shards, metric, kind, n, d, k, stale):
    """stale=False: each shard's replay is bounded by the block keys of its
    local search (k_blk_replay with a handed-over heap); stale=True: another
    search in between invalidates them, every row is scanned (run_replay)."""
    from weaviate_amd.sharded import GpuShardBackend
    dev = torch.device("cuda", 0)
    data = oracle.gen_matrix(kind, 41, 0, n, d)
    queries = oracle.gen_matrix(kind, 42, 0, 200, d)
    per = (n + shards - 1) // shards
    backs = []
    for r in range(shards):
        lo, hi = r * per, min(n, (r + 1) * per)
        idx = wv.FlatIndex(distance=metric, id_base=lo, variant="avx256")
        idx.add_batch(np.arange(lo, hi, dtype=np.uint64), data[lo:hi])
        backs.append(GpuShardBackend(idx, 0))
    q = torch.from_numpy(queries).to(dev)
    parts = [b.local_search(q, k) for b in backs]
    gi, gd, gc, gf = (torch.stack([p[j] for p in parts]) for j in range(4))
    oi, od, on, of = backs[0].merge(shards, k, gi, gd, gc, gf)
    if stale:
        for b in backs:
            b.index.search_by_vector_batch(queries[:1], 1)
    flagged = torch.nonzero(of).flatten().to(torch.int32)
    if kind == 1:
        assert flagged.numel() > 0  # integer data: the replay chain must run
    if flagged.numel():
        state = None
        for r, b in enumerate(backs):
            state = b.replay(q, flagged, state, k, r == shards - 1)
        rows = flagged.long()
        oi[rows], od[rows], on[rows] = state
    oi, od, on = oi.cpu().numpy(), od.cpu().numpy(), on.cpu().numpy()
    single = wv.FlatIndex(distance=metric, variant="avx256")
    single.add_batch(np.arange(n, dtype=np.uint64), data)
    si, sd, sn = single.search_by_vector_batch(queries, k)
    om = oracle.METRIC[metric]
    orc = oracle.OracleFlat(om, 1, d, n)
    orc.add_batch(np.arange(n), data)
    for i in range(len(queries)):
        assert on[i] == sn[i]
        np.testing.assert_array_equal(oi[i, :on[i]].astype(np.uint64), si[i, :sn[i]], err_msg=f"q{i}")
        np.testing.assert_array_equal(od[i, :on[i]].view(np.uint32), sd[i, :sn[i]].view(np.uint32))
        # and the reference heap over the whole corpus (oracle/oracle.c or_flat_search)
        rc, ei, ed = orc.search(queries[i], k)
        assert rc == 0 and on[i] == len(ei)
        np.testing.assert_array_equal(oi[i, :on[i]].astype(np.uint64), ei, err_msg=f"q{i} vs oracle")
        np.testing.assert_array_equal(od[i, :on[i]].view(np.uint32), ed.view(np.uint32), err_msg=f"q{i} vs oracle")
    for b in backs:
        b.index.close()
    single.close()


@pytest.mark.parametrize("shards,metric,kind,n,d,k", [(2, "cosine", 0, 12000, 768, 10),
                                                     (3, "l2-squared", 1, 6000, 64, 10),   # integer data: ties
                                                     (4, "dot", 0, 5000, 100, 24),
                                                     (8, "cosine", 0, 16000, 128, 10),
                                                     (2, "l2-squared", 1, 20000, 32, 100)])
def test_sharded_two_phase_and_flag_chain(wv, oracle, shards, metric, kind, n, d, k):
    """The protocol ShardedFlatSearch runs on the block-key path: phase 1 (keys
    + each shard's k+1 smallest key values) -> gather -> phase 2 (global
    threshold cuts the candidates, exact rows) -> packed gather -> merge ->
    replay chain of the flagged queries with device-built lists and states
    indexed by query.  Shards are separate indexes on one GPU; gathers and
    broadcasts become local hand-overs.  Must equal the oracle."""
    from weaviate_amd.sharded import GpuShardBackend, ShardedFlatSearch
    dev = torch.device("cuda", 0)
    data = oracle.gen_matrix(kind, 43, 0, n, d)
    queries = oracle.gen_matrix(kind, 44, 0, 300, d)
    per = (n + shards - 1) // shards
    backs = []
    for r in range(shards):
        lo, hi = r * per, min(n, (r + 1) * per)
        idx = wv.FlatIndex(distance=metric, id_base=lo, variant="avx256")
        idx.add_batch(np.arange(lo, hi, dtype=np.uint64), data[lo:hi])
        backs.append(GpuShardBackend(idx, 0))
    q = torch.from_numpy(queries).to(dev)
    p1 = [b.phase1(q, k) for b in backs]
    gA = torch.stack([t for t, _ in p1])
    gE = torch.stack([e for _, e in p1])
    parts = [b.phase2(gA, gE, k) for b in backs]
    gi, gd, gc, gf = (torch.stack([p[j] for p in parts]) for j in range(4))
    oi, od, on, of = backs[0].merge(shards, k, gi, gd, gc, gf)
    nflag = int(of.count_nonzero())
    if kind == 1:
        assert nflag > 0  # integer data: the replay chain must run
    state = None
    for r, b in enumerate(backs):
        last = r == shards - 1
        res = b.replay_flags(q, of, state, k, last, out=(oi, od, on) if last else None)
        state = ShardedFlatSearch._unpack_state(ShardedFlatSearch._pack_state(*res), k)
    oi, od, on = (t.cpu().numpy() for t in state)
    orc = oracle.OracleFlat(oracle.METRIC[metric], 1, d, n)
    orc.add_batch(np.arange(n), data)
    for i in range(len(queries)):
        rc, ei, ed = orc.search(queries[i], k)
        assert rc == 0 and on[i] == len(ei), f"q{i}"
        np.testing.assert_array_equal(oi[i, :on[i]].astype(np.uint64), ei, err_msg=f"q{i} vs oracle")
        np.testing.assert_array_equal(od[i, :on[i]].view(np.uint32), ed.view(np.uint32), err_msg=f"q{i} vs oracle")
    for b in backs:
        b.index.close()


@pytest.mark.parametrize("shards,metric,kind,n,d,k", [(3, "l2-squared", 1, 6000, 64, 10),   # integer data: ties
                                                     (8, "cosine", 0, 16000, 128, 10),
                                                     (4, "l2-squared", 1, 8000, 24, 50)])
def test_sharded_parallel_replay_records(wv, oracle, shards, metric, kind, n, d, k):
    """The parallel cross-shard replay (ShardedFlatSearch._replay_parallel):
    shard 0 replays from empty heaps, shards r >= 1 from k copies of T_r
    (weaviate_amd.sharded.prefix_bound) recording their insertions,
    wv_heap_merge_records applies the records in shard order.  Must equal the
    oracle; also with a 2-entry record cap (overflow -> serial chain)."""
    from weaviate_amd.sharded import GpuShardBackend, fake_heaps, prefix_bound
    dev = torch.device("cuda", 0)
    data = oracle.gen_matrix(kind, 45, 0, n, d)
    queries = oracle.gen_matrix(kind, 46, 0, 200, d)
    per = (n + shards - 1) // shards
    backs = []
    for r in range(shards):
        lo, hi = r * per, min(n, (r + 1) * per)
        idx = wv.FlatIndex(distance=metric, id_base=lo, variant="avx256")
        idx.add_batch(np.arange(lo, hi, dtype=np.uint64), data[lo:hi])
        backs.append(GpuShardBackend(idx, 0))
    q = torch.from_numpy(queries).to(dev)
    orc = oracle.OracleFlat(oracle.METRIC[metric], 1, d, n)
    orc.add_batch(np.arange(n), data)
    for cap in (256, 2):
        p1 = [b.phase1(q, k) for b in backs]
        gA = torch.stack([t for t, _ in p1])
        gE = torch.stack([e for _, e in p1])
        parts = [b.phase2(gA, gE, k) for b in backs]
        gi, gd, gc, gf = (torch.stack([p[j] for p in parts]) for j in range(4))
        oi, od, on, of = backs[0].merge(shards, k, gi, gd, gc, gf)
        ql = torch.nonzero(of).flatten()
        F = int(ql.numel())
        if kind == 1:
            assert F > 0
        ql32 = ql.to(torch.int32)
        ti, td, tn = backs[0].replay(q, ql32, None, k, False)
        rec = [(None, None, None)]
        for r in range(1, shards):
            T = prefix_bound(r, ql, k, gd, gc, gf, (gA, gE))
            rec.append(backs[r].replay_record(q, ql32, fake_heaps(T, k), k, cap))
        ri = torch.zeros((shards, F, cap), dtype=torch.int64, device=dev)
        rd = torch.zeros((shards, F, cap), dtype=torch.float32, device=dev)
        rn = torch.zeros((shards, F), dtype=torch.int32, device=dev)
        for r in range(1, shards):
            ri[r], rd[r], rn[r] = rec[r]
        fi, fd, fn, un = backs[0].merge_records(shards, k, cap, (ti.contiguous(), td.contiguous(), tn), (ri, rd, rn))
        oi[ql], od[ql], on[ql] = fi, fd, fn
        bad = ql32[un.bool()]
        if cap == 2 and F:
            assert bad.numel() > 0  # tiny records overflow
        if bad.numel():  # the serial chain for the overflowed ones
            state = None
            for r, b in enumerate(backs):
                state = b.replay(q, bad, state, k, r == shards - 1)
            oi[bad.long()], od[bad.long()], on[bad.long()] = state
        ai, ad, an = oi.cpu().numpy(), od.cpu().numpy(), on.cpu().numpy()
        for i in range(len(queries)):
            rc, ei, ed = orc.search(queries[i], k)
            assert rc == 0 and an[i] == len(ei), f"cap{cap} q{i}"
            np.testing.assert_array_equal(ai[i, :an[i]].astype(np.uint64), ei, err_msg=f"cap{cap} q{i}")
            np.testing.assert_array_equal(ad[i, :an[i]].view(np.uint32), ed.view(np.uint32), err_msg=f"cap{cap} q{i}")
    for b in backs:
        b.index.close()
