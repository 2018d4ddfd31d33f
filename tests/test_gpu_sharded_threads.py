"""GPU: weaviate_amd.sharded.ShardedFlatSearch itself (not a restatement of its
steps) with every rank a thread on one GPU.  The collectives are an in-process
stand-in (FakeGroup: all_gather / broadcast through a barrier, same calls as
torch.distributed), the per-rank engines are real GpuShardBackends over HIP
indexes.  Covers shards off the block-key path next to shards on it: a shard
with a non-finite row (phase 1 refused, one-shot local search, replay without
block keys), an empty shard, and both replay forms (parallel records for
k < 64, the device-flag chain for k >= 64).  Must equal the oracle's single
index over the same rows (flat/index.go:578-688)."""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class FakeGroup:
    """torch.distributed stand-in for ranks that are threads of one process."""

    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world)
        self.slots = [None] * world
        self.tl = threading.local()

    def get_rank(self):
        return self.tl.rank

    def get_world_size(self):
        return self.world

    def get_backend(self):
        return "fake"

    def all_gather(self, parts, t):
        r = self.get_rank()
        self.slots[r] = t.clone()
        self.bar.wait()
        for i in range(self.world):
            parts[i].copy_(self.slots[i])
        torch.cuda.synchronize()
        self.bar.wait()

    def all_reduce(self, t, op=None):  # MIN (the only reduction the protocols use)
        r = self.get_rank()
        self.slots[r] = t.clone()
        self.bar.wait()
        m = self.slots[0].clone()
        for i in range(1, self.world):
            m = torch.minimum(m, self.slots[i])
        t.copy_(m)
        torch.cuda.synchronize()
        self.bar.wait()

    def broadcast(self, t, src):
        r = self.get_rank()
        if r == src:
            self.slots[src] = t.clone()
        self.bar.wait()
        if r != src:
            t.copy_(self.slots[src])
        torch.cuda.synchronize()
        self.bar.wait()


def run_ranks(monkeypatch, backs, q, k):
    import weaviate_amd.sharded as sh
    g = FakeGroup(len(backs))
    monkeypatch.setattr(sh, "dist", g)
    out, err = [None] * len(backs), []

    def rank_main(r):
        g.tl.rank = r
        try:
            s = sh.ShardedFlatSearch(backs[r], torch.device("cuda", 0))
            res = s.search(q, k)
            torch.cuda.synchronize()
            out[r] = tuple(t.cpu() for t in res)
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            err.append(e)
            g.bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(len(backs))]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not any(t.is_alive() for t in th), "a rank is stuck in a collective"
    if err:
        raise err[0]
    return out


@pytest.mark.parametrize("metric,kind,d,k", [("cosine", 0, 96, 10),       # parallel record replay
                                             ("l2-squared", 1, 32, 10),   # integer ties: many flagged queries
                                             ("l2-squared", 1, 24, 100)])  # device-flag chain (k >= 64)
def test_sharded_search_with_off_path_and_empty_shards(wv, oracle, monkeypatch, metric, kind, d, k):
    per = 3000
    layout = ["normal", "nonfinite", "empty", "normal"]
    data = oracle.gen_matrix(kind, 51, 0, per * len(layout), d)
    data[per + 17, 3] = np.nan  # shard 1 holds a NaN row: off the block-key path
    queries = oracle.gen_matrix(kind, 52, 0, 160, d)
    backs, ids_all = [], []
    from weaviate_amd.sharded import GpuShardBackend
    for r, kind_r in enumerate(layout):
        lo = r * per
        idx = wv.FlatIndex(distance=metric, dims=d, id_base=lo, variant="avx256")
        if kind_r != "empty":
            ids = np.arange(lo, lo + per, dtype=np.uint64)
            idx.add_batch(ids, data[lo:lo + per])
            ids_all.append(ids)
        backs.append(GpuShardBackend(idx, 0))
    q = torch.from_numpy(queries).to("cuda")
    out = run_ranks(monkeypatch, backs, q, k)
    ids_all = np.concatenate(ids_all)
    orc = oracle.OracleFlat(oracle.METRIC[metric], 1, d, per * len(layout))
    orc.add_batch(ids_all, data[ids_all.astype(np.int64)])
    for r in range(len(backs)):  # every rank holds the merged result
        oi, od, on = (t.numpy() for t in out[r])
        for i in range(len(queries)):
            rc, ei, ed = orc.search(queries[i], k)
            assert rc == 0 and on[i] == len(ei), f"rank {r} q{i}"
            np.testing.assert_array_equal(oi[i, :on[i]].astype(np.uint64), ei, err_msg=f"rank {r} q{i}")
            np.testing.assert_array_equal(od[i, :on[i]].view(np.uint32), ed.view(np.uint32), err_msg=f"rank {r} q{i}")
    for b in backs:
        b.index.close()


def test_phase2_refused_after_interleaved_add(wv, oracle):
    """A batch's shard phase 1 ends with any Add / Delete / other query
    preparation on the index (the keys, eps and query rows it left would be
    stale): phase 2 is refused instead of reading them."""
    from weaviate_amd import WeaviateError
    from weaviate_amd.sharded import GpuShardBackend
    n, d, k = 4000, 64, 10
    data = oracle.gen_matrix(0, 53, 0, n + 500, d)
    idx = wv.FlatIndex(distance="l2-squared", dims=d, variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data[:n])
    b = GpuShardBackend(idx, 0)
    q = torch.from_numpy(oracle.gen_matrix(0, 54, 0, 64, d)).to("cuda")
    for interleave in ("add", "search", "delete"):
        topA, eps = b.phase1(q, k)
        if interleave == "add":
            idx.add_batch(np.arange(n, n + 500, dtype=np.uint64), data[n:])
        elif interleave == "search":
            idx.search_by_vector_batch(data[:2], 3)
        else:
            idx.delete(5)
        with pytest.raises(WeaviateError):
            b.phase2(topA[None], eps[None], k)
    idx.close()


def run_bq_ranks(monkeypatch, backs, q, k, id_stride):
    import weaviate_amd.sharded as sh
    g = FakeGroup(len(backs))
    monkeypatch.setattr(sh, "dist", g)
    out, paths, err = [None] * len(backs), [None] * len(backs), []

    def rank_main(r):
        g.tl.rank = r
        try:
            s = sh.ShardedBQSearch(backs[r], torch.device("cuda", 0), id_stride)
            res = s.search(q, k)
            torch.cuda.synchronize()
            out[r] = tuple(t.cpu() for t in res)
            paths[r] = s.path
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            err.append(e)
            g.bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(len(backs))]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not any(t.is_alive() for t in th), "a rank is stuck in a collective"
    if err:
        raise err[0]
    return out, paths


@pytest.mark.parametrize("shards,metric,kind,per,d,k,rl,path", [
    # the bounds T_r come from 256-row block minima: a finite, useful T_r needs
    # shards of several R blocks (C4: 24k blocks of a 6.25M-row shard at R = 200)
    (3, "cosine", 0, 52000, 1536, 10, 40, "parallel"),    # C4's width
    (4, "l2-squared", 0, 20000, 256, 10, 16, "parallel"),
    (2, "cosine", 1, 9000, 96, 10, 30, None)])           # integer data: ties (records may overflow -> chain)
def test_sharded_bq_parallel_replay(wv, oracle, monkeypatch, shards, metric, kind, per, d, k, rl, path):
    """ShardedBQSearch with GpuBQShardBackends as threads: the R-heap of
    searchByVectorQuantized (flat/index.go:460-532) across the shards in one
    parallel hop (wv_index_bq_bounds -> all-gather -> k copies of T_r ->
    wv_index_bq_replay_record -> all-gather -> wv_heap_merge_records), then
    rescoring and the final heap.  Must equal the single BQ index and the
    oracle exactly, on every rank."""
    from weaviate_amd.sharded import GpuBQShardBackend
    n = per * shards
    data = oracle.gen_matrix(kind, 71, 0, n, d)
    queries = oracle.gen_matrix(kind, 72, 0, 300, d)
    backs = []
    for r in range(shards):
        lo = r * per
        idx = wv.FlatIndex(distance=metric, bq=True, rescore_limit=rl, id_base=lo, variant="avx256")
        idx.add_batch(np.arange(lo, lo + per, dtype=np.uint64), data[lo:lo + per])
        backs.append(GpuBQShardBackend(idx, 0))
    q = torch.from_numpy(queries).to("cuda")
    out, paths = run_bq_ranks(monkeypatch, backs, q, k, per)
    if path is not None:
        assert paths == [path] * shards, paths
    single = wv.FlatIndex(distance=metric, bq=True, rescore_limit=rl, variant="avx256")
    single.add_batch(np.arange(n, dtype=np.uint64), data)
    si, sd, sn = single.search_by_vector_batch(queries, k)
    orc = oracle.OracleFlatBQ(oracle.METRIC[metric], 1, d, n, rl)
    orc.add_batch(np.arange(n), data)
    for r in range(shards):
        oi, od, on = (t.numpy() for t in out[r])
        for i in range(len(queries)):
            assert on[i] == sn[i], f"rank {r} q{i}"
            np.testing.assert_array_equal(oi[i, :on[i]].astype(np.uint64), si[i, :sn[i]], err_msg=f"rank {r} q{i}")
            np.testing.assert_array_equal(od[i, :on[i]].view(np.uint32), sd[i, :sn[i]].view(np.uint32))
    for i in range(0, len(queries), 37):
        rc, ids, dd = orc.search(queries[i], k)
        np.testing.assert_array_equal(out[0][0].numpy()[i, :len(ids)].astype(np.uint64), ids, err_msg=f"q{i} vs oracle")
    for b in backs:
        b.index.close()
    single.close()


def run_quant_ranks(monkeypatch, backs, q, k, id_stride):
    import weaviate_amd.sharded as sh
    g = FakeGroup(len(backs))
    monkeypatch.setattr(sh, "dist", g)
    out, paths, err = [None] * len(backs), [None] * len(backs), []

    def rank_main(r):
        g.tl.rank = r
        try:
            s = sh.ShardedQuantSearch(backs[r], torch.device("cuda", 0), id_stride)
            res = s.search(q, k)
            torch.cuda.synchronize()
            out[r] = tuple(t.cpu() for t in res)
            paths[r] = s.path
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            err.append(e)
            g.bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(len(backs))]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not any(t.is_alive() for t in th), "a rank is stuck in a collective"
    if err:
        raise err[0]
    return out, paths


@pytest.mark.parametrize("comp,shards,metric,kind,per,d,k,rl,rescore", [
    ("pq", 3, "l2-squared", 0, 6000, 32, 10, -1, False),   # worker heap = k (query chunks forced: below)
    ("pq", 2, "cosine", 0, 8000, 64, 10, 60, True),        # rescoring: owners' exact distances
    ("pq", 4, "l2-squared", 1, 3000, 24, 7, 40, True),     # integer data: ADC ties
    ("sq", 3, "l2-squared", 0, 5000, 48, 10, 20, True),    # SQ: ef limit, trim to the rescore limit
    ("sq", 2, "dot", 1, 6000, 32, 10, 0, True),            # SQ rescore limit 0: no rescoring
    ("rq8", 3, "cosine", 0, 6000, 64, 10, 30, True),       # flat rq-8: searchByVectorQuantized
    ("rq1", 2, "l2-squared", 1, 7000, 64, 10, 40, True),   # flat rq-1, integer data
])
def test_sharded_quant_equals_single_index(wv, oracle, monkeypatch, comp, shards, metric, kind, per, d, k, rl, rescore):
    """ShardedQuantSearch with GpuQuantShardBackends as threads: hnsw's flat
    search over PQ / SQ codes (hnsw/flat_search.go:28-141 + h.rescore) and
    flat's searchByVectorQuantized over rq-8 / rq-1 codes, with the
    worker heap across the shards in one parallel hop (or the chain when a
    record overflows), the result heap and the owners' rescoring.  Every rank
    must return the single index's result exactly (same quantizer)."""
    from weaviate_amd.sharded import GpuQuantShardBackend
    n = per * shards
    data = oracle.gen_matrix(kind, 91, 0, n, d)
    queries = oracle.gen_matrix(kind, 92, 0, 120, d)
    kw = dict(distance=metric, variant="avx256", rescore_limit=rl)
    if comp == "pq":
        kw["pq"] = {"segments": d // 4, "centroids": 32, "trainingLimit": 100000, "rescore": rescore}
    elif comp == "sq":
        kw["sq"] = True
    else:  # the rotation is seeded: the same on every shard
        kw["rq"] = {"bits": 8 if comp == "rq8" else 1}
    single = wv.FlatIndex(**kw)
    single.add_batch(np.arange(n, dtype=np.uint64), data)
    if comp == "pq":
        single.pq_fit(seed=3)
        centers = single.pq_centers()
    elif comp == "sq":
        single.sq_fit(2000)
        info = single.sq_info()
    si, sd, sn = single.search_by_vector_batch(queries, k)
    backs = []
    for r in range(shards):
        lo = r * per
        idx = wv.FlatIndex(id_base=lo, **kw)
        idx.add_batch(np.arange(lo, lo + per, dtype=np.uint64), data[lo:lo + per])
        if comp == "pq":
            idx.pq_set_centers(centers)
        elif comp == "sq":
            idx.sq_restore(info["a"], info["b"])
        backs.append(GpuQuantShardBackend(idx, 0))
    if comp == "pq" and not rescore:  # rank r's distance group holds 37 + 10 r queries: chunks of 37 on every rank
        for r, b in enumerate(backs):
            b.max_batch = (lambda v: (lambda k, world: v))(37 + 10 * r)
    q = torch.from_numpy(queries).to("cuda")
    out, paths = run_quant_ranks(monkeypatch, backs, q, k, per)
    assert len(set(paths)) == 1, paths
    for r in range(shards):
        oi, od, on = (t.numpy() for t in out[r])
        for i in range(len(queries)):
            assert on[i] == sn[i], f"rank {r} q{i}"
            np.testing.assert_array_equal(oi[i, :on[i]].astype(np.uint64), si[i, :sn[i]], err_msg=f"rank {r} q{i}")
            np.testing.assert_array_equal(od[i, :on[i]].view(np.uint32), sd[i, :sn[i]].view(np.uint32),
                                          err_msg=f"rank {r} q{i}")
    for b in backs:
        b.index.close()
    single.close()


def test_c5_sharded_pq_full_size(wv, oracle, monkeypatch):
    """configs[4] across 4 shards (ranks as threads): 10M x 960 U[0,1) rows in
    contiguous 2.5M-row ranges, one codebook (PQ m=240 x 256 trained on the
    first 100k rows, distributed as bench.py --workload pq does at N > 1), the
    bench's B = 256: ShardedQuantSearch on every rank equals the single index's
    search (the minima-only k_pq_adc3 path) bit for bit."""
    from weaviate_amd import _lib
    from weaviate_amd.sharded import GpuQuantShardBackend
    lib = _lib.load()
    n, d, k, B, W = 10_000_000, 960, 10, 256, 4
    per = n // W
    pqc = {"segments": 240, "centroids": 256, "trainingLimit": 100_000, "rescore": False}

    def build(lo, hi):
        idx = wv.FlatIndex(distance="l2-squared", dims=d, variant="avx256", id_base=lo, pq=pqc)
        idx.reserve(hi - lo)
        stage = torch.empty((1_000_000, d), dtype=torch.float32, device="cuda")
        for r0 in range(lo, hi, 1_000_000):
            m = min(1_000_000, hi - r0)
            _lib.check(lib.wv_gen_device(0, 2, 1, r0, m, d, stage.data_ptr(), None))
            _lib.check(lib.wv_index_add_range_device(idx._h, r0, stage.data_ptr(), m, d))
        torch.cuda.synchronize()
        return idx

    single = build(0, n)
    single.pq_fit(seed=1)
    centers = single.pq_centers()
    q = torch.empty((B, d), dtype=torch.float32, device="cuda")
    _lib.check(lib.wv_gen_device(0, 2, 2, 0, B, d, q.data_ptr(), None))
    torch.cuda.synchronize()
    si, sd, sn = single.search_by_vector_batch(q.cpu().numpy(), k)
    single.close()
    backs = []
    for r in range(W):
        idx = build(r * per, (r + 1) * per)
        idx.pq_set_centers(centers)
        backs.append(GpuQuantShardBackend(idx, 0))
    out, paths = run_quant_ranks(monkeypatch, backs, q, k, per)
    assert paths == ["parallel"] * W, paths
    for r in range(W):
        oi, od, on = (t.numpy() for t in out[r])
        np.testing.assert_array_equal(on, sn, err_msg=f"rank {r}")
        for i in range(B):
            np.testing.assert_array_equal(oi[i, :on[i]].astype(np.uint64), si[i, :sn[i]], err_msg=f"rank {r} q{i}")
            np.testing.assert_array_equal(od[i, :on[i]].view(np.uint32), sd[i, :sn[i]].view(np.uint32))
    for b in backs:
        b.index.close()


def test_bq_batch_refused_after_interleaved_add(wv, oracle):
    """A sharded BQ batch (bq_begin's minima and query codes) ends with any
    Add / Delete / other query preparation on the index: the later stages
    (bounds, recorded replay, replay, rescore) are refused instead of reading
    minima sized for the old corpus (invalidate_batch resets bq_nq)."""
    from weaviate_amd import WeaviateError
    from weaviate_amd.sharded import GpuBQShardBackend
    n, d, k = 6000, 128, 10
    data = oracle.gen_matrix(0, 57, 0, n + 500, d)
    idx = wv.FlatIndex(distance="cosine", variant="avx256", bq=True, rescore_limit=40)
    idx.add_batch(np.arange(n, dtype=np.uint64), data[:n])
    b = GpuBQShardBackend(idx, 0)
    q = torch.from_numpy(oracle.gen_matrix(0, 58, 0, 32, d)).to("cuda")
    # (another search replaces the batch with its own, consistent minima)
    for interleave in ("add", "delete"):
        b.bq_begin(q, k)
        b.bq_bounds()  # the batch is live
        if interleave == "add":
            idx.add_batch(np.arange(n, n + 500, dtype=np.uint64), data[n:])
        else:
            idx.delete(5)
        with pytest.raises(WeaviateError):
            b.bq_bounds()
    idx.close()


def test_sharded_rq_with_an_empty_shard(wv, oracle, monkeypatch):
    """An empty rank (no rows in its id range) beside rq-8 shards: its block
    minima are +inf (not a finite 0x7f-byte fill), so the bounds of
    the later ranks stay those of real rows and every rank returns the single
    index's result."""
    from weaviate_amd.sharded import GpuQuantShardBackend
    per, shards, d, k = 5000, 3, 64, 10
    data = oracle.gen_matrix(0, 93, 0, per * (shards - 1), d)
    queries = oracle.gen_matrix(0, 94, 0, 64, d)
    kw = dict(distance="cosine", variant="avx256", rescore_limit=30, rq={"bits": 8})
    single = wv.FlatIndex(**kw)
    single.add_batch(np.arange(per * (shards - 1), dtype=np.uint64), data)
    si, sd, sn = single.search_by_vector_batch(queries, k)
    backs = []
    for r in range(shards):
        lo = r * per
        idx = wv.FlatIndex(id_base=lo, dims=d, **kw)
        if r < shards - 1:
            idx.add_batch(np.arange(lo, lo + per, dtype=np.uint64), data[lo:lo + per])
        backs.append(GpuQuantShardBackend(idx, 0))
    q = torch.from_numpy(queries).to("cuda")
    out, paths = run_quant_ranks(monkeypatch, backs, q, k, per)
    for r in range(shards):
        oi, od, on = (t.numpy() for t in out[r])
        for i in range(len(queries)):
            assert on[i] == sn[i], f"rank {r} q{i}"
            np.testing.assert_array_equal(oi[i, :on[i]].astype(np.uint64), si[i, :sn[i]], err_msg=f"rank {r} q{i}")
            np.testing.assert_array_equal(od[i, :on[i]].view(np.uint32), sd[i, :sn[i]].view(np.uint32),
                                          err_msg=f"rank {r} q{i}")
    for b in backs:
        b.index.close()
    single.close()
