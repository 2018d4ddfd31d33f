"""CPU, world_size 2 (gloo): the multi-GPU protocol of weaviate_amd/sharded.py
(shard-local verified top-(k+1) -> all-gather -> merge -> cross-rank exact heap
replay for flagged queries) reproduces the single-index reference result,
including heap tie order.  The per-rank engine is an oracle-backed stand-in
(test infrastructure): this test covers the distributed control flow; the GPU
kernels behind it are covered by the gpu-marked tests.
"""
import ctypes as C
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class OracleShardBackend:
    """Stand-in for GpuShardBackend: same tensors in, same tensors out."""

    def __init__(self, orc, metric, corpus, begin, end):
        self.o = orc
        self.metric = metric
        self.n, self.d = corpus.shape
        self.store = corpus.copy()
        if metric == orc.COSINE:
            orc.lib().or_normalize_rows(orc.f(self.store), self.n, self.d)
        self.present = np.zeros(self.n, np.uint8)
        self.present[begin:end] = 1
        self.begin, self.end = begin, end

    def _qnorm(self, qv):
        return self.o.normalize(qv) if self.metric == self.o.COSINE else np.ascontiguousarray(qv, np.float32)

    def local_search(self, q, k):
        qn = q.numpy()
        nq = qn.shape[0]
        ids = np.zeros((nq, k + 1), np.int64)
        dd = np.zeros((nq, k + 1), np.float32)
        cnt = np.zeros(nq, np.int32)
        flg = np.zeros(nq, np.int32)
        for i in range(nq):
            qv = self._qnorm(qn[i])
            dist_ = np.array([self.o.single_dist(self.metric, 1, qv, self.store[s])
                              for s in range(self.begin, self.end)], np.float32)
            order = np.lexsort((np.arange(self.begin, self.end), dist_))[: k + 1]
            m = len(order)
            ids[i, :m] = np.arange(self.begin, self.end)[order]
            dd[i, :m] = dist_[order]
            cnt[i] = m
            flg[i] = int(np.any(np.diff(dd[i, :m]) <= 0))
        return torch.from_numpy(ids), torch.from_numpy(dd), torch.from_numpy(cnt), torch.from_numpy(flg)

    # -- two-phase form (exact distances stand in for the block keys, eps = 0) --
    two_phase = True

    def _dists(self, qv):
        return np.array([self.o.single_dist(self.metric, 1, qv, self.store[s]) for s in range(self.begin, self.end)],
                        np.float32)

    def phase1(self, q, k):
        qn = q.numpy()
        nq = qn.shape[0]
        topA = np.full((nq, k + 1), np.inf, np.float32)
        self._d = []
        for i in range(nq):
            dist_ = self._dists(self._qnorm(qn[i]))
            self._d.append(dist_)
            srt = np.sort(dist_)[: k + 1]
            topA[i, : len(srt)] = srt
        return torch.from_numpy(topA), torch.zeros(nq, dtype=torch.float32)

    def phase2(self, gA, gE, k):
        gA = gA.numpy()
        nq = gA.shape[1]
        ids = np.zeros((nq, k + 1), np.int64)
        dd = np.zeros((nq, k + 1), np.float32)
        cnt = np.zeros(nq, np.int32)
        flg = np.zeros(nq, np.int32)
        for i in range(nq):
            T = np.sort(gA[:, i, :].ravel())[k] + float(gE.numpy()[:, i].max()) * 2
            dist_ = self._d[i]
            keep = np.nonzero(dist_ <= T)[0]
            order = keep[np.lexsort((keep, dist_[keep]))][: k + 1]
            m = len(order)
            ids[i, :m] = np.arange(self.begin, self.end)[order]
            dd[i, :m] = dist_[order]
            cnt[i] = m
            flg[i] = int(np.any(np.diff(dd[i, :m]) <= 0))
        return torch.from_numpy(ids), torch.from_numpy(dd), torch.from_numpy(cnt), torch.from_numpy(flg)

    def replay_flags(self, q, flags, state, k, extract, out=None):
        nq = q.shape[0]
        ql = torch.nonzero(flags).flatten().to(torch.int32)
        st = None if state is None else (state[0][ql.long()], state[1][ql.long()], state[2][ql.long()])
        oi = torch.zeros((nq, k), dtype=torch.int64) if out is None else out[0]
        od = torch.zeros((nq, k), dtype=torch.float32) if out is None else out[1]
        on = torch.zeros(nq, dtype=torch.int32) if out is None else out[2]
        if ql.numel():
            ti, td, tn = self.replay(q, ql, st, k, extract)
            rows = ql.long()
            oi[rows], od[rows], on[rows] = ti, td, tn
        return oi, od, on

    # -- parallel replay: recorded insertions + merge (oracle heap restatement) --
    def _heap(self, k):
        o = self.o
        lib = o.lib()
        lib.or_insert_to_heap.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_float]
        lib.or_heap_pop.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_float)]

        class H(C.Structure):
            _fields_ = [("id", C.POINTER(C.c_uint64)), ("dist", C.POINTER(C.c_float)), ("len", C.c_int)]
        hid = np.zeros(k + 2, np.uint64)
        hd = np.zeros(k + 2, np.float32)
        return lib, H(hid.ctypes.data_as(C.POINTER(C.c_uint64)), hd.ctypes.data_as(C.POINTER(C.c_float)), 0), hid, hd

    def replay_record(self, q, qlist, state, k, cap):
        qn = q.numpy()
        ql = qlist.numpy()
        si, sd, sn = (t.numpy() for t in state)
        nl = len(ql)
        ri = np.zeros((nl, cap), np.int64)
        rd = np.zeros((nl, cap), np.float32)
        rn = np.zeros(nl, np.int32)
        for li, qi in enumerate(ql):
            lib, h, hid, hd = self._heap(k)
            h.len = int(sn[li])
            hid[:h.len] = si[li, :h.len].view(np.uint64)
            hd[:h.len] = sd[li, :h.len]
            dist_ = self._dists(self._qnorm(qn[qi]))
            n = 0
            for j, e in enumerate(dist_):
                if h.len < k or hd[0] > e:
                    lib.or_insert_to_heap(C.byref(h), k, self.begin + j, float(e))
                    if n < cap:
                        ri[li, n], rd[li, n] = self.begin + j, e
                    n += 1
            rn[li] = cap + 1 if n > cap else n
        return torch.from_numpy(ri), torch.from_numpy(rd), torch.from_numpy(rn)

    def merge_records(self, world, k, cap, st, rec):
        si, sd, sn = (t.numpy() for t in st)
        rids, rds, rns = (t.numpy() for t in rec)
        nl = len(sn)
        oi = np.zeros((nl, k), np.int64)
        od = np.zeros((nl, k), np.float32)
        on = np.zeros(nl, np.int32)
        un = np.zeros(nl, np.int32)
        for li in range(nl):
            lib, h, hid, hd = self._heap(k)
            h.len = int(sn[li])
            hid[:h.len] = si[li, :h.len].view(np.uint64)
            hd[:h.len] = sd[li, :h.len]
            for r in range(1, world):
                m = int(rns[r, li])
                if m > cap:
                    un[li] = 1
                    continue
                for j in range(m):
                    lib.or_insert_to_heap(C.byref(h), k, int(rids[r, li, j]), float(rds[r, li, j]))
            n = lib.or_extract_heap(C.byref(h), oi[li].view(np.uint64).ctypes.data_as(self.o.pu), self.o.f(od[li]))
            on[li] = n
        return torch.from_numpy(oi), torch.from_numpy(od), torch.from_numpy(on), torch.from_numpy(un)

    def merge(self, G, k, ids, dd, cnt, flg):
        """numpy restatement of k_merge_shards (runtime: kernels.hip)."""
        ids, dd, cnt, flg = ids.numpy(), dd.numpy(), cnt.numpy(), flg.numpy()
        nq = cnt.shape[1]
        oi = np.zeros((nq, k), np.int64)
        od = np.zeros((nq, k), np.float32)
        on = np.zeros(nq, np.int32)
        of = np.zeros(nq, np.int32)
        for q in range(nq):
            cand = [(dd[g, q, j], g * (k + 1) + j, ids[g, q, j]) for g in range(G) for j in range(cnt[g, q])]
            cand.sort(key=lambda t: (t[0], t[1]))
            m = min(k + 1, len(cand))
            inc = all(cand[j][0] > cand[j - 1][0] for j in range(1, m))
            n = min(k, len(cand))
            oi[q, :n] = [c[2] for c in cand[:n]]
            od[q, :n] = [c[0] for c in cand[:n]]
            on[q] = n
            of[q] = int(flg[:, q].any() or not inc)
        return torch.from_numpy(oi), torch.from_numpy(od), torch.from_numpy(on), torch.from_numpy(of)

    def replay(self, q, qlist, state, k, extract):
        o = self.o
        lib = o.lib()
        lib.or_find_top_vectors.restype = C.c_int
        lib.or_find_top_vectors.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, o.pf, o.pb, C.c_long, C.c_long,
                                            o.pf, C.c_long, o.pb, C.c_long, C.c_long]

        class H(C.Structure):
            _fields_ = [("id", C.POINTER(C.c_uint64)), ("dist", C.POINTER(C.c_float)), ("len", C.c_int)]
        qlist = qlist.numpy()
        if state is not None:
            state = (state[0].numpy().view(np.uint64), state[1].numpy(), state[2].numpy())
        nl = len(qlist)
        oi = np.zeros((nl, k), np.uint64)
        od = np.zeros((nl, k), np.float32)
        on = np.zeros(nl, np.int32)
        qn = q.numpy()
        for li, qi in enumerate(qlist):
            hid = np.zeros(k + 1, np.uint64)
            hd = np.zeros(k + 1, np.float32)
            ln = 0
            if state is not None:
                ln = int(state[2][li])
                hid[:ln] = state[0][li, :ln]
                hd[:ln] = state[1][li, :ln]
            h = H(hid.ctypes.data_as(C.POINTER(C.c_uint64)), hd.ctypes.data_as(C.POINTER(C.c_float)), ln)
            qv = self._qnorm(qn[qi])
            rc = lib.or_find_top_vectors(C.byref(h), k, self.metric, 1, o.f(self.store),
                                         self.present.ctypes.data_as(o.pb), self.n, self.d, o.f(qv), self.d, None,
                                         self.begin, self.end)
            assert rc == 0
            if extract:
                n = lib.or_extract_heap(C.byref(h), oi[li].ctypes.data_as(o.pu), o.f(od[li]))
                on[li] = n
            else:
                oi[li, :h.len] = hid[:h.len]
                od[li, :h.len] = hd[:h.len]
                on[li] = h.len
        return torch.from_numpy(oi.view(np.int64)), torch.from_numpy(od), torch.from_numpy(on)


def _worker(rank, world, port, metric, kind, n, d, nq, k, dup, outpath, two_phase=True, replay="parallel",
            off_rank=-1):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as orc
    from weaviate_amd.sharded import ShardedFlatSearch
    corpus = orc.gen_matrix(kind, 3, 0, n, d)
    if dup:
        corpus = np.concatenate([corpus[: n // 8]] * 8)
    queries = orc.gen_matrix(kind, 4, 0, nq, d)
    per = (n + world - 1) // world
    b = OracleShardBackend(orc, metric, corpus, rank * per, min(n, (rank + 1) * per))
    if not two_phase:
        b.two_phase = False
    if rank == off_rank:  # this rank's index is off the block-key path (e.g. a non-finite row)
        from weaviate_amd._lib import WV_ERR_UNSUPPORTED, WeaviateError

        def off_path(q, k):
            raise WeaviateError(WV_ERR_UNSUPPORTED, "two-phase shard search: not on the block-key path")
        b.phase1 = off_path
    if replay != "parallel":  # the chain on device flags, or the list chain
        b.replay_record = None
    if replay == "list":
        b.replay_flags = None
    s = ShardedFlatSearch(b, torch.device("cpu"))
    oi, od, on = s.search(torch.from_numpy(queries), k)
    if rank == 0:
        np.savez(outpath, ids=oi.numpy(), dists=od.numpy(), counts=on.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("two_phase,replay,world", [(True, "parallel", 2), (True, "parallel", 3), (False, "parallel", 2),
                                                   (True, "flags", 2), (False, "list", 2)])
@pytest.mark.parametrize("metric,kind,dup", [(0, 0, False), (0, 1, True), (2, 0, True), (1, 1, False)])
def test_sharded_protocol_matches_single_index(tmp_path, oracle, metric, kind, dup, two_phase, replay, world):
    n, d, nq, k = 400, 8, 12, 10
    out = str(tmp_path / "res.npz")
    mp.start_processes(_worker, args=(world, _free_port(), metric, kind, n, d, nq, k, dup, out, two_phase, replay),
                       nprocs=world,
                       join=True, start_method="spawn")
    r = np.load(out)
    corpus = oracle.gen_matrix(kind, 3, 0, n, d)
    if dup:
        corpus = np.concatenate([corpus[: n // 8]] * 8)
    queries = oracle.gen_matrix(kind, 4, 0, nq, d)
    ref = oracle.OracleFlat(metric, 1, d, n)
    ref.add_batch(np.arange(n), corpus)
    for q in range(nq):
        rc, ids, dd = ref.search(queries[q], k)
        c = int(r["counts"][q])
        np.testing.assert_array_equal(r["ids"][q, :c].astype(np.uint64), ids, err_msg=f"q{q}")
        np.testing.assert_array_equal(r["dists"][q, :c].view(np.uint32), dd.view(np.uint32))


@pytest.mark.parametrize("replay,world,off_rank", [("parallel", 2, 1), ("parallel", 3, 0), ("flags", 3, 2)])
def test_sharded_protocol_rank_off_block_key_path(tmp_path, oracle, replay, world, off_rank):
    """One rank's phase 1 is refused (WV_ERR_UNSUPPORTED: its index is off the
    block-key path): it still joins the phase-1 all-gather with +inf keys and
    answers with the one-shot local search, the others keep the two phases;
    no rank waits alone in a collective and the result is the single index's."""
    n, d, nq, k, metric, kind = 400, 8, 10, 10, 0, 1
    out = str(tmp_path / "res.npz")
    mp.start_processes(_worker, args=(world, _free_port(), metric, kind, n, d, nq, k, True, out, True, replay,
                                      off_rank), nprocs=world, join=True, start_method="spawn")
    r = np.load(out)
    corpus = np.concatenate([oracle.gen_matrix(kind, 3, 0, n, d)[: n // 8]] * 8)
    queries = oracle.gen_matrix(kind, 4, 0, nq, d)
    ref = oracle.OracleFlat(metric, 1, d, corpus.shape[0])
    ref.add_batch(np.arange(corpus.shape[0]), corpus)
    for q in range(nq):
        rc, ids, dd = ref.search(queries[q], k)
        c = int(r["counts"][q])
        np.testing.assert_array_equal(r["ids"][q, :c].astype(np.uint64), ids, err_msg=f"q{q}")
        np.testing.assert_array_equal(r["dists"][q, :c].view(np.uint32), dd.view(np.uint32))
