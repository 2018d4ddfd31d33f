"""CPU, world_size 2 and 3 (gloo): the sharded hnsw flat search over PQ codes
of weaviate_amd/sharded.py (ShardedQuantSearch: per-rank compressed distances
and block minima -> the worker heap across the ranks in id order, one parallel
recorded hop or the serial chain -> result heap -> the owners' rescoring ->
h.rescore) reproduces the single index's hnsw.flatSearch (oracle
pq_flat_search) exactly, including ADC tie order.  The per-rank engine is an
oracle-backed stand-in (test infrastructure); the GPU kernels behind the same
interface are covered by tests/test_gpu_sharded_threads.py.
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


class _H(C.Structure):
    _fields_ = [("id", C.POINTER(C.c_uint64)), ("dist", C.POINTER(C.c_float)), ("len", C.c_int)]


class OracleQuantShardBackend:
    """Stand-in for GpuQuantShardBackend (PQ) over rows [begin, end)."""

    def __init__(self, orc, metric, store, centers, begin, end, rl, rescore):
        self.o = orc
        self.metric = metric
        self.store = store  # normalised for cosine
        self.centers = centers
        self.codes = [orc.pq_encode(centers, x) for x in store[begin:end]]
        self.begin, self.end = begin, end
        self.rl, self.rescore = rl, rescore
        lib = orc.lib()
        lib.or_insert_to_heap.argtypes = [C.POINTER(_H), C.c_int, C.c_uint64, C.c_float]
        lib.or_heap_insert.argtypes = [C.POINTER(_H), C.c_uint64, C.c_float]
        lib.or_heap_pop.argtypes = [C.POINTER(_H), C.POINTER(C.c_uint64), C.POINTER(C.c_float)]

    def _heap(self, R):
        hid = np.zeros(R + 2, np.uint64)
        hd = np.zeros(R + 2, np.float32)
        return hid, hd, _H(hid.ctypes.data_as(C.POINTER(C.c_uint64)), hd.ctypes.data_as(C.POINTER(C.c_float)), 0)

    def _pop_all(self, h):
        out = []
        while h.len > 0:
            a, b = C.c_uint64(), C.c_float()
            self.o.lib().or_heap_pop(C.byref(h), C.byref(a), C.byref(b))
            out.append((a.value, b.value))
        return out  # max first

    def quant_begin(self, q, k):
        self.k = k
        qn = q.numpy()
        self.q = np.stack([self.o.normalize(x) if self.metric == self.o.COSINE else x for x in qn])
        self.R = max(self.rl, k) if self.rescore else k
        self.cd = np.array([[self.o.pq_distance(self.metric, self.centers, qv, c) for c in self.codes]
                            for qv in self.q], np.float32)
        return self.R

    def quant_bounds(self):
        nq, R = self.q.shape[0], self.R
        out = np.full((nq, R), np.inf, np.float32)
        for i in range(nq):
            mins = np.array([self.cd[i, b:b + 256].min() for b in range(0, self.cd.shape[1], 256)], np.float32)
            srt = np.sort(mins)[:R]
            out[i, :len(srt)] = srt
        return torch.from_numpy(out)

    def _replay(self, state, i, rec=None, cap=0):
        lib = self.o.lib()
        hid, hd, h = self._heap(self.R)
        if state is not None:
            ln = int(state[2][i])
            hid[:ln] = state[0][i, :ln].numpy().view(np.uint64)
            hd[:ln] = state[1][i, :ln].numpy()
            h.len = ln
        n = 0
        for j in range(self.end - self.begin):
            e = float(self.cd[i, j])
            if h.len < self.R or hd[0] > e:
                lib.or_insert_to_heap(C.byref(h), self.R, self.begin + j, e)
                if rec is not None:
                    if n < cap:
                        rec[0][i, n], rec[1][i, n] = self.begin + j, e
                    n += 1
        return hid, hd, h, n

    def quant_replay(self, state, extract):
        nq, R = self.q.shape[0], self.R
        oi, od, on = np.zeros((nq, R), np.int64), np.zeros((nq, R), np.float32), np.zeros(nq, np.int32)
        for i in range(nq):
            hid, hd, h, _ = self._replay(state, i)
            n = h.len
            if extract:  # ascending
                items = self._pop_all(h)[::-1]
                for j, (a, b) in enumerate(items):
                    oi[i, j], od[i, j] = a, b
            else:
                oi[i, :n] = hid[:n].astype(np.int64)
                od[i, :n] = hd[:n]
            on[i] = n
        return torch.from_numpy(oi), torch.from_numpy(od), torch.from_numpy(on)

    def quant_replay_record(self, state, cap):
        nq = self.q.shape[0]
        ri, rd, rn = np.zeros((nq, cap), np.int64), np.zeros((nq, cap), np.float32), np.zeros(nq, np.int32)
        for i in range(nq):
            n = self._replay(state, i, (ri, rd), cap)[3]
            rn[i] = cap + 1 if n > cap else n
        return torch.from_numpy(ri), torch.from_numpy(rd), torch.from_numpy(rn)

    def merge_records(self, world, k, cap, st, rec):
        lib = self.o.lib()
        si, sd, sn = (t.numpy() for t in st)
        rids, rds, rns = (t.numpy() for t in rec)
        nl = len(sn)
        oi, od = np.zeros((nl, k), np.int64), np.zeros((nl, k), np.float32)
        on, un = np.zeros(nl, np.int32), np.zeros(nl, np.int32)
        for li in range(nl):
            hid, hd, h = self._heap(k)
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
            items = self._pop_all(h)[::-1]
            for j, (a, b) in enumerate(items):
                oi[li, j], od[li, j] = a, b
            on[li] = len(items)
        return torch.from_numpy(oi), torch.from_numpy(od), torch.from_numpy(on), torch.from_numpy(un)

    def quant_finish(self, ai, ad, an):
        lib = self.o.lib()
        ai, ad, an = ai.numpy(), ad.numpy(), an.numpy()
        nq, k, R = ai.shape[0], self.k, self.R
        res = []
        for i in range(nq):  # the result heap in the worker heap's pop order (flat_search.go)
            hid, hd, h = self._heap(R)
            for j in range(int(an[i]) - 1, -1, -1):
                lib.or_insert_to_heap(C.byref(h), R, int(ai[i, j]), float(ad[i, j]))
            res.append(self._pop_all(h)[::-1])  # ascending
        if self.rescore:
            ci, cn = np.full((nq, R), -1, np.int64), np.zeros(nq, np.int32)
            for i, items in enumerate(res):
                for j, (a, _) in enumerate(items):
                    ci[i, j] = a
                cn[i] = len(items)
            return torch.from_numpy(ci), torch.from_numpy(cn)
        oi, od, on = np.zeros((nq, k), np.int64), np.zeros((nq, k), np.float32), np.zeros(nq, np.int32)
        for i, items in enumerate(res):
            for j, (a, b) in enumerate(items[:k]):
                oi[i, j], od[i, j] = a, b
            on[i] = min(len(items), k)
        return torch.from_numpy(oi), torch.from_numpy(od), torch.from_numpy(on)

    def quant_rescore(self, ci, cn):
        ci, cn = ci.numpy(), cn.numpy()
        E = np.zeros(ci.shape, np.float32)
        for i in range(ci.shape[0]):
            for j in range(cn[i]):
                s = int(ci[i, j])
                if self.begin <= s < self.end:
                    E[i, j] = self.o.single_dist(self.metric, 1, self.q[i], self.store[s])
        return torch.from_numpy(E)

    def quant_rescore_final(self, world, id_stride, ci, cn, E_all):
        lib = self.o.lib()
        ci, cn, E_all = ci.numpy(), cn.numpy(), E_all.numpy()
        nq, k = ci.shape[0], self.k
        oi, od, on = np.zeros((nq, k), np.int64), np.zeros((nq, k), np.float32), np.zeros(nq, np.int32)
        for i in range(nq):  # h.rescore: Insert then Pop while Len > k, then extraction
            hid, hd, h = self._heap(k + 1)
            for j in range(cn[i]):
                idv = int(ci[i, j])
                owner = min(idv // id_stride, world - 1)
                lib.or_heap_insert(C.byref(h), idv, float(E_all[owner, i, j]))
                if h.len > k:
                    a, b = C.c_uint64(), C.c_float()
                    lib.or_heap_pop(C.byref(h), C.byref(a), C.byref(b))
            items = self._pop_all(h)[::-1]
            for j, (a, b) in enumerate(items):
                oi[i, j], od[i, j] = a, b
            on[i] = len(items)
        return torch.from_numpy(oi), torch.from_numpy(od), torch.from_numpy(on)


def _setup(orc, metric, kind, n, d, m, ks):
    corpus = orc.gen_matrix(kind, 15, 0, n, d)
    store = np.stack([orc.normalize(x) for x in corpus]) if metric == orc.COSINE else corpus.copy()
    centers = orc.pq_fit(store, m, ks, seed=4)
    return corpus, store, centers


def _worker(rank, world, port, metric, kind, n, d, m, ks, nq, k, rl, rescore, outpath, parallel):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as orc
    from weaviate_amd.sharded import ShardedQuantSearch
    _, store, centers = _setup(orc, metric, kind, n, d, m, ks)
    queries = orc.gen_matrix(kind, 16, 0, nq, d)
    per = (n + world - 1) // world
    b = OracleQuantShardBackend(orc, metric, store, centers, rank * per, min(n, (rank + 1) * per), rl, rescore)
    s = ShardedQuantSearch(b, torch.device("cpu"), per)
    if not parallel:  # the serial worker-heap chain
        s._replay_parallel = lambda nq_, R_: None
    oi, od, on = s.search(torch.from_numpy(queries), k)
    if rank == 0:
        np.savez(outpath, ids=oi.numpy(), dists=od.numpy(), counts=on.numpy(), path=np.array(s.path))
    dist.destroy_process_group()


# parallel: each shard needs >= R 256-row blocks for a finite bound T_r
@pytest.mark.parametrize("world,metric,kind,rl,rescore,parallel,n", [
    (2, 0, 0, -1, False, True, 5400),     # l2, worker heap = k, parallel hop
    (3, 2, 0, 12, True, True, 46080),     # cosine, rescoring by the owners (60 blocks per shard)
    (2, 0, 1, 16, True, False, 3000),     # integer data (ADC ties), the serial chain
    (3, 1, 0, -1, False, False, 3000),    # dot, chain
])
def test_sharded_quant_matches_single_index(tmp_path, oracle, world, metric, kind, rl, rescore, parallel, n):
    d, m, ks, nq, k = 16, 4, 16, 5, 8
    out = str(tmp_path / "res.npz")
    mp.start_processes(_worker, args=(world, _free_port(), metric, kind, n, d, m, ks, nq, k, rl, rescore, out, parallel),
                       nprocs=world, join=True, start_method="spawn")
    r = np.load(out)
    if parallel and kind != 1:
        assert str(r["path"]) == "parallel"
    corpus, store, centers = _setup(oracle, metric, kind, n, d, m, ks)
    codes = np.stack([oracle.pq_encode(centers, x) for x in store])
    queries = oracle.gen_matrix(kind, 16, 0, nq, d)
    present = np.ones(n, np.uint8)
    R = max(rl, k) if rescore else k
    for q in range(nq):
        qv = oracle.normalize(queries[q]) if metric == oracle.COSINE else queries[q]
        ids, dd = oracle.pq_flat_search(metric, 1, centers, codes, store, present, qv, k, R, rescore)
        c = int(r["counts"][q])
        np.testing.assert_array_equal(r["ids"][q, :c].astype(np.uint64), ids, err_msg=f"q{q}")
        np.testing.assert_array_equal(r["dists"][q, :c].view(np.uint32), dd.view(np.uint32), err_msg=f"q{q}")
