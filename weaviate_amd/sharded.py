"""Corpus sharded across the GPUs of one node (one process per GPU).

Mirrors Weaviate's shard-local top-k + coordinator merge
(adapters/repos/db/index.go:1928-2071) with contiguous doc-id ranges per rank,
so the id-ordered scan of the single reference index is the concatenation of
the rank scans in rank order.  Exactness:

1. every rank computes its block keys and its k+1 smallest block-key values
   (phase 1); one all-gather of those (B*(k+2)*4 bytes per rank) gives every
   rank the global (k+1)-th smallest key, which cuts its candidate blocks to
   those that can hold a global top-(k+1) row; exact distances of those rows
   give the rank's verified top-(k+1) or a flag (phase 2).  Backends without
   the two phases run both at once (mode 1 of wv_index_search_device);
2. one all-gather of the packed lists (B*(3(k+1)+2)*4 bytes per rank) and an
   on-device merge (wv_merge_shards);
3. if no rank flagged a query and the merged k+1 smallest distances are
   distinct, the merged top-k IS the reference heap's result;
4. otherwise the reference heap is replayed exactly across the ranks in id
   order: rank r continues the heap states handed over by rank r-1 (one packed
   broadcast per hop, states indexed by query, the flagged list built on the
   device: no host synchronisation), the last rank applies extractHeap.

The GPU product path is the library's multi-shard index (multi.hip, the
wv_multi_* C ABI): it runs these protocols -- exact two-phase, BQ R-heap,
PQ / SQ / rq worker heap, allow lists -- in C++ with its own RCCL
communicator, so a cgo host reaches them without Python.  open_multi() below
is the thin torch.distributed client of it (one process per GPU, rank 0's
RCCL id broadcast over the launcher's group).  The protocol classes that
follow (ShardedFlatSearch, ShardedBQSearch, ShardedQuantSearch) are the same
protocols over torch.distributed with the per-rank kernels behind a small
backend interface, kept as the CPU-testable statement of the protocols
(gloo, oracle-backed backends: tests/test_sharded*_gloo.py).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch.distributed import ReduceOp


def open_multi(n_total: int, local_rank: int, **index_kw):
    """The corpus of n_total doc ids over the ranks of the default process
    group (contiguous id ranges of ceil(n_total / world)), this process's rank
    as one shard of a wv_multi index on GPU `local_rank` with a library-owned
    RCCL communicator (weaviate_amd.multi.MultiFlatIndex).  index_kw: the
    shards' FlatIndex configuration (distance, dims, bq, rescore_limit, pq, rq,
    sq, variant)."""
    from .multi import MultiFlatIndex, rccl_unique_id
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    uid = [rccl_unique_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(uid, src=0)
    return MultiFlatIndex(devices=[local_rank], world=world, rank0=rank, id_stride=(n_total + world - 1) // world,
                          transport="rccl", unique_id=uid[0], **index_kw)


def prefix_bound(r: int, ql: torch.Tensor, k: int, gd, gc, gf, bounds=None) -> torch.Tensor:
    """T_r [F] for the listed queries ql: the k-th smallest of upper bounds of
    distinct rows of the shards before r -- exact distances from their
    unflagged lists (gd [W, nq, k+1], counts gc, flags gf), and the block-key
    bounds A + eps of their phase-1 keys (bounds = (gA [W, nq, k+1], gE [W, nq]));
    +inf when fewer than k are known.  Each source gives its own k-th smallest
    (the two may name the same row); T_r is the smaller.  The real heap top at
    shard r's first row is at most T_r (the heap holds the k smallest
    distances seen)."""
    F = int(ql.numel())
    k1 = gd.shape[-1]
    inf = torch.full((F,), float("inf"), dtype=torch.float32, device=gd.device)

    def kth(v):  # k-th smallest per row; the values of one source belong to distinct rows
        return torch.kthvalue(v, k, dim=1).values.contiguous() if v.shape[1] >= k and F > 0 else inf

    ex = gd[:r][:, ql, :]
    ok = (torch.arange(k1, device=gd.device)[None, None, :] < gc[:r][:, ql, None]) & (gf[:r][:, ql, None] == 0)
    T = kth(torch.where(ok, ex, torch.full_like(ex, float("inf"))).permute(1, 0, 2).reshape(F, r * k1))
    if bounds is not None:  # a separate order statistic: a listed row may also be a block's bound row
        gA, gE = bounds
        T = torch.minimum(T, kth((gA[:r][:, ql, :] + gE[:r][:, ql, None]).permute(1, 0, 2).reshape(F, r * k1)))
    return T


def fake_heaps(T: torch.Tensor, k: int):
    """Full heaps of k copies of T (ids -1), empty where T is infinite."""
    F = int(T.numel())
    return (torch.full((F, k), -1, dtype=torch.int64, device=T.device), T[:, None].expand(F, k).contiguous(),
            torch.where(torch.isfinite(T), k, 0).to(torch.int32))


class GpuShardBackend:
    """Rank-local engine: a FlatIndex holding ids [id_base, id_base + n)."""

    def __init__(self, index, device: int):
        self.index = index
        self.device = device
        self.dev = torch.device("cuda", device)
        from . import _lib
        self._l = _lib.load()
        self._check = _lib.check

    def local_search(self, q: torch.Tensor, k: int):
        nq, d = q.shape
        ids = torch.empty((nq, k + 1), dtype=torch.int64, device=self.dev)
        dd = torch.empty((nq, k + 1), dtype=torch.float32, device=self.dev)
        cnt = torch.empty(nq, dtype=torch.int32, device=self.dev)
        flg = torch.empty(nq, dtype=torch.int32, device=self.dev)
        s = torch.cuda.current_stream(self.dev).cuda_stream
        self._check(self._l.wv_index_search_device(self.index._h, q.data_ptr(), nq, d, k, 1, ids.data_ptr(),
                                                   dd.data_ptr(), cnt.data_ptr(), flg.data_ptr(), s))
        return ids, dd, cnt, flg

    two_phase = True

    def phase1(self, q: torch.Tensor, k: int):
        """Block keys + local candidate selection; -> (topA [nq][k+1], eps [nq]).
        Raises WeaviateError (WV_ERR_UNSUPPORTED) when the index is not on the
        block-key path; the caller then uses local_search."""
        nq, d = q.shape
        topA = torch.empty((nq, k + 1), dtype=torch.float32, device=self.dev)
        eps = torch.empty(nq, dtype=torch.float32, device=self.dev)
        s = torch.cuda.current_stream(self.dev).cuda_stream
        self._check(self._l.wv_index_shard_phase1(self.index._h, q.data_ptr(), nq, d, k, topA.data_ptr(),
                                                  eps.data_ptr(), s))
        self._nq = nq
        return topA, eps

    def phase2(self, gA: torch.Tensor, gE: torch.Tensor, k: int):
        """Global threshold + exact distances; -> the local_search tensors."""
        W, nq = int(gA.shape[0]), int(gA.shape[1])
        ids = torch.empty((nq, k + 1), dtype=torch.int64, device=self.dev)
        dd = torch.empty((nq, k + 1), dtype=torch.float32, device=self.dev)
        cnt = torch.empty(nq, dtype=torch.int32, device=self.dev)
        flg = torch.empty(nq, dtype=torch.int32, device=self.dev)
        s = torch.cuda.current_stream(self.dev).cuda_stream
        self._check(self._l.wv_index_shard_phase2(self.index._h, W, nq, gA.data_ptr(), gE.data_ptr(), k,
                                                  ids.data_ptr(), dd.data_ptr(), cnt.data_ptr(), flg.data_ptr(), s))
        return ids, dd, cnt, flg

    def replay_flags(self, q: torch.Tensor, flags: torch.Tensor, state, k: int, extract: bool, out=None):
        """Continue the reference heap of every flagged query over this shard
        (wv_index_replay_flags_device: the list is built on the device).  state
        and result rows are indexed by query: (ids [nq, k], dists [nq, k],
        len [nq]) in heap layout order, or None for empty heaps; `out` receives
        the result (rows of unflagged queries are left untouched)."""
        nq = q.shape[0]
        if out is None:
            out = (torch.empty((nq, k), dtype=torch.int64, device=self.dev),
                   torch.empty((nq, k), dtype=torch.float32, device=self.dev),
                   torch.empty(nq, dtype=torch.int32, device=self.dev))
        si, sd, sl = (None, None, None) if state is None else (state[0].data_ptr(), state[1].data_ptr(),
                                                               state[2].data_ptr())
        s = torch.cuda.current_stream(self.dev).cuda_stream
        self._check(self._l.wv_index_replay_flags_device(self.index._h, q.data_ptr(), nq, q.shape[1], k,
                                                         flags.data_ptr(), si, sd, sl, 1 if extract else 0,
                                                         out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), s))
        return out

    def replay_record(self, q: torch.Tensor, qlist: torch.Tensor, state, k: int, cap: int):
        """This shard's replay of the listed queries from `state` (by list
        position), recording every insertion: (ids [nl, cap], dists, n [nl]),
        n = cap + 1 when the record overflowed."""
        nl = int(qlist.numel())
        ri = torch.empty((nl, cap), dtype=torch.int64, device=self.dev)
        rd = torch.empty((nl, cap), dtype=torch.float32, device=self.dev)
        rn = torch.empty(nl, dtype=torch.int32, device=self.dev)
        if nl == 0:
            return ri, rd, rn
        s = torch.cuda.current_stream(self.dev).cuda_stream
        self._check(self._l.wv_index_replay_record_device(self.index._h, q.data_ptr(), q.shape[0], q.shape[1], k,
                                                          qlist.data_ptr(), nl, state[0].data_ptr(),
                                                          state[1].data_ptr(), state[2].data_ptr(), cap,
                                                          ri.data_ptr(), rd.data_ptr(), rn.data_ptr(), s))
        return ri, rd, rn

    def merge_records(self, world: int, k: int, cap: int, st, rec):
        """Shard 0's states + the later shards' records -> extracted results
        [nl, k] and unresolved [nl] (wv_heap_merge_records)."""
        nl = int(st[2].numel())
        oi = torch.empty((nl, k), dtype=torch.int64, device=self.dev)
        od = torch.empty((nl, k), dtype=torch.float32, device=self.dev)
        on = torch.empty(nl, dtype=torch.int32, device=self.dev)
        un = torch.zeros(nl, dtype=torch.int32, device=self.dev)
        if nl == 0:
            return oi, od, on, un
        s = torch.cuda.current_stream(self.dev).cuda_stream
        self._check(self._l.wv_heap_merge_records(self.device, nl, k, world, cap, st[0].data_ptr(), st[1].data_ptr(),
                                                  st[2].data_ptr(), rec[0].data_ptr(), rec[1].data_ptr(),
                                                  rec[2].data_ptr(), oi.data_ptr(), od.data_ptr(), on.data_ptr(),
                                                  un.data_ptr(), s))
        return oi, od, on, un

    def merge(self, G: int, k: int, ids, dd, cnt, flg):
        nq = cnt.shape[-1]
        oi = torch.empty((nq, k), dtype=torch.int64, device=self.dev)
        od = torch.empty((nq, k), dtype=torch.float32, device=self.dev)
        on = torch.empty(nq, dtype=torch.int32, device=self.dev)
        of = torch.empty(nq, dtype=torch.int32, device=self.dev)
        s = torch.cuda.current_stream(self.dev).cuda_stream
        self._check(self._l.wv_merge_shards(self.device, G, nq, k, ids.data_ptr(), dd.data_ptr(), cnt.data_ptr(),
                                            flg.data_ptr(), oi.data_ptr(), od.data_ptr(), on.data_ptr(),
                                            of.data_ptr(), s))
        return oi, od, on, of

    def replay(self, q: torch.Tensor, qlist: torch.Tensor, state, k: int, extract: bool):
        """Continue the reference heap over this shard for the listed query rows
        (wv_index_replay_device: device tensors in and out, stream-ordered).
        state: (ids int64 [nl, k], dists float32 [nl, k], len int32 [nl]) in
        heap layout order, or None for empty heaps."""
        nl = int(qlist.numel())
        oi = torch.empty((nl, k), dtype=torch.int64, device=self.dev)
        od = torch.empty((nl, k), dtype=torch.float32, device=self.dev)
        on = torch.empty(nl, dtype=torch.int32, device=self.dev)
        si, sd, sl = (None, None, None) if state is None else (state[0].data_ptr(), state[1].data_ptr(),
                                                               state[2].data_ptr())
        s = torch.cuda.current_stream(self.dev).cuda_stream
        self._check(self._l.wv_index_replay_device(self.index._h, q.data_ptr(), q.shape[0], q.shape[1], k,
                                                   qlist.data_ptr(), nl, si, sd, sl, 1 if extract else 0,
                                                   oi.data_ptr(), od.data_ptr(), on.data_ptr(), s))
        return oi, od, on


class GpuBQShardBackend(GpuShardBackend):
    """Rank-local BQ engine (wv_index_bq_* entry points, include/wv_knn.h)."""

    def R(self, k: int) -> int:
        return max(int(self.index.rescore_limit), k)

    def _s(self):
        return torch.cuda.current_stream(self.dev).cuda_stream

    def bq_begin(self, q: torch.Tensor, k: int):
        nq, d = q.shape
        self.nq, self.k = nq, k
        self._check(self._l.wv_index_bq_begin(self.index._h, q.data_ptr(), nq, d, k, self._s()))

    def bq_replay(self, state, pop: bool):
        R = self.R(self.k)
        ids = torch.empty((self.nq, R), dtype=torch.int64, device=self.dev)
        dd = torch.empty((self.nq, R), dtype=torch.float32, device=self.dev)
        ln = torch.empty(self.nq, dtype=torch.int32, device=self.dev)
        si, sd, sl = (None, None, None) if state is None else (state[0].data_ptr(), state[1].data_ptr(),
                                                               state[2].data_ptr())
        self._check(self._l.wv_index_bq_replay(self.index._h, si, sd, sl, 1 if pop else 0, ids.data_ptr(),
                                               dd.data_ptr(), ln.data_ptr(), self._s()))
        return ids, dd, ln

    def bq_bounds(self):
        """[nq, R] ascending: the R smallest block minima of this shard (+inf padded)."""
        R = self.R(self.k)
        out = torch.empty((self.nq, R), dtype=torch.float32, device=self.dev)
        self._check(self._l.wv_index_bq_bounds(self.index._h, out.data_ptr(), self._s()))
        return out

    def bq_replay_record(self, state, cap: int):
        """This shard's R-heap replay from `state` (by query), recording every
        insertion: (ids [nq, cap], dists, n [nq]), n = cap + 1 on overflow."""
        ri = torch.empty((self.nq, cap), dtype=torch.int64, device=self.dev)
        rd = torch.empty((self.nq, cap), dtype=torch.float32, device=self.dev)
        rn = torch.empty(self.nq, dtype=torch.int32, device=self.dev)
        self._check(self._l.wv_index_bq_replay_record(self.index._h, state[0].data_ptr(), state[1].data_ptr(),
                                                      state[2].data_ptr(), cap, ri.data_ptr(), rd.data_ptr(),
                                                      rn.data_ptr(), self._s()))
        return ri, rd, rn

    def bq_rescore(self, ids, ln):
        E = torch.zeros(ids.shape, dtype=torch.float32, device=self.dev)
        self._check(self._l.wv_index_bq_rescore(self.index._h, ids.data_ptr(), ln.data_ptr(), E.data_ptr(),
                                                self._s()))
        return E

    def bq_final(self, world: int, id_stride: int, ids, ln, E_all):
        nq, R = ids.shape
        oi = torch.empty((nq, self.k), dtype=torch.int64, device=self.dev)
        od = torch.empty((nq, self.k), dtype=torch.float32, device=self.dev)
        on = torch.empty(nq, dtype=torch.int32, device=self.dev)
        self._check(self._l.wv_bq_final(self.device, nq, R, self.k, world, id_stride, ids.data_ptr(), ln.data_ptr(),
                                        E_all.data_ptr(), oi.data_ptr(), od.data_ptr(), on.data_ptr(), self._s()))
        return oi, od, on


class ShardedBQSearch:
    """BQ-compressed search over contiguous id-range shards (one per rank) with
    the single index's exact semantics (flat/index.go:460-532):
      1. every rank: query codes + hamming block minima of its shard (parallel,
         the expensive VALU pass);
      2. the R-heap over all shards in id order, in one parallel hop (backends
         with bq_replay_record): each rank's R smallest block minima are
         all-gathered; rank r >= 1 replays its range from R copies of T_r (the
         R-th smallest minimum of the ranks before it: distances of distinct
         rows, so T_r >= the real heap top at its first row) and records every
         insertion; rank 0 replays from empty heaps; one all-gather of the
         records, and every rank applies them on rank 0's states in rank
         order (wv_heap_merge_records) -- the serial chain's heaps.  A record
         that overflows its cap sends the batch down the serial chain (rank r
         continues rank r-1's heap states, one broadcast per hop);
      3. every rank rescores the candidates it holds (exact SingleDist) in the
         reference's pop order, all-gather of the [B][R] distance tiles;
      4. the rescoring heap (insertToHeap in pop order, extractHeap)."""

    def __init__(self, backend, device: torch.device, id_stride: int):
        self.b = backend
        self.dev = device
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.id_stride = int(id_stride)

    def _all_gather(self, t: torch.Tensor) -> torch.Tensor:
        return ShardedFlatSearch._all_gather(self, t)

    def search(self, q: torch.Tensor, k: int):
        nq = q.shape[0]
        R = self.b.R(k)
        self.b.bq_begin(q, k)
        self.path = "chain"
        if getattr(self.b, "bq_replay_record", None) is not None and self.world > 1:
            res = self._replay_parallel(nq, R)
            if res is not None:
                self.path = "parallel"
                ids, ln = res
                E = self.b.bq_rescore(ids, ln)
                E_all = self._all_gather(E)
                return self.b.bq_final(self.world, self.id_stride, ids, ln, E_all)
        return self._chain(q, nq, R)

    def _replay_parallel(self, nq: int, R: int):
        """Step 2 in one hop; -> (candidate ids in pop order [nq, R], lengths)
        or None when a record overflowed (host sync: one flag)."""
        cap = 2 * R
        G = self._all_gather(self.b.bq_bounds())  # [W, nq, R]
        if self.rank == 0:
            ti, td, tn = self.b.bq_replay(None, False)  # heap states from empty heaps
            ri = torch.zeros((nq, cap), dtype=torch.int64, device=self.dev)
            rd = torch.zeros((nq, cap), dtype=torch.float32, device=self.dev)
            ri[:, :R], rd[:, :R] = ti, td
            rn = tn
        else:
            allq = torch.arange(nq, device=self.dev)
            T = prefix_bound(self.rank, allq, R, G, torch.full((self.rank, nq), R, dtype=torch.int32, device=self.dev),
                             torch.zeros((self.rank, nq), dtype=torch.int32, device=self.dev))
            ri, rd, rn = self.b.bq_replay_record(fake_heaps(T, R), cap)
        pk = torch.cat([ri.contiguous().view(torch.int32).reshape(nq, 2 * cap), rd.contiguous().view(torch.int32),
                        rn[:, None]], 1)
        A = self._all_gather(pk)  # [W, nq, 3 cap + 1]
        rec = (A[..., : 2 * cap].contiguous().view(torch.int64), A[..., 2 * cap: 3 * cap].contiguous().view(torch.float32),
               A[..., 3 * cap].contiguous())
        st = (rec[0][0, :, :R].contiguous(), rec[1][0, :, :R].contiguous(), rec[2][0].contiguous())
        ai, _, an, un = self.b.merge_records(self.world, R, cap, st, rec)  # extracted ascending
        if bool(un.any()):
            return None
        # pop order (max first) = the ascending extraction read back to front
        back = (an[:, None].long() - 1 - torch.arange(R, device=self.dev)[None, :]).clamp(min=0)
        return ai.gather(1, back), an

    def _chain(self, q: torch.Tensor, nq: int, R: int):
        """Step 2 as the serial chain: rank r continues rank r-1's heaps."""
        state = None
        for r in range(self.world):
            last = r == self.world - 1
            if self.rank == r:  # one packed broadcast per hop: [nq][2R ids | R dists | len]
                buf = ShardedFlatSearch._pack_state(*self.b.bq_replay(state, last))
            else:
                buf = torch.empty((nq, 3 * R + 1), dtype=torch.int32, device=self.dev)
            dist.broadcast(buf, src=r)
            state = ShardedFlatSearch._unpack_state(buf, R)
        ids, _, ln = state
        E = self.b.bq_rescore(ids, ln)
        E_all = self._all_gather(E)
        return self.b.bq_final(self.world, self.id_stride, ids, ln, E_all)


class GpuQuantShardBackend(GpuShardBackend):
    """Rank-local engine of the search over compressed vectors (wv_index_quant_*
    entry points, include/wv_knn.h): a trained PQ, an SQ or a flat rq-8 / rq-1
    index holding ids [id_base, id_base + n), the quantizer shared by all ranks
    (RQ: the same seeded rotation on every rank)."""

    def _s(self):
        return torch.cuda.current_stream(self.dev).cuda_stream

    def quant_begin(self, q: torch.Tensor, k: int):
        import ctypes
        nq, d = q.shape
        out = (ctypes.c_int64 * 4)()
        self._check(self._l.wv_index_quant_begin(self.index._h, q.data_ptr(), nq, d, k, ctypes.addressof(out), self._s()))
        self.nq, self.k = nq, k
        self.R, self.nblk, self.rescore, self.form = int(out[0]), int(out[1]), bool(out[2]), int(out[3])
        return self.R

    def max_batch(self, k: int, world: int) -> int:
        """Queries per quant_begin on this shard: its distance group, LUT and
        the all-gathered replay records all fit (wv_index_quant_max_batch)."""
        import ctypes
        out = ctypes.c_int64()
        self._check(self._l.wv_index_quant_max_batch(self.index._h, int(k), int(world), ctypes.addressof(out)))
        return int(out.value)

    def quant_bounds(self):
        """[nq, R] ascending: the R smallest block minima of this shard (+inf padded)."""
        bm = torch.empty((self.nq, self.nblk), dtype=torch.float32, device=self.dev)
        self._check(self._l.wv_index_quant_blockmin(self.index._h, bm.data_ptr(), self._s()))
        out = torch.full((self.nq, self.R), float("inf"), dtype=torch.float32, device=self.dev)
        m = min(self.R, self.nblk)
        out[:, :m] = torch.topk(bm, m, dim=1, largest=False, sorted=True).values
        return out

    def quant_replay(self, state, extract: bool):
        ids = torch.empty((self.nq, self.R), dtype=torch.int64, device=self.dev)
        dd = torch.empty((self.nq, self.R), dtype=torch.float32, device=self.dev)
        ln = torch.empty(self.nq, dtype=torch.int32, device=self.dev)
        si, sd, sl = (None, None, None) if state is None else (state[0].data_ptr(), state[1].data_ptr(),
                                                               state[2].data_ptr())
        self._check(self._l.wv_index_quant_replay(self.index._h, si, sd, sl, 1 if extract else 0, ids.data_ptr(),
                                                  dd.data_ptr(), ln.data_ptr(), self._s()))
        return ids, dd, ln

    def quant_replay_record(self, state, cap: int):
        ri = torch.empty((self.nq, cap), dtype=torch.int64, device=self.dev)
        rd = torch.empty((self.nq, cap), dtype=torch.float32, device=self.dev)
        rn = torch.empty(self.nq, dtype=torch.int32, device=self.dev)
        self._check(self._l.wv_index_quant_replay_record(self.index._h, state[0].data_ptr(), state[1].data_ptr(),
                                                         state[2].data_ptr(), cap, ri.data_ptr(), rd.data_ptr(),
                                                         rn.data_ptr(), self._s()))
        return ri, rd, rn

    def quant_finish(self, ai, ad, an):
        """-> (ids, dists, counts) [nq, k] without rescoring, else the rescoring
        candidates (global ids [nq, R], counts)."""
        k = self.k
        if self.rescore:
            ci = torch.empty((self.nq, self.R), dtype=torch.int64, device=self.dev)
            cn = torch.empty(self.nq, dtype=torch.int32, device=self.dev)
            self._check(self._l.wv_index_quant_finish(self.index._h, ai.data_ptr(), ad.data_ptr(), an.data_ptr(),
                                                      None, None, None, ci.data_ptr(), cn.data_ptr(), self._s()))
            return ci, cn
        oi = torch.empty((self.nq, k), dtype=torch.int64, device=self.dev)
        od = torch.empty((self.nq, k), dtype=torch.float32, device=self.dev)
        on = torch.empty(self.nq, dtype=torch.int32, device=self.dev)
        self._check(self._l.wv_index_quant_finish(self.index._h, ai.data_ptr(), ad.data_ptr(), an.data_ptr(),
                                                  oi.data_ptr(), od.data_ptr(), on.data_ptr(), None, None, self._s()))
        return oi, od, on

    def quant_rescore(self, ci, cn):
        E = torch.zeros(ci.shape, dtype=torch.float32, device=self.dev)
        self._check(self._l.wv_index_quant_rescore(self.index._h, ci.data_ptr(), cn.data_ptr(), E.data_ptr(),
                                                   self._s()))
        return E

    def quant_rescore_final(self, world: int, id_stride: int, ci, cn, E_all):
        nq, R = ci.shape
        oi = torch.empty((nq, self.k), dtype=torch.int64, device=self.dev)
        od = torch.empty((nq, self.k), dtype=torch.float32, device=self.dev)
        on = torch.empty(nq, dtype=torch.int32, device=self.dev)
        self._check(self._l.wv_quant_rescore_final(self.device, self.form, nq, R, self.k, world, id_stride, ci.data_ptr(),
                                                   cn.data_ptr(), E_all.data_ptr(), oi.data_ptr(), od.data_ptr(),
                                                   on.data_ptr(), self._s()))
        return oi, od, on


class ShardedQuantSearch:
    """hnsw's flat search over compressed vectors (trained PQ, SQ;
    hnsw/flat_search.go:28-141 + h.rescore, hnsw/search.go:1047-1110) and
    flat's searchByVectorQuantized over rq-8 / rq-1 codes
    (flat/index.go:460-532: every worker-heap item rescored) over
    contiguous id-range shards with the single index's exact semantics:
      1. every rank: the compressed distances of its rows to the batch and
         their 256-row block minima (wv_index_quant_begin, parallel);
      2. the worker heap (limit R) over all shards in id order in one parallel
         hop, BQ's record scheme (ShardedBQSearch): the R smallest block minima
         of each rank are all-gathered; rank r >= 1 replays from R copies of
         T_r and records its insertions; rank 0 replays from empty heaps; the
         records are all-gathered and merged on rank 0's states
         (wv_heap_merge_records).  A record over its cap sends the batch down
         the serial chain;
      3. the result heap in pop order; with rescoring, every rank computes the
         exact distances of the candidates it holds, one all-gather, and
         h.rescore picks each candidate's distance from its owner."""

    def __init__(self, backend, device: torch.device, id_stride: int):
        self.b = backend
        self.dev = device
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.id_stride = int(id_stride)

    def _all_gather(self, t: torch.Tensor) -> torch.Tensor:
        return ShardedFlatSearch._all_gather(self, t)

    def search(self, q: torch.Tensor, k: int):
        """Query chunks that every rank's distance group holds (one all-reduce
        agrees on the size), each through steps 1-3."""
        nq = q.shape[0]
        mb = getattr(self.b, "max_batch", None)
        chunk = nq
        if mb is not None:
            t = torch.tensor([min(int(mb(k, self.world)), nq)], dtype=torch.int64, device=self.dev)
            if self.world > 1:
                dist.all_reduce(t, op=ReduceOp.MIN)
            chunk = max(1, int(t.item()))
        if chunk >= nq:
            return self._search(q, k)
        parts = [self._search(q[i:i + chunk], k) for i in range(0, nq, chunk)]
        return tuple(torch.cat(p) for p in zip(*parts))

    def _search(self, q: torch.Tensor, k: int):
        nq = q.shape[0]
        R = self.b.quant_begin(q, k)
        self.path = "chain"
        res = self._replay_parallel(nq, R) if self.world > 1 else None
        if res is not None:
            self.path = "parallel"
            ai, ad, an = res
        else:
            ai, ad, an = self._chain(nq, R)
        fin = self.b.quant_finish(ai, ad, an)
        if not self.b.rescore:
            return fin
        ci, cn = fin
        E_all = self._all_gather(self.b.quant_rescore(ci, cn))
        return self.b.quant_rescore_final(self.world, self.id_stride, ci, cn, E_all)

    def _replay_parallel(self, nq: int, R: int):
        """Step 2 in one hop; -> the merged worker heaps extracted ascending, or
        None when a record overflowed (host sync: one flag).  A small worker
        heap (PQ without rescoring: R = k) records a few dozen insertions
        beyond R on a shard holding that many rows under T_r: cap = 2R + 64."""
        cap = 2 * R + 64
        G = self._all_gather(self.b.quant_bounds())  # [W, nq, R]
        if self.rank == 0:
            ti, td, tn = self.b.quant_replay(None, False)  # heap states from empty heaps
            ri = torch.zeros((nq, cap), dtype=torch.int64, device=self.dev)
            rd = torch.zeros((nq, cap), dtype=torch.float32, device=self.dev)
            ri[:, :R], rd[:, :R] = ti, td
            rn = tn
        else:
            allq = torch.arange(nq, device=self.dev)
            T = prefix_bound(self.rank, allq, R, G, torch.full((self.rank, nq), R, dtype=torch.int32, device=self.dev),
                             torch.zeros((self.rank, nq), dtype=torch.int32, device=self.dev))
            ri, rd, rn = self.b.quant_replay_record(fake_heaps(T, R), cap)
        pk = torch.cat([ri.contiguous().view(torch.int32).reshape(nq, 2 * cap), rd.contiguous().view(torch.int32),
                        rn[:, None]], 1)
        A = self._all_gather(pk)  # [W, nq, 3 cap + 1]
        rec = (A[..., : 2 * cap].contiguous().view(torch.int64), A[..., 2 * cap: 3 * cap].contiguous().view(torch.float32),
               A[..., 3 * cap].contiguous())
        st = (rec[0][0, :, :R].contiguous(), rec[1][0, :, :R].contiguous(), rec[2][0].contiguous())
        ai, ad, an, un = self.b.merge_records(self.world, R, cap, st, rec)  # extracted ascending
        if bool(un.any()):
            return None
        return ai, ad, an

    def _chain(self, nq: int, R: int):
        """Step 2 as the serial chain: rank r continues rank r-1's heaps; the
        last rank extracts (ascending)."""
        state = None
        for r in range(self.world):
            last = r == self.world - 1
            if self.rank == r:  # one packed broadcast per hop: [nq][2R ids | R dists | len]
                buf = ShardedFlatSearch._pack_state(*self.b.quant_replay(state, last))
            else:
                buf = torch.empty((nq, 3 * R + 1), dtype=torch.int32, device=self.dev)
            dist.broadcast(buf, src=r)
            state = ShardedFlatSearch._unpack_state(buf, R)
        return state


class ShardedFlatSearch:
    """search(queries) over all ranks of the default process group."""

    def __init__(self, backend, device: torch.device):
        self.b = backend
        self.dev = device
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.flagged = 0  # queries that went through the cross-shard replay (device tensor after a search)

    def _all_gather(self, t: torch.Tensor) -> torch.Tensor:
        t = t.contiguous()
        if dist.get_backend() == "nccl":  # RCCL: one fused gather into a [world, ...] tensor
            out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(out, t)
            return out
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t)
        return torch.stack(parts)

    def _local(self, q: torch.Tensor, k: int):
        """Phases 1-2 (or the one-shot local search) -> the rank's lists.

        Every rank takes part in the phase-1 all-gather, also a rank whose
        index is off the block-key path (non-finite rows, an empty shard, k or
        a batch the path does not take): it contributes +inf keys and eps 0 --
        no bound rows, so the global (k+1)-th key of the other ranks stays a
        valid cut (fewer sources only weaken it) -- and answers with the
        one-shot local search."""
        if getattr(self.b, "two_phase", False):
            off = False
            try:
                topA, eps = self.b.phase1(q, k)
            except Exception as e:
                from ._lib import WeaviateError, WV_ERR_UNSUPPORTED
                if not (isinstance(e, WeaviateError) and e.code == WV_ERR_UNSUPPORTED):
                    raise
                off = True
                topA = torch.full((q.shape[0], k + 1), float("inf"), dtype=torch.float32, device=q.device)
                eps = torch.zeros(q.shape[0], dtype=torch.float32, device=q.device)
            g = self._all_gather(torch.cat([topA, eps[:, None]], 1))  # [W, nq, k+2]
            gA, gE = g[..., : k + 1].contiguous(), g[..., k + 1].contiguous()
            self._bounds = (gA, gE)
            if not off:
                return self.b.phase2(gA, gE, k)
        return self.b.local_search(q, k)

    def search(self, q: torch.Tensor, k: int):
        self._bounds = None
        ids, dd, cnt, flg = self._local(q, k)
        nq = cnt.shape[0]
        # one all-gather of the packed lists: ids (as 2 int32), dists, count, flag
        packed = torch.cat([ids.contiguous().view(torch.int32).reshape(nq, 2 * (k + 1)),
                            dd.contiguous().view(torch.int32), cnt[:, None], flg[:, None]], 1)
        G = self._all_gather(packed)
        k1 = k + 1
        gi = G[..., : 2 * k1].contiguous().view(torch.int64)
        gd = G[..., 2 * k1: 3 * k1].contiguous().view(torch.float32)
        gc = G[..., 3 * k1].contiguous()
        gf = G[..., 3 * k1 + 1].contiguous()
        oi, od, on, of = self.b.merge(self.world, k, gi, gd, gc, gf)
        self.flagged = self.flagged + (of != 0).sum()  # no host sync
        if getattr(self.b, "replay_record", None) is not None and k < 64:
            return self._replay_parallel(q, k, of, oi, od, on, gd, gc, gf)
        if getattr(self.b, "replay_flags", None) is not None:
            return self._replay_chain_flags(q, k, of, oi, od, on)
        flagged = torch.nonzero(of).flatten().to(torch.int32)  # (host sync: the list length)
        if flagged.numel():
            oi, od, on = self._replay_chain(q, k, flagged, oi, od, on)
        return oi, od, on

    def _replay_parallel(self, q, k, of, oi, od, on, gd, gc, gf):
        """The cross-shard replay in one parallel hop: shard 0 replays its
        range from empty heaps, every shard r >= 1 from k copies of T_r while
        recording its insertions; one all-gather; wv_heap_merge_records applies
        the records in shard order.  Overflowed records fall
        back to the serial chain."""
        ql = torch.nonzero(of).flatten()  # (host sync: the list length; ascending on every rank)
        F = int(ql.numel())
        if F == 0:
            return oi, od, on
        ql32 = ql.to(torch.int32)
        cap = max(256, 16 * k)
        if self.rank == 0:
            ti, td, tn = self.b.replay(q, ql32, None, k, False)
            ri = torch.zeros((F, cap), dtype=torch.int64, device=self.dev)
            rd = torch.zeros((F, cap), dtype=torch.float32, device=self.dev)
            ri[:, :k], rd[:, :k] = ti, td
            rn = tn
        else:
            T = prefix_bound(self.rank, ql, k, gd, gc, gf, self._bounds)
            ri, rd, rn = self.b.replay_record(q, ql32, fake_heaps(T, k), k, cap)
        pk = torch.cat([ri.contiguous().view(torch.int32).reshape(F, 2 * cap), rd.contiguous().view(torch.int32),
                        rn[:, None]], 1)
        G = self._all_gather(pk)  # [W, F, 3 cap + 1]
        rec = (G[..., : 2 * cap].contiguous().view(torch.int64), G[..., 2 * cap: 3 * cap].contiguous().view(torch.float32),
               G[..., 3 * cap].contiguous())
        st = (rec[0][0, :, :k].contiguous(), rec[1][0, :, :k].contiguous(), rec[2][0].contiguous())
        fi, fd, fn, un = self.b.merge_records(self.world, k, cap, st, rec)
        oi[ql], od[ql], on[ql] = fi, fd, fn
        if bool(un.any()):  # a record overflowed: those queries replay serially
            oi, od, on = self._replay_chain(q, k, ql32[un.bool()], oi, od, on)
        return oi, od, on

    @staticmethod
    def _pack_state(ti, td, tn):
        nq, k = ti.shape
        return torch.cat([ti.contiguous().view(torch.int32).reshape(nq, 2 * k), td.contiguous().view(torch.int32),
                          tn[:, None]], 1)

    @staticmethod
    def _unpack_state(p, k):
        return (p[:, : 2 * k].contiguous().view(torch.int64), p[:, 2 * k: 3 * k].contiguous().view(torch.float32),
                p[:, 3 * k].contiguous())

    def _replay_chain_flags(self, q, k, of, oi, od, on):
        """Exact heap replay of the flagged queries across the ranks in id order
        (rank 0 first), states indexed by query, one packed broadcast per hop;
        the last rank extracts into the merged results."""
        nq = of.shape[0]
        state = None
        for r in range(self.world):
            last = r == self.world - 1
            if self.rank == r:
                res = self.b.replay_flags(q, of, state, k, last, out=(oi, od, on) if last else None)
                buf = self._pack_state(*res)
            else:
                buf = torch.empty((nq, 3 * k + 1), dtype=torch.int32, device=self.dev)
            if self.world > 1:
                dist.broadcast(buf, src=r)
            state = self._unpack_state(buf, k)
        return state

    def _replay_chain(self, q, k, qlist, oi, od, on):
        """Exact heap replay across ranks in id order (rank 0 first); heap
        states move rank to rank as device tensors over the collective."""
        nl = int(qlist.numel())
        state = None
        for r in range(self.world):
            extract = r == self.world - 1
            if self.rank == r:
                ti, td, tn = self.b.replay(q, qlist, state, k, extract)
            else:
                ti = torch.empty((nl, k), dtype=torch.int64, device=self.dev)
                td = torch.empty((nl, k), dtype=torch.float32, device=self.dev)
                tn = torch.empty(nl, dtype=torch.int32, device=self.dev)
            dist.broadcast(ti, src=r)
            dist.broadcast(td, src=r)
            dist.broadcast(tn, src=r)
            state = (ti, td, tn)
        fi, fd, fn = state
        rows = qlist.to(torch.int64)
        oi[rows] = fi
        od[rows] = fd
        on[rows] = fn
        return oi, od, on
