"""The corpus sharded over GPUs, searched from one process (wv_multi, include/wv_knn.h).

Weaviate searches every shard of a node inside one Go process and merges the
shard results there (adapters/repos/db/index.go:1928-2071).  MultiFlatIndex is
that caller's view of the C library's multi-shard index: the library holds one
flat index per rank (contiguous doc-id ranges of ``id_stride`` ids), drives
the two-phase protocol and owns the collectives -- an RCCL
communicator per local shard (``transport="rccl"``), or device copies between
shards of this process (``transport="local"``, several shards may share a GPU).
A multi-process world (one process per GPU, e.g. under torch.distributed.run)
passes rank 0's ``rccl_unique_id()`` to every process.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check
from .flat import AllowList, FlatIndex, _allow_args, _fptr, _iptr, _uptr, make_config

TRANSPORTS = {"local": 0, "rccl": 1, "host": 2}
STAGES = ("phase1", "phase2", "merge", "replay", "merge_records", "chain", "collectives")


def rccl_unique_id() -> bytes:
    """ncclGetUniqueId of rank 0 (128 bytes), to hand to every process of the world."""
    buf = C.create_string_buffer(128)
    check(_lib.load().wv_rccl_unique_id(buf, 128))
    return buf.raw


def torch_host_callbacks(world: int, group=None):
    """WV_TRANSPORT_HOST callbacks over torch.distributed (e.g. a gloo group):
    the library hands host buffers, the collective runs on CPU tensors."""
    import torch
    import torch.distributed as dist

    def view(p, n):
        return torch.frombuffer((C.c_uint8 * n).from_address(p), dtype=torch.uint8)

    def allgather(send_p, recv_p, nbytes, user):
        try:
            if nbytes > 0:
                parts = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(world)]
                dist.all_gather(parts, view(send_p, nbytes).clone(), group=group)
                out = torch.cat(parts)  # alive across the copy
                C.memmove(recv_p, out.data_ptr(), world * nbytes)
            return 0
        except Exception:
            return 1

    def broadcast(buf_p, nbytes, root, user):
        try:
            if nbytes > 0:
                t = view(buf_p, nbytes).clone()
                dist.broadcast(t, src=int(root), group=group)
                C.memmove(buf_p, t.data_ptr(), nbytes)
            return 0
        except Exception:
            return 1

    return _lib.HOST_ALLGATHER_FN(allgather), _lib.HOST_BROADCAST_FN(broadcast)


class _ShardView(FlatIndex):
    """A local shard of a MultiFlatIndex: the FlatIndex surface on an index the
    multi-shard index owns (close() does not free it)."""

    def __init__(self, h, owner: "MultiFlatIndex", device: int, id_base: int, cfg_args: dict):
        self._l = _lib.load()
        self._h = h
        self._owner = owner  # keeps the multi-shard index alive
        self._root = cfg_args.get("root_path", b"")
        self._cfg_args = dict(cfg_args, device=device, id_base=id_base)
        self.metric = owner.metric
        self.bq = bool(cfg_args.get("bq"))
        self.pq = cfg_args.get("pq") is not None
        self.rq = cfg_args.get("rq") is not None
        self.sq = bool(cfg_args.get("sq"))
        self.rescore_limit = int(cfg_args.get("rescore_limit", -1))
        self.device = device
        self.id_base = id_base

    def close(self) -> None:
        self._h = None


class MultiFlatIndex:
    """Ranks [rank0, rank0 + len(devices)) of a world of `world` ranks, rank r
    holding doc ids [r * id_stride, (r + 1) * id_stride) (the last rank: every id
    above)."""

    def __init__(self, distance: str = "cosine", dims: int = 0, devices: Sequence[int] = (0,), world: int = 0,
                 rank0: int = 0, id_stride: int = 0, transport: str = "local", unique_id: Optional[bytes] = None,
                 variant: str = "auto", host_callbacks=None, bq: bool = False, rescore_limit: int = -1,
                 pq: Optional[dict] = None, rq: Optional[dict] = None, sq: bool = False):
        """transport "host": host_callbacks = (allgather, broadcast) ctypes
        callbacks (torch_host_callbacks(world) by default).  bq / rescore_limit
        / pq / rq / sq: every shard's compression, as FlatIndex takes them."""
        self._l = _lib.load()
        devs = [int(x) for x in devices]
        world = int(world) or len(devs)
        self._devs = (C.c_int32 * len(devs))(*devs)
        self._uid = C.create_string_buffer(unique_id, 128) if unique_id is not None else None
        self._cbs = None
        if transport == "host":
            self._cbs = host_callbacks or torch_host_callbacks(world)
        cfg_args = dict(distance=distance, dims=dims, variant=variant, bq=bq, rescore_limit=rescore_limit, pq=pq, rq=rq,
                        sq=sq)
        self._cfg = _lib.WvMultiConfig(make_config(**cfg_args), world, int(rank0), len(devs),
                                       C.cast(self._devs, C.POINTER(C.c_int32)), int(id_stride),
                                       TRANSPORTS[transport], C.cast(self._uid, C.c_void_p) if self._uid else None,
                                       C.cast(self._cbs[0], C.c_void_p) if self._cbs else None,
                                       C.cast(self._cbs[1], C.c_void_p) if self._cbs else None, None)
        h = C.c_void_p()
        check(self._l.wv_multi_create(C.byref(self._cfg), C.byref(h)))
        self._h = h
        self.metric = make_config(**cfg_args).metric
        self.world, self.rank0, self.id_stride = world, int(rank0), int(id_stride)
        self.devices = devs
        self.shards = [_ShardView(self._l.wv_multi_shard(h, i), self, devs[i], (int(rank0) + i) * int(id_stride),
                                  cfg_args) for i in range(len(devs))]

    def close(self) -> None:
        if getattr(self, "_h", None):
            for s in self.shards:
                s.close()
            self._l.wv_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_option(self, key: str, value: int) -> None:
        check(self._l.wv_multi_set_option(self._h, key.encode(), int(value)))

    def add_batch(self, ids: np.ndarray, vectors: np.ndarray) -> None:
        """flat.AddBatch, each row to the shard owning its id."""
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        v = np.ascontiguousarray(vectors, dtype=np.float32)
        if v.ndim != 2 or v.shape[0] != ids.size:
            raise _lib.WeaviateError(_lib.WV_ERR_INSERT, "ids and vectors sizes does not match")
        check(self._l.wv_multi_add_batch(self._h, ids.ctypes.data_as(C.POINTER(C.c_uint64)),
                                         v.ctypes.data_as(C.POINTER(C.c_float)), ids.size, v.shape[1]))

    def search_by_vector_batch(self, queries: np.ndarray, k: int, allow: Optional[AllowList] = None):
        """SearchByVector over every rank (under `allow`, each shard its part of
        the list) -> (ids [nq, k] uint64, dists [nq, k] float32, counts [nq])."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        nq, d = q.shape
        ids = np.zeros((nq, k), dtype=np.uint64)
        dd = np.zeros((nq, k), dtype=np.float32)
        cnt = np.zeros(nq, dtype=np.int32)
        ap, na, mode, _keep = _allow_args(allow)
        check(self._l.wv_multi_search_by_vector_batch_allow(self._h, _fptr(q), nq, d, int(k), ap, na, mode, _uptr(ids),
                                                            _fptr(dd), _iptr(cnt)))
        return ids, dd, cnt

    def search_by_vector_batch_multi_allow(self, queries: np.ndarray, k: int, allows):
        """Row i under its own allow list allows[i] (None = unfiltered)."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        nq, d = q.shape
        allows = list(allows)
        if len(allows) != nq:
            raise _lib.WeaviateError(_lib.WV_ERR_INVALID, f"{len(allows)} allow lists for {nq} queries")
        ids = np.zeros((nq, k), dtype=np.uint64)
        dd = np.zeros((nq, k), dtype=np.float32)
        cnt = np.zeros(nq, dtype=np.int32)
        modes = np.array([0 if a is None else 1 for a in allows], dtype=np.int32)
        parts = [np.asarray(a.ids, dtype=np.uint64) for a in allows if a is not None]
        aids = np.ascontiguousarray(np.concatenate(parts) if parts else np.zeros(1, np.uint64), dtype=np.uint64)
        off = np.zeros(nq + 1, dtype=np.int64)
        off[1:] = np.cumsum([0 if a is None else a.ids.size for a in allows])
        check(self._l.wv_multi_search_by_vector_batch_multi_allow(
            self._h, _fptr(q), nq, d, int(k), _uptr(aids), off.ctypes.data_as(C.c_void_p), _iptr(modes), _uptr(ids),
            _fptr(dd), _iptr(cnt)))
        return ids, dd, cnt

    def search_by_vector_distance(self, vector, target_distance: float, max_limit: int,
                                  allow: Optional[AllowList] = None):
        """SearchByVectorDistance over every rank (flat/index.go:699-761)."""
        v = np.ascontiguousarray(vector, dtype=np.float32).ravel()
        ids = np.zeros(100, dtype=np.uint64)
        dists = np.zeros(100, dtype=np.float32)
        n = np.zeros(1, dtype=np.int32)
        ap, na, mode, _keep = _allow_args(allow)
        check(self._l.wv_multi_search_by_vector_distance(self._h, _fptr(v), v.size, float(target_distance),
                                                         int(max_limit), ap, na, mode, _uptr(ids), _fptr(dists),
                                                         _iptr(n)))
        return ids[: n[0]].copy(), dists[: n[0]].copy()

    def pq_fit(self, seed: int = 0) -> None:
        """ProductQuantizer.Fit over the shards' first trainingLimit rows in id
        order; the codebook installed on every shard."""
        check(self._l.wv_multi_pq_fit(self._h, int(seed)))

    def pq_set_centers(self, centers: np.ndarray) -> None:
        c = np.ascontiguousarray(centers, dtype=np.float32).ravel()
        check(self._l.wv_multi_pq_set_centers(self._h, _fptr(c), c.size))

    def search_device(self, q_ptr: int, nq: int, d: int, k: int, ids_ptr: int, dists_ptr: int, counts_ptr: int,
                      stream: Optional[int] = None, allow: Optional[AllowList] = None) -> None:
        """Device buffers on local shard 0's GPU, ordered on `stream`."""
        if allow is None:
            check(self._l.wv_multi_search_device(self._h, q_ptr, nq, d, int(k), ids_ptr, dists_ptr, counts_ptr, stream))
            return
        ap, na, mode, _keep = _allow_args(allow)
        check(self._l.wv_multi_search_device_allow(self._h, q_ptr, nq, d, int(k), ap, na, mode, ids_ptr, dists_ptr,
                                                   counts_ptr, stream))

    def stats(self) -> dict:
        out = (C.c_int64 * 12)()
        check(self._l.wv_multi_stats(self._h, out, 12))
        keys = ("searches", "flagged", "overflowed", "chain_hops", "last_flagged", "last_overflowed", "world",
                "rank0", "n_local", "transport", "host_us", "host_wait_us")
        return dict(zip(keys, [int(x) for x in out]))

    def stage_ms(self) -> dict:
        """Option sim: the last search's per-shard stage times (ms)."""
        n = len(self.devices)
        out = (C.c_double * (len(STAGES) * n))()
        check(self._l.wv_multi_stage_ms(self._h, out, n))
        return {s: [float(out[i * n + j]) for j in range(n)] for i, s in enumerate(STAGES)}
