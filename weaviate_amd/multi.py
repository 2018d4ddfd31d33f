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
from .flat import FlatIndex, make_config

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
        self.bq = self.pq = self.rq = self.sq = False
        self.rescore_limit = -1
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
                 variant: str = "auto", host_callbacks=None):
        """transport "host": host_callbacks = (allgather, broadcast) ctypes
        callbacks (torch_host_callbacks(world) by default)."""
        self._l = _lib.load()
        devs = [int(x) for x in devices]
        world = int(world) or len(devs)
        self._devs = (C.c_int32 * len(devs))(*devs)
        self._uid = C.create_string_buffer(unique_id, 128) if unique_id is not None else None
        self._cbs = None
        if transport == "host":
            self._cbs = host_callbacks or torch_host_callbacks(world)
        cfg_args = dict(distance=distance, dims=dims, variant=variant)
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

    def search_by_vector_batch(self, queries: np.ndarray, k: int):
        """SearchByVector over every rank -> (ids [nq, k] uint64, dists [nq, k]
        float32, counts [nq])."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        nq, d = q.shape
        ids = np.zeros((nq, k), dtype=np.uint64)
        dd = np.zeros((nq, k), dtype=np.float32)
        cnt = np.zeros(nq, dtype=np.int32)
        check(self._l.wv_multi_search_by_vector_batch(self._h, q.ctypes.data_as(C.POINTER(C.c_float)), nq, d, int(k),
                                                      ids.ctypes.data_as(C.POINTER(C.c_uint64)),
                                                      dd.ctypes.data_as(C.POINTER(C.c_float)),
                                                      cnt.ctypes.data_as(C.POINTER(C.c_int32))))
        return ids, dd, cnt

    def search_device(self, q_ptr: int, nq: int, d: int, k: int, ids_ptr: int, dists_ptr: int, counts_ptr: int,
                      stream: Optional[int] = None) -> None:
        """Device buffers on local shard 0's GPU, ordered on `stream`."""
        check(self._l.wv_multi_search_device(self._h, q_ptr, nq, d, int(k), ids_ptr, dists_ptr, counts_ptr, stream))

    def stats(self) -> dict:
        out = (C.c_int64 * 10)()
        check(self._l.wv_multi_stats(self._h, out, 10))
        keys = ("searches", "flagged", "overflowed", "chain_hops", "last_flagged", "last_overflowed", "world",
                "rank0", "n_local", "transport")
        return dict(zip(keys, [int(x) for x in out]))

    def stage_ms(self) -> dict:
        """Option sim: the last search's per-shard stage times (ms)."""
        n = len(self.devices)
        out = (C.c_double * (len(STAGES) * n))()
        check(self._l.wv_multi_stage_ms(self._h, out, n))
        return {s: [float(out[i * n + j]) for j in range(n)] for i, s in enumerate(STAGES)}
