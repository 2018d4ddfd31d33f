"""The dynamic vector index (adapters/repos/db/vector/dynamic/index.go) wired to
this engine.  Below its threshold a dynamic index IS its inner flat index:
New builds flat.New(flatConfig, uc.FlatUC, store) (:210-216) and every
VectorIndex call forwards to it under the read lock (:321-458).  Here the inner
index is the HIP-backed FlatIndex, so a dynamic index gets the GPU flat path
unchanged; a Go maintainer wires it the same way (dynamic.New
creates the cgo-backed flat instead of flat.New).

The upgrade to HNSW (doUpgrade, :511-615) builds a graph index, which is out of
scope of this engine: ShouldUpgrade reports the threshold as the
reference does, Upgrade raises WV_ERR_UNSUPPORTED and leaves the flat index
serving, so the caller (vector_index_queue.go:263-290) logs the error and keeps
the exact results.
"""
from __future__ import annotations

import threading
from typing import Optional

from . import _lib
from ._lib import WeaviateError
from .flat import AllowList, FlatIndex

DEFAULT_THRESHOLD = 10_000  # entities/vectorindex/dynamic/config.go:24


class DynamicIndex:
    """dynamic.New with a not-yet-upgraded state (init, :245-303, read the
    upgraded flag as 0).  flat: the FlatIndex keyword arguments (uc.FlatUC);
    threshold: UserConfig.Threshold."""

    def __init__(self, threshold: int = DEFAULT_THRESHOLD, upgraded: bool = False, **flat):
        if upgraded:  # New(:177-208): an upgraded dynamic index opens HNSW
            raise WeaviateError(_lib.WV_ERR_UNSUPPORTED, "dynamic index upgraded to hnsw: hnsw is not served by "
                                                         "this engine")
        self.threshold = int(threshold)
        self._flat_args = dict(flat)
        self.index = FlatIndex(**flat)
        self._mu = threading.RLock()  # dynamic.RWMutex (write side only matters for Upgrade / Shutdown)
        self._closed = False

    # -- identity (:219-221, :705-716) ----------------------------------------
    def type(self) -> str:
        return "dynamic"

    def underlying_index(self) -> str:
        return self.index.type()

    def is_upgraded(self) -> bool:
        return False

    # -- forwarded VectorIndex surface (:309-458, :671-703) --------------------
    def compressed(self) -> bool:
        return self.index.compressed()

    def multivector(self) -> bool:
        return False

    def add(self, id: int, vector) -> None:
        with self._mu:
            self.index.add(id, vector)

    def add_batch(self, ids, vectors) -> None:
        with self._mu:
            self.index.add_batch(ids, vectors)

    def delete(self, *ids: int) -> None:
        with self._mu:
            self.index.delete(*ids)

    def search_by_vector(self, vector, k: int, allow: Optional[AllowList] = None):
        return self.index.search_by_vector(vector, k, allow)

    def search_by_vector_batch(self, queries, k: int, allow: Optional[AllowList] = None):
        return self.index.search_by_vector_batch(queries, k, allow)

    def search_by_vector_distance(self, vector, target_distance: float, max_limit: int,
                                  allow: Optional[AllowList] = None):
        return self.index.search_by_vector_distance(vector, target_distance, max_limit, allow)

    def validate_before_insert(self, vector) -> None:
        self.index.validate_before_insert(vector)

    def contains_doc(self, id: int) -> bool:
        return self.index.contains_doc(id)

    def preload(self, id: int, vector) -> None:
        self.index.preload(id, vector)

    def already_indexed(self) -> int:
        return self.index.already_indexed()

    def query_vector_distancer(self, query):
        return self.index.query_vector_distancer(query)

    def iterate(self, fn) -> None:
        self.index.iterate(fn)

    def compression_stats(self) -> dict:
        return self.index.compression_stats()

    def update_user_config(self, threshold: Optional[int] = None, **flat_uc) -> None:
        """UpdateUserConfig (:351-368): not upgraded -> keep the new config
        (threshold included) and forward FlatUC to the flat index."""
        with self._mu:
            if threshold is not None:
                self.threshold = int(threshold)
            if flat_uc:
                self.index.update_user_config(**flat_uc)

    def stats(self):  # (:679-688): "index is not hnsw"
        raise WeaviateError(_lib.WV_ERR_INVALID, "index is not hnsw")

    # -- upgradableIndexer (:462-510) ------------------------------------------
    def should_upgrade(self) -> tuple:
        return True, self.threshold

    def upgraded(self) -> bool:
        return False

    def upgrade(self, callback=None) -> None:
        """doUpgrade would build an HNSW graph from the flat vectors; the graph
        index is out of scope, so the flat index keeps serving."""
        try:
            raise WeaviateError(_lib.WV_ERR_UNSUPPORTED, "upgrade to hnsw: hnsw is not served by this engine; "
                                                         "the flat index keeps serving")
        finally:
            if callback is not None:
                callback()

    # -- lifecycle (:370-412) -------------------------------------------------------
    def shutdown(self) -> None:
        with self._mu:
            if not self._closed:
                self._closed = True
                self.index.close()

    close = shutdown

    def drop(self) -> None:
        self.shutdown()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.shutdown()


def should_trigger_upgrade(idx) -> bool:
    """VectorIndexQueue.checkCompressionSettings (vector_index_queue.go:263-290):
    true when the queue would pause and call Upgrade."""
    should, at = idx.should_upgrade()
    if not should or idx.upgraded():
        return False
    return idx.already_indexed() > int(at)
