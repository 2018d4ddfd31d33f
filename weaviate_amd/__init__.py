"""weaviate_amd -- MI355X-native (gfx950) engine for Weaviate's flat vector
index and distancer hot path.  See DESIGN.md and include/wv_knn.h."""
from ._lib import WeaviateError, load  # noqa: F401
from .flat import (AllowList, FlatIndex, bq_encode_batch, hamming_bitwise_batch,  # noqa: F401
                   normalize_batch, single_dist_batch, lsm_segment_header, lsm_segment_scan)
from .dynamic import DynamicIndex  # noqa: F401

__all__ = ["FlatIndex", "DynamicIndex", "AllowList", "WeaviateError", "single_dist_batch", "hamming_bitwise_batch",
           "bq_encode_batch", "normalize_batch", "load", "lsm_segment_header",
           "lsm_segment_scan"]
