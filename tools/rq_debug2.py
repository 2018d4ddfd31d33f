"""rq-1 MFMA debugging: the +-1 plane against the exported bit codes, and
key stability over repeated searches."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle as orc  # noqa: E402
import weaviate_amd as wv  # noqa: E402

n, d, nq = 5000, 768, 24
data = orc.gen_matrix(0, 11, 0, n, d)
qs = orc.gen_matrix(0, 12, 0, nq, d)
idx = wv.FlatIndex(distance="cosine", rq={"bits": 1}, rescore_limit=-1, variant="avx256")
idx.add_batch(np.arange(n, dtype=np.uint64), data)
codes = idx.rq_codes(n)  # [n][1 + W] u64, word 0 meta
D = idx.rq_info()["output_dim"]
idx.set_option("rq_serial", 16)
pm = np.zeros((n, D), np.int8)
wv._lib.check(idx._l.wv_index_rq_codes(idx._h, pm.ctypes.data, n))
idx.set_option("rq_serial", 0)
bits = np.unpackbits(codes[:, 1:].view(np.uint8), axis=1, bitorder="little")[:, :D].astype(np.int64)
exp = (1 - 2 * bits).astype(np.int8)
badrows = np.nonzero((pm != exp).any(axis=1))[0]
print("plane rows wrong:", len(badrows), badrows[:10])
E = idx.rq_distances(qs, n)
keys = []
for rep, dbg in enumerate((0, 0, 0, 1, 2, 4)):
    idx.set_option("rq_serial", dbg)
    idx.search_by_vector_batch(qs, 10)
    K = np.stack([idx.debug_blockkeys(q)[0] for q in range(nq)])
    keys.append(K)
    nb = K.shape[1]
    e = np.full((nq, nb * 32), np.inf, np.float32)
    e[:, :n] = E
    ref = e.reshape(nq, nb, 32).min(axis=2)
    bad = np.argwhere(K.view(np.uint32) != ref.view(np.uint32))
    print("rep", rep, "dbg", dbg, "mismatched", len(bad), "same as rep0", np.array_equal(K.view(np.uint32), keys[0].view(np.uint32)))
    if len(bad):
        q, b = bad[0]
        print("  q", q, "block", b, "key", K[q, b], "ref", ref[q, b])
        qb = bad[:, 1]
        print("  blocks hist (mod 8):", np.bincount(qb % 8, minlength=8), "by query:", np.bincount(bad[:, 0], minlength=nq)[:24])
idx.close()
