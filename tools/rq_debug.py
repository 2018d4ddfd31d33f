"""rq MFMA route debugging: block minima of k_rq8_keys (debug_blockkeys)
against the minima of the distance-matrix kernel's rows (rq_distances), over
repeated runs and with option rq_serial."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle as orc  # noqa: E402
import weaviate_amd as wv  # noqa: E402

nq = 24
for bits, metric, n, d in ((8, "cosine", 5000, 768), (1, "cosine", 5000, 768), (1, "l2-squared", 3000, 128)):
    data = orc.gen_matrix(0, 11, 0, n, d)
    qs = orc.gen_matrix(0, 12, 0, nq, d)
    idx = wv.FlatIndex(distance=metric, rq={"bits": bits}, rescore_limit=-1, variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    E = idx.rq_distances(qs, n)
    for serial in (0, 1, 0, 1):
        idx.set_option("rq_serial", serial)
        idx.search_by_vector_batch(qs, 10)
        tot = 0
        for q in range(nq):
            A, eps = idx.debug_blockkeys(q)
            nb = len(A)
            e = np.full(nb * 32, np.inf, np.float32)
            e[:n] = E[q]
            ref = e.reshape(nb, 32).min(axis=1)
            bad = np.nonzero(A.view(np.uint32) != ref.view(np.uint32))[0]
            tot += len(bad)
            if q == 0 and len(bad):
                b = bad[0]
                print("   q0 block", b, "key", A[b], "ref", ref[b], "rows", e.reshape(nb, 32)[b][:8])
        print(bits, metric, "serial", serial, "mismatched blocks over", nq, "queries:", tot)
    idx.close()
