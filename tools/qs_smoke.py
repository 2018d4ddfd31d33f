"""Quick GPU check of the block-key path (kernel 7) against the oracle on a
few small shapes; prints per-shape status.  Test infrastructure."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as orc  # noqa: E402
import weaviate_amd as wv  # noqa: E402

shapes = [("cosine", 0, 3000, 768, 10, 40), ("l2-squared", 0, 5000, 128, 10, 40), ("dot", 0, 2000, 96, 7, 30),
          ("l2-squared", 1, 4000, 128, 100, 20), ("cosine", 0, 2500, 40, 24, 20)]
bad = 0
for metric, kind, n, d, k, nq in shapes:
    data = orc.gen_matrix(kind, 11, 0, n, d)
    queries = orc.gen_matrix(kind, 12, 0, nq, d)
    idx = wv.FlatIndex(distance=metric, variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    t0 = time.time()
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    dt = time.time() - t0
    ref = orc.OracleFlat(orc.METRIC[metric], orc.AVX256, d, n)
    ref.add_batch(np.arange(n), data)
    nbad = 0
    for q in range(nq):
        rc, oi, od = ref.search(queries[q], k)
        c = counts[q]
        if not (c == len(oi) and np.array_equal(ids[q, :c], oi) and
                np.array_equal(dists[q, :c].view(np.uint32), od.view(np.uint32))):
            nbad += 1
            if nbad <= 2:
                print("  mismatch q", q, "count", c, len(oi), "ids", ids[q, :min(c, 6)], oi[:6], "d", dists[q, :3], od[:3])
    st = idx.stats()
    print(f"{metric} kind={kind} n={n} d={d} k={k} nq={nq}: bad={nbad} replayed={st['replayed_queries']} {dt*1e3:.1f} ms",
          flush=True)
    bad += nbad
    idx.close()
print("QS SMOKE", "OK" if bad == 0 else f"FAIL {bad}")
sys.exit(1 if bad else 0)
