"""CPU simulation of C2's exact heap replay (1M x 128 U{0..127} rows, l2-squared,
k = 100): per query the reference heap's insertions (insertToHeap over id
order) and the 32-row blocks the block-key replay visits (heap short or
top > block min - eps, eps ~ 113 for this data).  Test infrastructure: uses
the oracle's generator; prints the means over a few queries."""
import heapq
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402

n, d, k, eps, nq = 1_000_000, 128, 100, 113.0, 24
X = oracle.gen_matrix(1, 1, 0, n, d).astype(np.float64)
Q = oracle.gen_matrix(1, 2, 0, nq, d).astype(np.float64)
xn = (X * X).sum(1)
ins_all, vis_all = [], []
for qi in range(nq):
    q = Q[qi]
    D = xn - 2 * X @ q + q @ q
    Bm = D.reshape(-1, 32).min(1)
    h, ins, vis = [], 0, 0
    for b in range(len(Bm)):
        if len(h) == k and not (-h[0] > Bm[b] - eps):
            continue
        vis += 1
        for dist in D[b * 32:(b + 1) * 32]:
            if len(h) < k:
                heapq.heappush(h, -dist)
                ins += 1
            elif -h[0] > dist:
                heapq.heapreplace(h, -dist)
                ins += 1
    ins_all.append(ins)
    vis_all.append(vis)
print(f"insertions per query {np.mean(ins_all):.1f}, visited blocks per query {np.mean(vis_all):.1f}")
