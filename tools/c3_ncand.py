"""Diagnostic (C3 shape: 10M x 768 cosine, k=10, B=8192): how many 32-row
blocks the block-key filter lists per query (key <= M + 2 eps, M = the
(k+1)-th smallest key), from wv_index_debug_blockkeys on sampled queries.
That count sets k_blk_exact's row-bound work (24 KiB of int8 plane per block).
Usage: c3_ncand.py [n_queries_sampled]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import weaviate_amd as wv  # noqa: E402
from weaviate_amd import _lib  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
n, d, B, k = 10_000_000, 768, 8192, 10
idx = wv.FlatIndex(distance="cosine", dims=d, variant="avx256")
idx.reserve(n)
stage = torch.empty((1_000_000, d), dtype=torch.float32, device=dev)
for r0 in range(0, n, 1_000_000):
    _lib.check(lib.wv_gen_device(0, 0, 1, r0, 1_000_000, d, stage.data_ptr(), None))
    _lib.check(lib.wv_index_add_range_device(idx._h, r0, stage.data_ptr(), 1_000_000, d))
del stage
q = torch.empty((B, d), dtype=torch.float32, device=dev)
_lib.check(lib.wv_gen_device(0, 0, 2, 0, B, d, q.data_ptr(), None))
oi = torch.empty((B, k), dtype=torch.int64, device=dev)
od = torch.empty((B, k), dtype=torch.float32, device=dev)
on = torch.empty(B, dtype=torch.int32, device=dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
_lib.check(lib.wv_index_search_device(idx._h, q.data_ptr(), B, d, k, 0, oi.data_ptr(), od.data_ptr(),
                                      on.data_ptr(), None, torch.cuda.current_stream(dev).cuda_stream))
torch.cuda.synchronize()
print(f"batch {1e3 * (time.perf_counter() - t0):.1f} ms, route {idx.stats()['last_route']}", flush=True)
ns = int(sys.argv[1]) if len(sys.argv) > 1 else 32
ncs, gaps = [], []
for qi in np.linspace(0, B - 1, ns).astype(int):
    A, eps = idx.debug_blockkeys(int(qi))
    s = np.sort(A[np.isfinite(A)])
    M = s[k]
    nc = int(np.count_nonzero(A <= M + 2 * eps))
    ncs.append(nc)
    gaps.append((float(M - s[0]), eps))
    print(f"q{qi:5d} eps {eps:.3e} M-min {M - s[0]:.3e} nc {nc}", flush=True)
ncs = np.array(ncs)
print(f"nc: mean {ncs.mean():.1f} median {np.median(ncs):.0f} p90 {np.percentile(ncs, 90):.0f} max {ncs.max()}")
print(f"int8 plane bytes per batch at the mean: {ncs.mean() * B * 32 * 768 / 1e9:.2f} GB")
