import sys, numpy as np
sys.path.insert(0, "/root/repo")
import weaviate_amd as wv
wv.load()
import torch
k = 10
for (n, d) in [(200000, 128), (200000, 768)]:
    g = torch.Generator().manual_seed(1)
    data = torch.randn(n, d, generator=g).numpy()
    nq = 64
    queries = data[np.random.default_rng(2).integers(0, n, nq)] + 0.1 * np.random.default_rng(3).standard_normal((nq, d)).astype(np.float32)
    idx = wv.FlatIndex(distance="cosine", variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    for opt in [None, ("exact_cap", 0), ("q8_bm", 0), ("exact_filter", 0), ("sel_filter", 0), ("q8", 0)]:
        if opt: idx.set_option(*opt)
        r0 = idx.stats()["replayed_queries"]
        idx.search_by_vector_batch(queries, k)
        r1 = idx.stats()["replayed_queries"]
        idx.search_by_vector_batch_multi_allow(queries, k, [None] * nq)
        r2 = idx.stats()
        print(n, d, opt, "plain", r1 - r0, "multi", r2["replayed_queries"] - r1, "route", r2["last_route"], flush=True)
    idx.close()
