import sys, numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/oracle")
import weaviate_amd as wv, oracle
wv.load(); oracle.lib()
sys.path.insert(0, "/root/repo/tests")
from test_gpu_multi_allow import _allow_lists
n, d, k, nq = 20000, 128, 10, 54
data = oracle.gen_matrix(0, 71, 0, n, d)
queries = oracle.gen_matrix(0, 72, 0, nq, d)
idx = wv.FlatIndex(distance="cosine", variant="avx256")
idx.add_batch(np.arange(n, dtype=np.uint64), data)
deleted = list(range(5, n, 97))
idx.delete(*deleted)
allows = _allow_lists(wv, n, nq, k, seed=n + d)
for opt in [None, ("replay_par", 0), ("exact_bm", 0), ("exact_cap", 0)]:
    if opt: idx.set_option(*opt)
    s0 = idx.stats()
    ids, dists, counts = idx.search_by_vector_batch_multi_allow(queries, k, allows)
    s1 = idx.stats()
    bad = []
    for i in range(nq):
        ei, ed, ec = idx.search_by_vector_batch(queries[i:i + 1], k, allow=allows[i])
        if counts[i] != ec[0] or not np.array_equal(ids[i, :counts[i]], ei[0, :ec[0]]):
            al = set() if allows[i] is None else set(int(x) for x in allows[i].ids)
            notin = [int(x) for x in ids[i, :counts[i]] if allows[i] is not None and int(x) not in al]
            bad.append((i, i % 9, int(counts[i]), int(ec[0]), len(notin)))
    print(opt, "replayed", s1["replayed_queries"] - s0["replayed_queries"], "route", s1["last_route"], "bad", bad, flush=True)
