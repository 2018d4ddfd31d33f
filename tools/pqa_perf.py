"""per-query allow lists: one shared launch vs one call per list (host-inclusive)"""
import sys, time, json, numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import weaviate_amd as wv
wv.load()
import torch
n, d, k = int(sys.argv[1]), int(sys.argv[2]), 10
nq = int(sys.argv[3])
from weaviate_amd import _lib
lib = _lib.load()
def gen(seed, rows):
    t = torch.empty(rows, d, dtype=torch.float32, device="cuda")
    _lib.check(lib.wv_gen_device(0, 0, seed, 0, rows, d, t.data_ptr(), None))
    torch.cuda.synchronize()
    return t.cpu().numpy()
data = gen(1, n)
queries = gen(2, nq)
idx = wv.FlatIndex(distance="cosine", variant="avx256")
for s in range(0, n, 1 << 20):
    e = min(n, s + (1 << 20))
    idx.add_batch(np.arange(s, e, dtype=np.uint64), data[s:e])
rng = np.random.default_rng(4)
idx.set_option("timing", 1)
res = {}
if len(sys.argv) > 4:
    idx.set_option("q8", int(sys.argv[4]))
dlist = [float(x) for x in sys.argv[5].split(",")] if len(sys.argv) > 5 else [1.0, 0.5, 0.1, 0.01]
ncalls = 0 if len(sys.argv) > 6 else 64
for dens in dlist:
    allows = [None if dens == 1.0 else wv.AllowList(np.flatnonzero(rng.random(n) < dens)) for _ in range(nq)]
    idx.search_by_vector_batch_multi_allow(queries, k, allows)
    s0 = idx.stats()
    t = time.perf_counter()
    idx.search_by_vector_batch_multi_allow(queries, k, allows)
    t_multi = time.perf_counter() - t
    s1 = idx.stats()
    t = time.perf_counter()
    for i in range(min(nq, ncalls)):
        idx.search_by_vector_batch(queries[i:i + 1], k, allow=allows[i])
    t_one = (time.perf_counter() - t) / max(1, min(nq, ncalls)) * nq
    res[dens] = dict(multi_ms=round(t_multi * 1e3, 2), gpu_ms=round(s1["last_total_ms"], 2), per_query_calls_ms=round(t_one * 1e3, 2),
                     replayed=s1["replayed_queries"] - s0["replayed_queries"])
    print(dens, res[dens], flush=True)
print(json.dumps({"n": n, "d": d, "nq": nq, "k": k, "res": res}))
