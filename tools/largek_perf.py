"""block-key route time vs k (device time from the index's own events)"""
import sys, json, time, numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import weaviate_amd as wv
from weaviate_amd import _lib
import torch
lib = _lib.load()
n, d, B = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
def gen(seed, rows):
    t = torch.empty(rows, d, dtype=torch.float32, device="cuda")
    _lib.check(lib.wv_gen_device(0, 0, seed, 0, rows, d, t.data_ptr(), None))
    torch.cuda.synchronize()
    return t.cpu().numpy()
idx = wv.FlatIndex(distance="cosine", variant="avx256")
data = gen(1, n)
for s0 in range(0, n, 1 << 20):
    e = min(n, s0 + (1 << 20))
    idx.add_batch(np.arange(s0, e, dtype=np.uint64), data[s0:e])
q = gen(2, B)
idx.set_option("timing", 1)
for kv in sys.argv[5:]:
    key, val = kv.split("=")
    idx.set_option(key, int(val))
out = {}
for k in [int(x) for x in sys.argv[4].split(",")]:
    idx.search_by_vector_batch(q, k)
    r0 = idx.stats()["replayed_queries"]
    t = time.perf_counter()
    idx.search_by_vector_batch(q, k)
    wall = time.perf_counter() - t
    st = idx.stats()
    out[k] = dict(gpu_ms=round(st["last_total_ms"], 2), key_ms=round(st["last_select_ms"], 2), wall_ms=round(wall * 1e3, 1),
                  replayed=st["replayed_queries"] - r0, route=_lib.ROUTES[st["last_route"]])
    print(k, out[k], flush=True)
print(json.dumps({"n": n, "d": d, "B": B, "res": out}))
