"""Debug: the sharded replay chain step by step with syncs (3 shards, integer data)."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle
import weaviate_amd as wv
from weaviate_amd.sharded import GpuShardBackend

def log(*a):
    print(time.strftime("%H:%M:%S"), *a, flush=True)

shards, metric, kind, n, d, k = 3, "l2-squared", 1, 6000, 64, 10
dev = torch.device("cuda", 0)
data = oracle.gen_matrix(kind, 41, 0, n, d)
queries = oracle.gen_matrix(kind, 42, 0, 200, d)
per = (n + shards - 1) // shards
backs = []
for r in range(shards):
    lo, hi = r * per, min(n, (r + 1) * per)
    idx = wv.FlatIndex(distance=metric, id_base=lo, variant="avx256")
    idx.add_batch(np.arange(lo, hi, dtype=np.uint64), data[lo:hi])
    backs.append(GpuShardBackend(idx, 0))
q = torch.from_numpy(queries).to(dev)
parts = []
for r, b in enumerate(backs):
    parts.append(b.local_search(q, k))
    torch.cuda.synchronize()
    log("local", r, "flags", int((parts[-1][3] != 0).sum()), "keys_nq", b.index.stats())
gi, gd, gc, gf = (torch.stack([p[j] for p in parts]) for j in range(4))
oi, od, on, of = backs[0].merge(shards, k, gi, gd, gc, gf)
torch.cuda.synchronize()
flagged = torch.nonzero(of).flatten().to(torch.int32)
log("flagged", flagged.numel())
state = None
for r, b in enumerate(backs):
    state = b.replay(q, flagged, state, k, r == shards - 1)
    torch.cuda.synchronize()
    log("replay", r, "len min/max", int(state[2].min()), int(state[2].max()))
log("done")
