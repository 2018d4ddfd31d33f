"""GPU: the multi-shard index across PROCESSES (one shard per process, as
the bench's N-GPU run places them), here two processes sharing the box's one
GPU: the library's protocol driver with the host transport (collectives
staged through host memory over a gloo process group; RCCL refuses two ranks
on one device).  Every process must return the single index's results bit for
bit -- the decisions each process takes on its own (flagged list, record
overflow, chain hops) must agree for the collectives to match."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys, json
import numpy as np
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.path.join(os.environ["REPO"], "oracle"))
import torch, torch.distributed as dist
import oracle as orc
import weaviate_amd as wv
from weaviate_amd.multi import MultiFlatIndex
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:" + os.environ["PORT"], rank=rank, world_size=world)
metric, kind, n, d, k, cap = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
comp, filt = sys.argv[7], int(sys.argv[8])
data = orc.gen_matrix(kind, 43, 0, n, d)
queries = orc.gen_matrix(kind, 44, 0, 300, d)
per = (n + world - 1) // world
kw = {"bq": dict(bq=True, rescore_limit=40), "rq8": dict(rq={"bits": 8}, rescore_limit=30),
      "pq": dict(pq={"segments": d // 4, "centroids": 32, "trainingLimit": per // 2, "rescore": True},
                 rescore_limit=40)}.get(comp, {})
m = MultiFlatIndex(distance=metric, dims=d, devices=[0], world=world, rank0=rank, id_stride=per, transport="host",
                   variant="avx256", **kw)
lo, hi = rank * per, min(n, (rank + 1) * per)
m.add_batch(np.arange(lo, hi, dtype=np.uint64), data[lo:hi])
single = wv.FlatIndex(distance=metric, variant="avx256", **kw)
single.add_batch(np.arange(n, dtype=np.uint64), data)
if comp == "pq":  # rank 0 holds the first trainingLimit rows: it trains, the codebook goes to every process
    m.pq_fit(seed=7)
    single.pq_fit(seed=7)
if cap:
    m.set_option("rec_cap" if comp == "none" else "chain", cap)
allow = wv.AllowList(np.random.default_rng(3).choice(n, n // 7, replace=False).tolist()) if filt else None
ids, dd, cnt = m.search_by_vector_batch(queries, k, allow=allow)
st = m.stats()
si, sd, sn = single.search_by_vector_batch(queries, k, allow=allow)
ok = bool(np.array_equal(cnt, sn))
bad = []
for i in range(len(cnt)):
    same = bool(np.array_equal(ids[i, :cnt[i]], si[i, :sn[i]]) and
                np.array_equal(dd[i, :cnt[i]].view(np.uint32), sd[i, :sn[i]].view(np.uint32)))
    ok &= same
    if not same and len(bad) < 3:
        bad.append({"q": i, "got": ids[i, :cnt[i]].tolist(), "exp": si[i, :sn[i]].tolist(),
                    "gd": dd[i, :cnt[i]].tolist(), "ed": sd[i, :sn[i]].tolist()})
print(json.dumps({"rank": rank, "equal": ok, "flagged": st["last_flagged"], "overflowed": st["last_overflowed"],
                  "chain_hops": st["chain_hops"], "bad": bad}), flush=True)
m.close(); single.close()
dist.destroy_process_group()
'''


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,metric,kind,n,d,k,cap,comp,filt", [
    (2, "cosine", 0, 12000, 768, 10, 0, "none", 0),
    (2, "l2-squared", 1, 6000, 64, 10, 0, "none", 0),    # ties: parallel replay
    (3, "l2-squared", 1, 6000, 64, 10, 10, "none", 0),   # record overflow: chain
    (2, "l2-squared", 1, 20000, 32, 100, 0, "none", 0),  # k >= 64: flag chain
    (2, "l2-squared", 1, 9000, 64, 10, 0, "none", 1),    # allow list: each process its part
    (2, "cosine", 0, 104000, 1536, 10, 0, "bq", 0),      # BQ R-heap, parallel hop
    (3, "cosine", 0, 12000, 1536, 10, 1, "bq", 1),       # BQ serial chain + allow list
    (2, "cosine", 0, 8000, 64, 10, 0, "rq8", 0),         # rq-8 worker heap
    (2, "l2-squared", 0, 8000, 32, 10, 0, "pq", 0)])     # PQ: trained on rank 0, codebook broadcast
def test_multi_across_processes_equals_single(world, metric, kind, n, d, k, cap, comp, filt):
    import json
    port = str(free_port())
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), PORT=port, REPO=REPO)
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER, metric, str(kind), str(n), str(d), str(k), str(cap),
                                       comp, str(filt)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e[-2000:]
        outs.append(json.loads([ln for ln in o.splitlines() if ln.startswith("{")][-1]))
    assert all(o["equal"] for o in outs), outs
    if kind == 1 and comp == "none":
        assert outs[0]["flagged"] > 0
    if cap:
        assert outs[0]["chain_hops"] > 0 and (comp != "none" or outs[0]["overflowed"] > 0)
    assert len({(o["flagged"], o["overflowed"]) for o in outs}) == 1  # every process took the same decisions
