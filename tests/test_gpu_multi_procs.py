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
data = orc.gen_matrix(kind, 43, 0, n, d)
queries = orc.gen_matrix(kind, 44, 0, 300, d)
per = (n + world - 1) // world
m = MultiFlatIndex(distance=metric, dims=d, devices=[0], world=world, rank0=rank, id_stride=per, transport="host",
                   variant="avx256")
lo, hi = rank * per, min(n, (rank + 1) * per)
m.add_batch(np.arange(lo, hi, dtype=np.uint64), data[lo:hi])
if cap:
    m.set_option("rec_cap", cap)
ids, dd, cnt = m.search_by_vector_batch(queries, k)
st = m.stats()
single = wv.FlatIndex(distance=metric, variant="avx256")
single.add_batch(np.arange(n, dtype=np.uint64), data)
si, sd, sn = single.search_by_vector_batch(queries, k)
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


@pytest.mark.parametrize("world,metric,kind,n,d,k,cap", [(2, "cosine", 0, 12000, 768, 10, 0),
                                                        (2, "l2-squared", 1, 6000, 64, 10, 0),   # ties: parallel replay
                                                        (3, "l2-squared", 1, 6000, 64, 10, 10),  # record overflow: chain
                                                        (2, "l2-squared", 1, 20000, 32, 100, 0)])  # k >= 64: flag chain
def test_multi_across_processes_equals_single(world, metric, kind, n, d, k, cap):
    import json
    port = str(free_port())
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), PORT=port, REPO=REPO)
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER, metric, str(kind), str(n), str(d), str(k), str(cap)],
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
    if kind == 1:
        assert outs[0]["flagged"] > 0
    if cap:
        assert outs[0]["overflowed"] > 0 and outs[0]["chain_hops"] > 0
    assert len({(o["flagged"], o["overflowed"]) for o in outs}) == 1  # every process took the same decisions
