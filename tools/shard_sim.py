"""Per-rank cost of the sharded exact search at W ranks, measured on ONE GPU
through the library's multi-shard index (wv_multi, multi.hip): the C3 corpus
(10M x 768 cosine) split into W contiguous id-range shards on the same device,
local transport, option sim (every shard's part of every stage runs alone,
timed with HIP events; the collectives are device copies, timed apart).
Predicted step at W ranks = sum over stages of the max over shards + the
RCCL all-gathers (estimated from their bytes).  Also checks the results
against the single-GPU search of the same batch (bit-exact ids and distances).
Prints one JSON line."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--d", type=int, default=768)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--batch", type=int, default=8192)
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--no-single", action="store_true")
ap.add_argument("--rev", action="store_true", help="time the shards in reverse order (option sim_rev)")
args = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402
import weaviate_amd as wv  # noqa: E402
from weaviate_amd import _lib  # noqa: E402
from weaviate_amd.multi import MultiFlatIndex, STAGES  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
W, n, d, k, B = args.world, args.n, args.d, args.k, args.batch
per = (n + W - 1) // W
m = MultiFlatIndex(distance="cosine", dims=d, devices=[0] * W, id_stride=per, transport="local", variant="avx256")
stage = torch.empty((1_000_000, d), dtype=torch.float32, device=dev)
for r, sh in enumerate(m.shards):
    lo, hi = r * per, min(n, (r + 1) * per)
    sh.reserve(hi - lo)
    for r0 in range(lo, hi, 1_000_000):
        c = min(1_000_000, hi - r0)
        _lib.check(lib.wv_gen_device(0, 0, 1, r0, c, d, stage.data_ptr(), None))
        _lib.check(lib.wv_index_add_range_device(sh._h, r0, stage.data_ptr(), c, d))
del stage
q = torch.empty((B, d), dtype=torch.float32, device=dev)
_lib.check(lib.wv_gen_device(0, 0, 2, 0, B, d, q.data_ptr(), None))
oi = torch.empty((B, k), dtype=torch.int64, device=dev)
od = torch.empty((B, k), dtype=torch.float32, device=dev)
on = torch.empty(B, dtype=torch.int32, device=dev)
torch.cuda.synchronize()
m.set_option("sim_rev", 1 if args.rev else 0)
m.set_option("sim", 1)
m.search_device(q.data_ptr(), B, d, k, oi.data_ptr(), od.data_ptr(), on.data_ptr(), None)  # warm-up
m.set_option("sim", 1)  # restart the averaging: back-to-back searches, as the GPUs of a real run see them
for rep in range(args.reps):
    m.search_device(q.data_ptr(), B, d, k, oi.data_ptr(), od.data_ptr(), on.data_ptr(), None)
rows = [m.stage_ms()]
st = m.stats()
# without sim: one host thread issues every shard's stages back to back on its
# streams; its time in the call minus the time blocked in the protocol's host
# syncs is the issue cost a host thread pays per step for all shards
m.set_option("sim", 0)
s_ = torch.cuda.Stream(dev)
host_issue_ms, host_wait_ms = {}, {}
for ht in (1, 0):  # a host thread per shard (default), one thread for all shards
    m.set_option("host_threads", ht)
    host = []
    for rep in range(args.reps):
        with torch.cuda.stream(s_):
            m.search_device(q.data_ptr(), B, d, k, oi.data_ptr(), od.data_ptr(), on.data_ptr(), s_.cuda_stream)
        hs = m.stats()
        host.append((hs["host_us"], hs["host_wait_us"]))
        s_.synchronize()
    host_issue_ms[ht] = float(np.median([(a - b) / 1e3 for a, b in host]))
    host_wait_ms[ht] = float(np.median([b / 1e3 for a, b in host]))
m.set_option("host_threads", 1)
# the collectives' bytes per rank: keys + eps, the lists, the records
k1 = k + 1
gbytes = [B * k1 * 4 + B * 4, B * k1 * 16 + B * 8]
F = st["last_flagged"]
if F:
    gbytes.append(F * max(256, 16 * k) * 12 + F * 4)
stage_max = {s: float(np.mean([max(r[s]) for r in rows])) for s in STAGES[:-1]}
per_shard = {s: [float(x) for x in np.mean([r[s] for r in rows], 0)] for s in STAGES[:-1]}
compute = sum(stage_max.values())
# RCCL all-gather over 8 GPUs on xGMI: ~25 us launch + the ring at ~100 GB/s per link (estimate)
xfer_est = sum(25e-3 + (W - 1) * b / 100e9 * 1e3 for b in gbytes)
out = dict(world=W, n=n, d=d, batch=B, k=k, flagged=F, stage_max_ms=stage_max, per_shard_ms=per_shard,
           compute_ms=compute, allgather_bytes_per_rank=gbytes, allgather_est_ms=xfer_est,
           predicted_step_ms=compute + xfer_est, timed_order="reverse" if args.rev else "forward",
           host_issue_ms={"thread_per_shard": host_issue_ms[1], "one_thread": host_issue_ms[0]},
           host_wait_ms={"thread_per_shard": host_wait_ms[1], "one_thread": host_wait_ms[0]})
same = None
if not args.no_single:
    res = (oi.clone(), od.clone(), on.clone())
    m.close()
    torch.cuda.empty_cache()
    single = wv.FlatIndex(distance="cosine", dims=d, variant="avx256")
    single.reserve(n)
    stage = torch.empty((1_000_000, d), dtype=torch.float32, device=dev)
    for r0 in range(0, n, 1_000_000):
        c = min(1_000_000, n - r0)
        _lib.check(lib.wv_gen_device(0, 0, 1, r0, c, d, stage.data_ptr(), None))
        _lib.check(lib.wv_index_add_range_device(single._h, r0, stage.data_ptr(), c, d))
    del stage
    si = torch.empty((B, k), dtype=torch.int64, device=dev)
    sd = torch.empty((B, k), dtype=torch.float32, device=dev)
    sn = torch.empty(B, dtype=torch.int32, device=dev)
    _lib.check(lib.wv_index_search_device(single._h, q.data_ptr(), B, d, k, 0, si.data_ptr(), sd.data_ptr(),
                                          sn.data_ptr(), None, None))
    torch.cuda.synchronize()
    same = bool(torch.equal(res[2], sn) and torch.equal(res[0], si) and torch.equal(res[1].view(torch.int32),
                                                                                    sd.view(torch.int32)))
out["equal_to_single"] = same
print(json.dumps(out), flush=True)
if same is False:
    sys.exit(3)
