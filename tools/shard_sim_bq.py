"""Per-rank cost of the sharded BQ search (ShardedBQSearch, BASELINE configs[3]:
50M x 1536 over 8 GPUs = one 6.25M-row shard per GPU), measured on ONE GPU.

Eight 6.25M x 1536 shards (fp32 rows for rescoring + codes) do not fit one
GPU's HBM together, so every rank is the same physical shard: rank r's stages
run on it with rank r's inputs (the gathered bounds of ranks < r, its fake
heaps of R copies of T_r).  That reproduces each rank's work -- the block
minima, the bounds, rank 0's replay from empty heaps, the recorded replays of
ranks >= 1 from their T_r, the record merge, rescoring and the final heap --
on statistically identical data; the collectives are not timed (one GPU).
Predicted step at W ranks = max(begin) + gather + max_r(replay / record) +
gather + merge + rescore + gather + final; the serial chain it replaces costs
begin + W x replay.  Prints one JSON line."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=6_250_000)
ap.add_argument("--d", type=int, default=1536)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--batch", type=int, default=2048)
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--rescore", type=int, default=200)
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402
import weaviate_amd as wv  # noqa: E402
from weaviate_amd import _lib  # noqa: E402
from weaviate_amd.sharded import GpuBQShardBackend, fake_heaps, prefix_bound  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
W, n, d, k, B = args.world, args.n, args.d, args.k, args.batch
idx = wv.FlatIndex(distance="cosine", dims=d, variant="avx256", bq=True, rescore_limit=args.rescore)
idx.reserve(n)
stage = torch.empty((1_000_000, d), dtype=torch.float32, device=dev)
for r0 in range(0, n, 1_000_000):
    m = min(1_000_000, n - r0)
    _lib.check(lib.wv_gen_device(0, 0, 1, r0, m, d, stage.data_ptr(), None))
    _lib.check(lib.wv_index_add_range_device(idx._h, r0, stage.data_ptr(), m, d))
del stage
b = GpuBQShardBackend(idx, 0)
q = torch.empty((B, d), dtype=torch.float32, device=dev)
_lib.check(lib.wv_gen_device(0, 0, 2, 0, B, d, q.data_ptr(), None))
torch.cuda.synchronize()
R = b.R(k)
cap = 2 * R


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = fn()
    e1.record()
    torch.cuda.synchronize()
    return out, e0.elapsed_time(e1)


best = None
for rep in range(args.reps):
    st = {}
    _, st["begin"] = timed(lambda: b.bq_begin(q, k))
    bnd, st["bounds"] = timed(lambda: b.bq_bounds())
    G = bnd[None].expand(W, B, R).contiguous()  # every rank's bounds (the same shard)
    (ti, td, tn), t0 = timed(lambda: b.bq_replay(None, False))
    rep_ms, rec_n = [t0], [int(R)]
    recs = [None]
    allq = torch.arange(B, device=dev)
    for r in range(1, W):
        T = prefix_bound(r, allq, R, G, torch.full((r, B), R, dtype=torch.int32, device=dev),
                         torch.zeros((r, B), dtype=torch.int32, device=dev))
        fh = fake_heaps(T, R)
        rec, t = timed(lambda: b.bq_replay_record(fh, cap))
        rep_ms.append(t)
        recs.append(rec)
        rec_n.append(float(rec[2].float().mean()))
    ri = torch.zeros((W, B, cap), dtype=torch.int64, device=dev)
    rd = torch.zeros((W, B, cap), dtype=torch.float32, device=dev)
    rn = torch.zeros((W, B), dtype=torch.int32, device=dev)
    for r in range(1, W):
        ri[r], rd[r], rn[r] = recs[r]
    overflow = int((rn > cap).sum())
    (ai, ad, an, un), st["merge"] = timed(lambda: b.merge_records(W, R, cap, (ti, td, tn), (ri, rd, rn)))
    back = (an[:, None].long() - 1 - torch.arange(R, device=dev)[None, :]).clamp(min=0)
    ids = ai.gather(1, back)
    E, st["rescore"] = timed(lambda: b.bq_rescore(ids, an))
    E_all = E[None].expand(W, B, R).contiguous()
    _, st["final"] = timed(lambda: b.bq_final(W, n, ids, an, E_all))
    st["replay_rank0"] = rep_ms[0]
    st["record_max_r>=1"] = max(rep_ms[1:]) if W > 1 else 0.0
    st["replay_stage"] = max(rep_ms)
    pred = st["begin"] + st["bounds"] + st["replay_stage"] + st["merge"] + st["rescore"] + st["final"]
    chain = st["begin"] + W * rep_ms[0] + st["rescore"] + st["final"]
    row = {"stages_ms": {kk: round(v, 3) for kk, v in st.items()}, "replay_ms_per_rank": [round(x, 3) for x in rep_ms],
           "mean_record_len_per_rank": rec_n, "records_overflowed": overflow,
           "gather_bytes_per_rank": {"bounds": B * R * 4, "records": B * (3 * cap + 1) * 4, "E": B * R * 4},
           "predicted_step_ms_gpu_work": round(pred, 3), "serial_chain_step_ms_gpu_work": round(chain, 3),
           "replay_stage_over_one_rank_replay": round(st["replay_stage"] / rep_ms[0], 3)}
    if best is None or pred < best["predicted_step_ms_gpu_work"]:
        best = row
print(json.dumps({"tool": "shard_sim_bq", "world": W, "rows_per_rank": n, "dims": d, "batch": B, "k": k, "R": R,
                  "cap": cap, **best}))
