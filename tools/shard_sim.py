"""Per-rank cost of the sharded exact search at W ranks, measured on ONE GPU:
the C3 corpus (10M x 768 cosine) split into W contiguous id-range shards held
as W indexes on the same device; every stage of ShardedFlatSearch is timed per
shard with HIP events (phase 1, phase 2, merge, each shard's part of the
parallel replay, the record merge), the collectives are not (one GPU).
Predicted step at W ranks = max_r(phase1) + gather + max_r(phase2) + gather +
merge + max_r(replay part) + gather + record merge.
Also checks the merged results against the single-GPU search of the same
batch (bit-exact ids and distances).  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--d", type=int, default=768)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--batch", type=int, default=2048)
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402
import weaviate_amd as wv  # noqa: E402
from weaviate_amd import _lib  # noqa: E402
from weaviate_amd.sharded import GpuShardBackend, ShardedFlatSearch, fake_heaps, prefix_bound  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
W, n, d, k, B = args.world, args.n, args.d, args.k, args.batch
per = (n + W - 1) // W
backs = []
stage = torch.empty((1_000_000, d), dtype=torch.float32, device=dev)
for r in range(W):
    lo, hi = r * per, min(n, (r + 1) * per)
    idx = wv.FlatIndex(distance="cosine", dims=d, variant="avx256", id_base=lo)
    idx.reserve(hi - lo)
    for r0 in range(lo, hi, 1_000_000):
        m = min(1_000_000, hi - r0)
        _lib.check(lib.wv_gen_device(0, 0, 1, r0, m, d, stage.data_ptr(), None))
        _lib.check(lib.wv_index_add_range_device(idx._h, r0, stage.data_ptr(), m, d))
    backs.append(GpuShardBackend(idx, 0))
del stage
q = torch.empty((B, d), dtype=torch.float32, device=dev)
_lib.check(lib.wv_gen_device(0, 0, 2, 0, B, d, q.data_ptr(), None))
torch.cuda.synchronize()


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = fn()
    e1.record()
    torch.cuda.synchronize()
    return out, e0.elapsed_time(e1)


rows = []
for rep in range(args.reps + 1):
    t = {}
    p1 = []
    t1 = []
    for b in backs:
        out, ms = timed(lambda b=b: b.phase1(q, k))
        p1.append(out)
        t1.append(ms)
    gA = torch.stack([a for a, _ in p1])
    gE = torch.stack([e for _, e in p1])
    parts, t2 = [], []
    for b in backs:
        out, ms = timed(lambda b=b: b.phase2(gA, gE, k))
        parts.append(out)
        t2.append(ms)
    k1 = k + 1
    packed = [torch.cat([p[0].view(torch.int32).reshape(B, 2 * k1), p[1].view(torch.int32), p[2][:, None],
                         p[3][:, None]], 1) for p in parts]
    G = torch.stack(packed)
    gi = G[..., : 2 * k1].contiguous().view(torch.int64)
    gd = G[..., 2 * k1: 3 * k1].contiguous().view(torch.float32)
    gc = G[..., 3 * k1].contiguous()
    gf = G[..., 3 * k1 + 1].contiguous()
    (oi, od, on, of), tm = timed(lambda: backs[0].merge(W, k, gi, gd, gc, gf))
    # parallel replay: shard 0 from empty heaps, shards >= 1 recording from T_r
    ql = torch.nonzero(of).flatten()
    F = int(ql.numel())
    ql32 = ql.to(torch.int32)
    cap = 256
    trec = []
    if F:
        (ti, td, tn), t0 = timed(lambda: backs[0].replay(q, ql32, None, k, False))
        trec.append(t0)
        ri = torch.zeros((W, F, cap), dtype=torch.int64, device=dev)
        rd = torch.zeros((W, F, cap), dtype=torch.float32, device=dev)
        rn = torch.zeros((W, F), dtype=torch.int32, device=dev)
        for r in range(1, W):
            T = prefix_bound(r, ql, k, gd, gc, gf, (gA, gE))
            out, ms = timed(lambda b=backs[r], T=T: b.replay_record(q, ql32, fake_heaps(T, k), k, cap))
            ri[r], rd[r], rn[r] = out
            trec.append(ms)
        (fi_, fd_, fn_, un), tmr = timed(lambda: backs[0].merge_records(W, k, cap, (ti.contiguous(), td.contiguous(), tn),
                                                                        (ri, rd, rn)))
        assert not bool(un.any())
        oi[ql], od[ql], on[ql] = fi_, fd_, fn_
        nrec = [int(x) for x in rn.max(1).values.tolist()]
    else:
        tmr, nrec = 0.0, []
    state = (oi, od, on)
    th = trec
    nflag = F
    if rep:
        rows.append(dict(phase1=t1, phase2=t2, merge=tm, replay=th, merge_rec=tmr, flagged=nflag, max_records=nrec))
    fi, fd, fn = state

# single-GPU reference of the same batch (the bench path)
single = wv.FlatIndex(distance="cosine", dims=d, variant="avx256")
for b in backs:
    b.index.close()
del backs
torch.cuda.empty_cache()
single.reserve(n)
stage = torch.empty((1_000_000, d), dtype=torch.float32, device=dev)
for r0 in range(0, n, 1_000_000):
    m = min(1_000_000, n - r0)
    _lib.check(lib.wv_gen_device(0, 0, 1, r0, m, d, stage.data_ptr(), None))
    _lib.check(lib.wv_index_add_range_device(single._h, r0, stage.data_ptr(), m, d))
del stage
si = torch.empty((B, k), dtype=torch.int64, device=dev)
sd = torch.empty((B, k), dtype=torch.float32, device=dev)
sn = torch.empty(B, dtype=torch.int32, device=dev)
_lib.check(lib.wv_index_search_device(single._h, q.data_ptr(), B, d, k, 0, si.data_ptr(), sd.data_ptr(), sn.data_ptr(),
                                      None, None))
torch.cuda.synchronize()
same = bool(torch.equal(fn, sn) and torch.equal(fi, si) and torch.equal(fd.view(torch.int32), sd.view(torch.int32)))


def avg(key, red):
    return float(np.mean([red(r[key]) for r in rows]))


pred = dict(phase1_max=avg("phase1", max), phase2_max=avg("phase2", max), merge=avg("merge", float),
            replay_max=avg("replay", lambda v: max(v) if v else 0.0), merge_rec=avg("merge_rec", float),
            replay_per_shard=rows[-1]["replay"],
            max_records=rows[-1]["max_records"])
pred["compute_ms"] = pred["phase1_max"] + pred["phase2_max"] + pred["merge"] + pred["replay_max"] + pred["merge_rec"]
print(json.dumps(dict(world=W, n=n, d=d, batch=B, k=k, flagged=rows[-1]["flagged"], equal_to_single=same,
                      phase1=[float(x) for x in np.mean([r["phase1"] for r in rows], 0)],
                      phase2=[float(x) for x in np.mean([r["phase2"] for r in rows], 0)], **pred)), flush=True)
if not same:
    sys.exit(3)
