"""A/B of index options on the C3 corpus (10M x 768 cosine, k = 10) in one
process: per batch size, each option set in alternating rounds (A B A B ...),
wall clock per search_device call and the block-key launch time from HIP
events (wv_stats.last_select_ms), results compared bit for bit across the
option sets.  One JSON line per (B, option set) with the median over rounds.

  python tools/ab_q8.py --batches 64,128,256 --sets '{"q8_live":0}' '{"q8_live":1}'
"""
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
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--batches", default="64,128,256")
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--sets", nargs="+", default=['{}'])
args = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402
import weaviate_amd as wv  # noqa: E402
from weaviate_amd import _lib  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
idx = wv.FlatIndex(distance="cosine", dims=args.d, variant="avx256")
idx.reserve(args.n)
chunk = 1_000_000
stage = torch.empty((min(chunk, args.n), args.d), dtype=torch.float32, device=dev)
for r0 in range(0, args.n, chunk):
    m = min(chunk, args.n - r0)
    _lib.check(lib.wv_gen_device(0, 0, 1, r0, m, args.d, stage.data_ptr(), None))
    _lib.check(lib.wv_index_add_range_device(idx._h, r0, stage.data_ptr(), m, args.d))
del stage
bmax = max(int(b) for b in args.batches.split(","))
q = torch.empty((bmax, args.d), dtype=torch.float32, device=dev)
_lib.check(lib.wv_gen_device(0, 0, 2, 0, bmax, args.d, q.data_ptr(), None))
oi = torch.empty((bmax, args.k), dtype=torch.int64, device=dev)
od = torch.empty((bmax, args.k), dtype=torch.float32, device=dev)
on = torch.empty(bmax, dtype=torch.int32, device=dev)
idx.set_option("timing", 1)
torch.cuda.synchronize()
print(json.dumps({"corpus": [args.n, args.d]}), flush=True)
sets = [json.loads(x) for x in args.sets]


def run(B):
    s = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(lib.wv_index_search_device(idx._h, q.data_ptr(), B, args.d, args.k, 0, oi.data_ptr(), od.data_ptr(),
                                          on.data_ptr(), None, s))


for B in (int(b) for b in args.batches.split(",")):
    wall = {i: [] for i in range(len(sets))}
    key = {i: [] for i in range(len(sets))}
    out = {}
    for r in range(args.rounds):
        for i, opts in enumerate(sets):
            for kk, vv in opts.items():
                idx.set_option(kk, int(vv))
            run(B)
            torch.cuda.synchronize()
            ks = []
            t0 = time.perf_counter()
            for _ in range(args.reps):
                run(B)
                ks.append(idx.stats()["last_select_ms"])
            torch.cuda.synchronize()
            wall[i].append((time.perf_counter() - t0) / args.reps * 1e3)
            key[i].append(float(np.median(ks)))
            out[i] = (oi[:B].cpu().clone(), od[:B].cpu().clone(), on[:B].cpu().clone())
            for kk in opts:  # back to the defaults for the next set
                idx.set_option(kk, {"q8_live": 1, "q8_prio": 0}.get(kk, 0))
    same = all(all(bool(torch.equal(out[0][j], out[i][j])) for j in range(3)) for i in out)
    for i, opts in enumerate(sets):
        print(json.dumps({"B": B, "opts": opts, "ms": round(float(np.median(wall[i])), 4),
                          "key_ms": round(float(np.median(key[i])), 4), "qps": round(B / np.median(wall[i]) * 1e3, 1),
                          "rounds_ms": [round(x, 3) for x in wall[i]], "same_results": same}), flush=True)
idx.close()
