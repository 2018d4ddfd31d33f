"""Small-batch route measurement on the C3 corpus (10M x 768 cosine, k = 10):
per batch size, the register-streaming int8 key kernel (q8_gemv, <= 32
queries), the padded block-key route (qs, the int8 key pass over 256-query
groups) and the HBM-streaming fp32 GEMV select (kernel 6), device-resident
queries, wall clock over repeated calls.  Prints one JSON line per (B, route)
and a final line with the crossover the runtime's `gemv_max` default encodes."""
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
ap.add_argument("--batches", default="1,2,4,8,16,32,64,128,256")
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()

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
torch.cuda.synchronize()
print("corpus ready", flush=True)


def run(B):
    s = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(lib.wv_index_search_device(idx._h, q.data_ptr(), B, args.d, args.k, 0, oi.data_ptr(), od.data_ptr(),
                                          on.data_ptr(), None, s))


best = {}
for B in (int(b) for b in args.batches.split(",")):
    res = {}
    for route, opts in (("q8_gemv", {"kernel": 0, "gemv_max": 0, "q8_gemv": 1}),
                        ("qs", {"kernel": 0, "gemv_max": 0, "q8_gemv": 0}),
                        ("gemv", {"kernel": 6, "gemv_max": 4096})):
        for kk, vv in opts.items():
            idx.set_option(kk, vv)
        run(B)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            run(B)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.reps
        st = idx.stats()
        res[route] = (dt, oi[:B].cpu().clone(), od[:B].cpu().clone())
        print(json.dumps({"B": B, "route": route, "ran": _lib.ROUTES.get(st["last_route"], st["last_route"]),
                          "ms": round(dt * 1e3, 3), "qps": round(B / dt, 1)}), flush=True)
    same = all(bool(torch.equal(res["qs"][1], res[r][1]) and torch.equal(res["qs"][2], res[r][2])) for r in res)
    best[B] = min(res, key=lambda r: res[r][0])
    print(json.dumps({"B": B, "faster": best[B], "same_results": same}), flush=True)
print(json.dumps({"faster_by_batch": best}), flush=True)
idx.close()
