"""Timing probe of the block-key kernel on the C3 corpus (10M x 768 cosine):
last_select_ms per option setting (sel_dbg / spans), and the whole batch."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--d", type=int, default=768)
ap.add_argument("--batch", type=int, default=2048)
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--metric", default="cosine")
ap.add_argument("--kind", type=int, default=0)
ap.add_argument("--configs", default="sel_dbg=0;sel_dbg=0")
ap.add_argument("--verify", type=int, default=1, help="compare every result with the f32 GEMV path (kernel 6)")
args = ap.parse_args()

import torch  # noqa: E402
import weaviate_amd as wv  # noqa: E402
from weaviate_amd import _lib  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
idx = wv.FlatIndex(distance=args.metric, dims=args.d, variant="avx256")
idx.reserve(args.n)
chunk = 1_000_000
stage = torch.empty((min(chunk, args.n), args.d), dtype=torch.float32, device=dev)
for r0 in range(0, args.n, chunk):
    m = min(chunk, args.n - r0)
    _lib.check(lib.wv_gen_device(0, args.kind, 1, r0, m, args.d, stage.data_ptr(), None))
    _lib.check(lib.wv_index_add_range_device(idx._h, r0, stage.data_ptr(), m, args.d))
del stage
B = args.batch
q = torch.empty((B, args.d), dtype=torch.float32, device=dev)
_lib.check(lib.wv_gen_device(0, args.kind, 2, 0, B, args.d, q.data_ptr(), None))
oi = torch.empty((B, args.k), dtype=torch.int64, device=dev)
od = torch.empty((B, args.k), dtype=torch.float32, device=dev)
on = torch.empty(B, dtype=torch.int32, device=dev)
idx.set_option("timing", 1)
torch.cuda.synchronize()


def run():
    s = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(lib.wv_index_search_device(idx._h, q.data_ptr(), B, args.d, args.k, 0, oi.data_ptr(), od.data_ptr(),
                                          on.data_ptr(), None, s))


for cfg in args.configs.split(";"):
    for kv in cfg.split(","):
        key, val = kv.split("=")
        idx.set_option(key, int(val))
    run()
    torch.cuda.synchronize()
    sel = []
    t0 = time.perf_counter()
    for _ in range(5):
        run()
        sel.append(idx.stats()["last_select_ms"])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    print(f"{cfg:30s} select {min(sel):8.2f} ms  batch {dt*1e3:8.2f} ms  QPS {B/dt:10.0f}  "
          f"replayed {idx.stats()['replayed_queries']}", flush=True)

if args.verify:
    idx.set_option("kernel", 0)
    run()
    a_i, a_d, a_n = oi.cpu().numpy().copy(), od.cpu().numpy().copy(), on.cpu().numpy().copy()
    idx.set_option("kernel", 6)
    idx.set_option("gemv_max", 1 << 12)
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    b_i, b_d, b_n = oi.cpu().numpy(), od.cpu().numpy(), on.cpu().numpy()
    import numpy as np
    bad = [q for q in range(B) if a_n[q] != b_n[q] or not np.array_equal(a_i[q, :a_n[q]], b_i[q, :b_n[q]])
           or not np.array_equal(a_d[q, :a_n[q]].view(np.uint32), b_d[q, :b_n[q]].view(np.uint32))]
    print(f"verify vs GEMV (kernel 6, {time.perf_counter() - t0:.1f} s): {len(bad)} of {B} queries differ", flush=True)
    for q in bad[:5]:
        print("  q", q, a_i[q, :5], b_i[q, :5], a_d[q, :3], b_d[q, :3])
