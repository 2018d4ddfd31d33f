"""A/B of select-kernel options on the C3 shape in one process (one index
build): each argument is an option set "k=v,k=v" (empty = defaults); prints
the mean select ms and the QPS of the whole search per set.
Usage: python tools/ab_opts.py [--n N] [--batch B] "qgroup=4" "qgroup=16" ..."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import weaviate_amd as wv
from weaviate_amd import _lib

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--batch", type=int, default=2048)
ap.add_argument("--dims", type=int, default=768)
ap.add_argument("--iters", type=int, default=4)
ap.add_argument("--lib", default=None, help="load this libwvknn build instead (A/B of two builds)")
ap.add_argument("sets", nargs="*")
args = ap.parse_args()
n, B, D = args.n, args.batch, args.dims
if args.lib:
    _lib.LIB_PATH = args.lib
lib = _lib.load()
dev = torch.device("cuda", 0)
idx = wv.FlatIndex(distance="cosine", dims=D, variant="avx256")
idx.reserve(n)
st = torch.empty((1_000_000, D), dtype=torch.float32, device=dev)
for r0 in range(0, n, 1_000_000):
    m = min(1_000_000, n - r0)
    _lib.check(lib.wv_gen_device(0, 0, 1, r0, m, D, st.data_ptr(), None))
    _lib.check(lib.wv_index_add_range_device(idx._h, r0, st.data_ptr(), m, D))
del st
q = torch.empty((B, D), dtype=torch.float32, device=dev)
_lib.check(lib.wv_gen_device(0, 0, 2, 0, B, D, q.data_ptr(), None))
oi = torch.empty((B, 10), dtype=torch.int64, device=dev)
od = torch.empty((B, 10), dtype=torch.float32, device=dev)
on = torch.empty(B, dtype=torch.int32, device=dev)
idx.set_option("timing", 1)
ref = None
for s in (args.sets or [""]):
    opts = [kv.split("=") for kv in s.split(",") if kv]
    for k, v in opts:
        idx.set_option(k, int(v))
    ms = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for it in range(args.iters):
        _lib.check(lib.wv_index_search_device(idx._h, q.data_ptr(), B, D, 10, 0, oi.data_ptr(), od.data_ptr(),
                                              on.data_ptr(), None, None))
        ms.append(idx.stats()["last_select_ms"])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ids = oi.cpu()
    same = "" if ref is None else f" ids==first:{bool((ids == ref).all())}"
    if ref is None:
        ref = ids
    print(f"[{s}] select ms: {sum(ms[1:]) / max(1, len(ms) - 1):.2f}  search QPS {B * args.iters / dt:.0f}{same}",
          flush=True)
    # restore defaults the set changed (only keys known to default to 0)
    for k, v in opts:
        if k in ("qgroup", "spans", "cbuf", "sel_dbg", "sel_opt"):
            idx.set_option(k, 0)
