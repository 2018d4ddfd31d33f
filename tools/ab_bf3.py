"""Timing breakdown of k_mfma_select_bf3 on the C3 shape: full kernel, without
the selection epilogue (sel_dbg=1), staging only (sel_dbg=2).  Results of the
dbg runs are not used.  Usage: python tools/ab_bf3.py [n] [batch]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import weaviate_amd as wv
from weaviate_amd import _lib

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
opts = [kv.split("=") for kv in sys.argv[3:]]
D = 768
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
fl = torch.empty(B, dtype=torch.int32, device=dev)
idx.set_option("timing", 1)
for k, v in opts:
    idx.set_option(k, int(v))
for dbg in [int(x) for x in os.environ.get('DBGS', '0,1,2').split(',')]:
    idx.set_option("sel_dbg", dbg)
    ms = []
    for it in range(4):
        _lib.check(lib.wv_index_search_device(idx._h, q.data_ptr(), B, D, 10, 1, oi.data_ptr(), od.data_ptr(),
                                              on.data_ptr(), fl.data_ptr(), None))
        if it:
            ms.append(idx.stats()["last_select_ms"])
    print(f"sel_dbg={dbg} {opts} select ms: {sum(ms) / len(ms):.2f}", flush=True)
