"""A/B the selection kernels in one process (rule: interleaved rounds).
python tools/ab_select.py [n_rows] [batch] [rounds] [variants...]"""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import weaviate_amd as wv
from weaviate_amd import _lib

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 4
variants = [int(v) for v in sys.argv[4:]] or [1, 2]
d, k = 768, 10
lib = _lib.load()
dev = torch.device("cuda", 0)
idx = wv.FlatIndex(distance="cosine", dims=d, variant="avx256")
idx.reserve(n)
stage = torch.empty((min(n, 1_000_000), d), dtype=torch.float32, device=dev)
for r0 in range(0, n, 1_000_000):
    m = min(1_000_000, n - r0)
    _lib.check(lib.wv_gen_device(0, 0, 1, r0, m, d, stage.data_ptr(), None))
    _lib.check(lib.wv_index_add_range_device(idx._h, r0, stage.data_ptr(), m, d))
q = torch.empty((B, d), dtype=torch.float32, device=dev)
_lib.check(lib.wv_gen_device(0, 0, 2, 0, B, d, q.data_ptr(), None))
oi = torch.empty((B, k), dtype=torch.int64, device=dev)
od = torch.empty((B, k), dtype=torch.float32, device=dev)
on = torch.empty(B, dtype=torch.int32, device=dev)
idx.set_option("timing", 1)
res = {v: [] for v in variants}
outs = {}
for r in range(rounds):
    for v in variants:
        idx.set_option("kernel", v)
        _lib.check(lib.wv_index_search_device(idx._h, q.data_ptr(), B, d, k, 0, oi.data_ptr(), od.data_ptr(),
                                              on.data_ptr(), None, None))
        res[v].append(idx.stats()["last_select_ms"])
        outs[v] = oi.cpu().numpy().copy()
flops = 2.0 * B * n * d
for v in variants:
    ms = np.array(res[v][1:] if rounds > 1 else res[v])
    print(f"kernel {v}: median {np.median(ms):.2f} ms min {ms.min():.2f} -> {flops / (np.median(ms) * 1e-3) / 1e12:.1f} TFLOP/s")
base = outs[variants[0]]
for v in variants[1:]:
    print(f"kernel {v} ids equal to kernel {variants[0]}: {np.array_equal(outs[v], base)}")
