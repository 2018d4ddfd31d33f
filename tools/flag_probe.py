"""Why are queries flagged?  C3 (or --workload c2) mode-1 search: flag values
(1 = proof failed: equal exact distances among the first k+1, 2 = candidate
list overflow / non-finite) and, for flagged queries, their k+1 distances."""
import argparse, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import weaviate_amd as wv
from weaviate_amd import _lib

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c3")
a = ap.parse_args()
cfg = {"c3": (10_000_000, 768, "cosine", 0, 10, 2048), "c2": (1_000_000, 128, "l2-squared", 1, 100, 10000)}[a.workload]
n, d, metric, kind, k, B = cfg
lib = _lib.load()
idx = wv.FlatIndex(distance=metric, dims=d, variant="avx256")
idx.reserve(n)
stage = torch.empty((1_000_000, d), dtype=torch.float32, device="cuda")
for r0 in range(0, n, 1_000_000):
    m = min(1_000_000, n - r0)
    _lib.check(lib.wv_gen_device(0, kind, 1, r0, m, d, stage.data_ptr(), None))
    _lib.check(lib.wv_index_add_range_device(idx._h, r0, stage.data_ptr(), m, d))
q = torch.empty((B, d), dtype=torch.float32, device="cuda")
_lib.check(lib.wv_gen_device(0, kind, 2, 0, B, d, q.data_ptr(), None))
oi = torch.empty((B, k + 1), dtype=torch.int64, device="cuda")
od = torch.empty((B, k + 1), dtype=torch.float32, device="cuda")
on = torch.empty(B, dtype=torch.int32, device="cuda")
of = torch.empty(B, dtype=torch.int32, device="cuda")
_lib.check(lib.wv_index_search_device(idx._h, q.data_ptr(), B, d, k, 1, oi.data_ptr(), od.data_ptr(), on.data_ptr(),
                                      of.data_ptr(), None))
torch.cuda.synchronize()
f = of.cpu().numpy()
print("flags:", {int(v): int((f == v).sum()) for v in np.unique(f)}, flush=True)
for qq in np.nonzero(f)[0][:12]:
    A, eps = idx.debug_blockkeys(int(qq))
    s = np.sort(A)
    M = s[k]
    print(f"q{qq} flag {f[qq]} eps {eps:.3e} M {M:.6f} blocks<=M+2eps {(A <= M + 2.0005 * eps).sum()}", flush=True)
    print("   dists", od[qq, :on[qq]].cpu().numpy())
