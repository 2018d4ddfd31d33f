"""A/B of the PQ ADC kernels on the C5 shape (10M x 960, m=240, ks=256, B=256),
interleaved in one process; ADC launch time (HIP events) and whole batch.
Default configs: k_pq_adc3 (pq_adc3=1), k_pq_adc2 (pq_adc3=0), and the adc3
timing experiments (pq_adc3=3: no LUT DMA, 4: no per-segment barrier; 5:
k_pq_adc4 without LUT DMA; debug library only, WV_LIB_PATH; their results are
wrong by construction and are not compared).  pq_adc3=2 is k_pq_adc4.  Results of the
other settings must be identical.  Usage: pq_probe.py [cfg ...]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import weaviate_amd as wv  # noqa: E402
from weaviate_amd import _lib  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
n, d, B, k = 10_000_000, 960, 256, 10
idx = wv.FlatIndex(distance="l2-squared", dims=d, variant="avx256",
                   pq={"segments": 240, "centroids": 256, "trainingLimit": 100_000, "rescore": False})
idx.reserve(n)
stage = torch.empty((1_000_000, d), dtype=torch.float32, device=dev)
for r0 in range(0, n, 1_000_000):
    _lib.check(lib.wv_gen_device(0, 2, 1, r0, 1_000_000, d, stage.data_ptr(), None))
    _lib.check(lib.wv_index_add_range_device(idx._h, r0, stage.data_ptr(), 1_000_000, d))
del stage
idx.pq_fit(seed=1)
q = torch.empty((B, d), dtype=torch.float32, device=dev)
_lib.check(lib.wv_gen_device(0, 2, 2, 0, B, d, q.data_ptr(), None))
oi = torch.empty((B, k), dtype=torch.int64, device=dev)
od = torch.empty((B, k), dtype=torch.float32, device=dev)
on = torch.empty(B, dtype=torch.int32, device=dev)
idx.set_option("timing", 1)
torch.cuda.synchronize()


def run():
    s = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(lib.wv_index_search_device(idx._h, q.data_ptr(), B, d, k, 0, oi.data_ptr(), od.data_ptr(),
                                          on.data_ptr(), None, s))


ref = None
cfgs = sys.argv[1:] or ["pq_adc3=1", "pq_adc3=0", "pq_adc3=3", "pq_adc3=4"] * 2
for cfg in cfgs:
    for kv in cfg.split(","):
        key, val = kv.split("=")
        idx.set_option(key, int(val))
    run()
    torch.cuda.synchronize()
    sel = []
    t0 = time.perf_counter()
    for _ in range(3):
        run()
        sel.append(idx.stats()["last_select_ms"])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    got = (oi.clone(), od.clone(), on.clone())
    timing_only = cfg in ("pq_adc3=3", "pq_adc3=4", "pq_adc3=5")
    if ref is None and not timing_only:
        ref = got
    same = None if timing_only else all(torch.equal(a, b) for a, b in zip(ref, got))
    print(f"{cfg:22s} adc {min(sel):8.2f} ms  batch {dt * 1e3:8.2f} ms  QPS {B / dt:8.0f}  same {same}", flush=True)
