"""Times the host-buffer batch path (wv_index_search_by_vector_batch) at a few
batch sizes on the C3 corpus, single caller -- a probe for the micro-batcher's
per-launch cost (compare bench.py --batch B, device buffers)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import weaviate_amd as wv
    from weaviate_amd import _lib
    lib = _lib.load()
    n, d = int(os.environ.get("N", 10_000_000)), 768
    idx = wv.FlatIndex(distance="cosine", dims=d, variant="avx256")
    idx.reserve(n)
    stage = torch.empty((1_000_000, d), dtype=torch.float32, device="cuda")
    for r0 in range(0, n, 1_000_000):
        m = min(1_000_000, n - r0)
        _lib.check(lib.wv_gen_device(0, 0, 1, r0, m, d, stage.data_ptr(), None))
        _lib.check(lib.wv_index_add_range_device(idx._h, r0, stage.data_ptr(), m, d))
    qd = torch.empty((512, d), dtype=torch.float32, device="cuda")
    _lib.check(lib.wv_gen_device(0, 0, 2, 0, 512, d, qd.data_ptr(), None))
    torch.cuda.synchronize()
    q = qd.cpu().numpy()
    idx.set_option("timing", 1)
    batches = [int(x) for x in os.environ.get("BATCHES", "1,64,111,128,205,256").split(",")]
    runs = [(int(x), None) for x in os.environ.get("KERNELS", "0").split(",")]
    runs += [(6, int(w)) for w in os.environ.get("GEMV_WGS", "").split(",") if w]
    for kern, wg in runs:
      idx.set_option("kernel", kern)
      if wg:
          idx.set_option("gemv_wg", wg)
      print(f"kernel option {kern} gemv_wg {wg}", flush=True)
      for b in batches:
        idx.search_by_vector_batch(q[:b], 10)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            idx.search_by_vector_batch(q[:b], 10)
            ts.append(time.perf_counter() - t0)
        st = idx.stats()
        print(f"  B={b}: host-path {min(ts)*1e3:.2f} ms  select {st['last_select_ms']:.2f} ms  total {st['last_total_ms']:.2f} ms  replayed {st['replayed_queries']}", flush=True)


if __name__ == "__main__":
    main()
