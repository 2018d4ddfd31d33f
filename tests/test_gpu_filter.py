"""GPU parity of filtered search (flat/index.go:578-619: the LSM cursor seeks
to allow.Min() and stops past allow.Max(), keeping only allowed keys).  The
allow bitmap is built on the device from the id list and the scan covers only
the allow list's slot span (ScanWindow): results equal the oracle, and the
rows scanned follow the span, not the corpus."""
import time

import numpy as np
import pytest

from test_gpu_flat import assert_same, build_pair, build_bq_pair, gen
from test_gpu_scale import assert_rows, device_index, oracle_threads

pytestmark = pytest.mark.gpu


def allow_cases(n, rng):
    return {
        "span": np.arange(n // 3, n // 3 + 5000, dtype=np.uint64),              # one contiguous id range
        "sparse_in_span": np.sort(rng.choice(np.arange(n // 2, n // 2 + 20000), 700, replace=False)).astype(np.uint64),
        "random_all": np.sort(rng.choice(n, 3000, replace=False)).astype(np.uint64),
        "single": np.array([n - 5], dtype=np.uint64),
        "with_absent": np.concatenate([np.arange(100, 400), np.arange(n + 10, n + 50)]).astype(np.uint64),
        "dup_unsorted": np.array([777, 5, 777, n - 1, 5, 3000], dtype=np.uint64),
    }


@pytest.mark.parametrize("metric,kind,d,k", [("cosine", 0, 768, 10), ("l2-squared", 1, 128, 100),
                                           ("dot", 0, 200, 10), ("l2-squared", 0, 1024, 24)])
def test_allow_list_window_matches_oracle(wv, oracle, metric, kind, d, k):
    n = 60000
    rng = np.random.default_rng(7)
    data = gen(oracle, kind, 88, n, d)
    queries = gen(oracle, kind, 89, 40, d)
    idx, orc = build_pair(wv, oracle, metric, "avx256", data)
    dele = np.arange(n // 3 + 100, n // 3 + 300, dtype=np.uint64)  # deleted rows inside a span
    idx.delete(*[int(x) for x in dele])
    orc.delete(dele)
    dset = set(int(x) for x in dele)
    for name, allow in allow_cases(n, rng).items():
        ids, dists, counts = idx.search_by_vector_batch(queries, k, allow=wv.AllowList(allow))
        live = sorted(set(int(x) for x in allow if x < n and int(x) not in dset))
        span = live[-1] + 1 - (live[0] // 256) * 256
        # sparse lists (8 x fewer rows than their span) search a gathered
        # sub-index of their rows; denser ones scan their slot span
        gathered = len(live) * 8 <= span
        assert idx.stats()["last_scan_rows"] == (len(live) if gathered else
                                                 int(allow[allow < n].max()) + 1 - (int(allow[allow < n].min()) // 256) * 256), name
        for q in range(0, len(queries), 3):
            assert_same(orc.search(queries[q], k, allow=allow), ids[q, :counts[q]], dists[q, :counts[q]],
                        f"{name} q{q}")
        idx.set_option("scan_window", 0)  # the whole-corpus scan gives the same rows
        idx.set_option("gather_max", 0)
        ref = idx.search_by_vector_batch(queries, k, allow=wv.AllowList(allow))
        assert idx.stats()["last_scan_rows"] == n
        idx.set_option("scan_window", 1)
        idx.set_option("gather_max", 1 << 20)
        for a, b in zip((ids, dists, counts), ref):
            np.testing.assert_array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
    idx.close()


def test_allow_list_window_bq(wv, oracle):
    n, d, k = 30000, 768, 10
    rng = np.random.default_rng(8)
    data = gen(oracle, 0, 90, n, d)
    queries = gen(oracle, 0, 91, 24, d)
    idx, orc = build_bq_pair(wv, oracle, "cosine", "avx256", data, 50)
    for name, allow in allow_cases(n, rng).items():
        ids, dists, counts = idx.search_by_vector_batch(queries, k, allow=wv.AllowList(allow))
        for q in range(0, len(queries), 4):
            assert_same(orc.search(queries[q], k, allow=allow), ids[q, :counts[q]], dists[q, :counts[q]],
                        f"bq {name} q{q}")
    idx.close()


def test_allow_list_10m_rows_scales_with_span(wv, oracle):
    """10M x 768 cosine (the C3 corpus): a 1 % contiguous allow list (100k ids,
    the scan window) and a 0.01 % one (1k random ids over the whole corpus, the
    gathered sub-index) against the oracle's heap over the allowed rows of the
    regenerated corpus; both run far faster than a whole-corpus scan of the
    same batch."""
    torch = pytest.importorskip("torch")
    n, d, k, B = 10_000_000, 768, 10, 2048
    idx = device_index(wv, torch, "cosine", 0, n, d)
    raw = oracle.gen_matrix(0, 2, 0, B, d)
    rng = np.random.default_rng(9)
    cases = {"1pct": np.arange(4_200_000, 4_300_000, dtype=np.uint64),
             "0.01pct": np.sort(rng.choice(n, 1000, replace=False)).astype(np.uint64)}
    sample = [0, 171, 2047]
    qn = np.stack([oracle.normalize(x) for x in raw[sample]])
    D = oracle.gen_dists(0, 1, n, d, oracle.COSINE, oracle.AVX256, qn, oracle_threads())
    times = {}
    for name, allow in cases.items():
        al = wv.AllowList(allow)
        idx.search_by_vector_batch(raw, k, allow=al)  # warm-up
        t0 = time.perf_counter()
        ids, dists, counts = idx.search_by_vector_batch(raw, k, allow=al)
        times[name] = time.perf_counter() - t0
        for i, q in enumerate(sample):
            oi, od = oracle.heap_scan(D[i][allow.astype(np.int64)], k)
            assert_rows(ids, dists, counts, q, allow[oi.astype(np.int64)], od, name)
    idx.search_by_vector_batch(raw, k)
    t0 = time.perf_counter()
    idx.search_by_vector_batch(raw, k)
    full = time.perf_counter() - t0
    print(f"B={B}: full scan {full*1e3:.1f} ms, 1% span {times['1pct']*1e3:.1f} ms, "
          f"0.01% (1k random ids, gathered) {times['0.01pct']*1e3:.1f} ms")
    assert times["1pct"] < full / 4, (times, full)
    assert times["0.01pct"] < full / 4, (times, full)
    idx.close()
