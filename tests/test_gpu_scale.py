"""GPU parity at the BASELINE configurations' full sizes (BASELINE.json
configs[0..4]): the HIP path against the oracle (oracle/oracle.c restatement,
oracle/scale.c regenerating the synthetic corpus on the fly, so no host copy
of a 30 GB corpus is needed).  Bit-exact ids and distances.

C1 is checked on every query; C2, C3, C4 on sampled queries of the full
batch, C5 (PQ d=960, m=240, ks=256: the LUT-chunk path) on codebook, codes,
ADC distances and searches.  MI355X only (marker gpu).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VARIANTS = {"avx256": 1, "avx512": 2}


def oracle_threads() -> int:
    """The CPU share of this process (cgroup quota), capped at 16."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return max(1, min(16, n))


def assert_rows(ids, dists, counts, q, oi, od, ctx):
    c = counts[q]
    assert c == len(oi), f"{ctx} q{q}: count {c} vs {len(oi)}"
    np.testing.assert_array_equal(ids[q, :c], oi, err_msg=f"{ctx} q{q}: ids")
    np.testing.assert_array_equal(np.asarray(dists[q, :c], np.float32).view(np.uint32),
                                  np.asarray(od, np.float32).view(np.uint32), err_msg=f"{ctx} q{q}: dists")


def device_index(wv, torch, metric, kind, n, d, seed=1, **kw):
    """flat index of rows [0, n) generated on the device (as bench.py builds it)."""
    from weaviate_amd import _lib
    lib = _lib.load()
    idx = wv.FlatIndex(distance=metric, dims=d, variant="avx256", **kw)
    idx.reserve(n)
    chunk = 1_000_000
    stage = torch.empty((min(chunk, n), d), dtype=torch.float32, device="cuda")
    for r0 in range(0, n, chunk):
        m = min(chunk, n - r0)
        _lib.check(lib.wv_gen_device(0, kind, seed, r0, m, d, stage.data_ptr(), None))
        _lib.check(lib.wv_index_add_range_device(idx._h, r0, stage.data_ptr(), m, d))
    torch.cuda.synchronize()
    return idx


def test_c1_full_every_query(wv, oracle):
    """configs[0]: 100k x 128 U(-1,1), l2-squared, k=10, all 1000 queries."""
    n, d, k, nq = 100_000, 128, 10, 1000
    data = oracle.gen_matrix(0, 1, 0, n, d)
    queries = oracle.gen_matrix(0, 2, 0, nq, d)
    idx = wv.FlatIndex(distance="l2-squared", variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    D = oracle.gen_dists(0, 1, n, d, oracle.L2, oracle.AVX256, queries, oracle_threads())
    for q in range(nq):
        oi, od = oracle.heap_scan(D[q], k)
        assert_rows(ids, dists, counts, q, oi, od, "c1")
    idx.close()


def test_c2_full_integer_k100(wv, oracle):
    """configs[1]: 1M x 128 integer-valued U{0..127} (exact ties everywhere),
    l2-squared, k=100, the full 10k-query batch; 64 queries checked."""
    torch = pytest.importorskip("torch")
    n, d, k, nq = 1_000_000, 128, 100, 10_000
    idx = device_index(wv, torch, "l2-squared", 1, n, d)
    queries = oracle.gen_matrix(1, 2, 0, nq, d)
    before = idx.stats()["replayed_queries"]
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    replayed = idx.stats()["replayed_queries"] - before
    sample = np.arange(0, nq, nq // 64)[:64]
    D = oracle.gen_dists(1, 1, n, d, oracle.L2, oracle.AVX256, queries[sample], oracle_threads())
    for i, q in enumerate(sample):
        oi, od = oracle.heap_scan(D[i], k)
        assert_rows(ids, dists, counts, q, oi, od, "c2")
    print(f"c2: {replayed} of {nq} queries resolved by the bounded heap replay")
    idx.close()


def test_c3_full_10m_x_768_bench_path(wv, oracle):
    """configs[2] exactly as bench.py times it: 10M x 768 cosine, k=10, one
    batch of B = 8192 queries (32 query groups per block-key launch, the XCD
    order over 32 * nspans workgroups) through wv_index_search_device, default
    kernel choice.  64 sampled queries plus every query the exactness proof
    flagged (those go through the bounded heap replay) against the
    regenerated-corpus oracle, and the block-key error bound
    |A_block - min_block E| <= eps(q) on every block of the sampled queries."""
    torch = pytest.importorskip("torch")
    from weaviate_amd import _lib
    lib = _lib.load()
    n, d, k, B = 10_000_000, 768, 10, 8192
    idx = device_index(wv, torch, "cosine", 0, n, d)
    qd = torch.empty((B, d), dtype=torch.float32, device="cuda")
    _lib.check(lib.wv_gen_device(0, 0, 2, 0, B, d, qd.data_ptr(), None))
    # mode 1 (the shard-candidate form) on the same batch exposes the proof's flags
    fi = torch.empty((B, k + 1), dtype=torch.int64, device="cuda")
    fd = torch.empty((B, k + 1), dtype=torch.float32, device="cuda")
    fn = torch.empty(B, dtype=torch.int32, device="cuda")
    ff = torch.empty(B, dtype=torch.int32, device="cuda")
    _lib.check(lib.wv_index_search_device(idx._h, qd.data_ptr(), B, d, k, 1, fi.data_ptr(), fd.data_ptr(),
                                          fn.data_ptr(), ff.data_ptr(), None))
    flagged = np.nonzero(ff.cpu().numpy())[0]
    oi_d = torch.empty((B, k), dtype=torch.int64, device="cuda")
    od_d = torch.empty((B, k), dtype=torch.float32, device="cuda")
    on_d = torch.empty(B, dtype=torch.int32, device="cuda")
    before = idx.stats()["replayed_queries"]
    _lib.check(lib.wv_index_search_device(idx._h, qd.data_ptr(), B, d, k, 0, oi_d.data_ptr(), od_d.data_ptr(),
                                          on_d.data_ptr(), None, None))
    torch.cuda.synchronize()
    replayed = idx.stats()["replayed_queries"] - before
    assert replayed == len(flagged), (replayed, len(flagged))
    ids = oi_d.cpu().numpy().view(np.uint64)
    dists = od_d.cpu().numpy()
    counts = on_d.cpu().numpy()
    spread = np.arange(0, B, B // 64)[:64]
    sample = np.unique(np.concatenate([spread, flagged]))
    raw = oracle.gen_matrix(0, 2, 0, B, d)[sample]
    qn = np.stack([oracle.normalize(x) for x in raw])
    D = oracle.gen_dists(0, 1, n, d, oracle.COSINE, oracle.AVX256, qn, oracle_threads())
    worst = 0.0
    for i, q in enumerate(sample):
        oi, od = oracle.heap_scan(D[i], k)
        assert_rows(ids, dists, counts, q, oi, od, "c3")
        if q in set(spread.tolist()):
            A, eps = idx.debug_blockkeys(int(q))
            bmin = D[i][: (n // 32) * 32].reshape(-1, 32).min(axis=1).astype(np.float64)
            err = np.abs(A[: bmin.size].astype(np.float64) - bmin)
            worst = max(worst, float(err.max() / eps))
            assert (err <= eps).all(), f"c3 q{q}: block-key error {err.max()} > eps {eps}"
    print(f"c3 B={B}: {len(sample)} queries checked ({len(flagged)} flagged -> replayed); "
          f"max |A_block - min E| / eps = {worst:.4f}")
    idx.close()


def test_c4_bq_shard_6_25m_x_1536(wv, oracle):
    """configs[3] per GPU as bench.py --workload bq times it: one 6.25M x 1536
    BQ shard, hamming R=200 + fp32 rescoring, k=10, a B = 2048 batch (8 query
    groups of 256 in k_bq_blockmin_lds); 24 queries spread over all 8 groups
    against the regenerated-corpus BQ oracle."""
    torch = pytest.importorskip("torch")
    from weaviate_amd import _lib
    lib = _lib.load()
    n, d, k, R, B = 6_250_000, 1536, 10, 200, 2048
    idx = device_index(wv, torch, "cosine", 0, n, d, bq=True, rescore_limit=R)
    qd = torch.empty((B, d), dtype=torch.float32, device="cuda")
    _lib.check(lib.wv_gen_device(0, 0, 2, 0, B, d, qd.data_ptr(), None))
    oi_d = torch.empty((B, k), dtype=torch.int64, device="cuda")
    od_d = torch.empty((B, k), dtype=torch.float32, device="cuda")
    on_d = torch.empty(B, dtype=torch.int32, device="cuda")
    _lib.check(lib.wv_index_search_device(idx._h, qd.data_ptr(), B, d, k, 0, oi_d.data_ptr(), od_d.data_ptr(),
                                          on_d.data_ptr(), None, None))
    torch.cuda.synchronize()
    ids, dists, counts = oi_d.cpu().numpy().view(np.uint64), od_d.cpu().numpy(), on_d.cpu().numpy()
    sample = np.array([g * 256 + o for g in range(8) for o in (0, 131, 255)])
    queries = oracle.gen_matrix(0, 2, 0, B, d)[sample]
    oi, od, on = oracle.bq_search_gen(0, 1, n, d, oracle.COSINE, oracle.AVX256, queries, k, R, oracle_threads())
    for i, q in enumerate(sample):
        assert_rows(ids, dists, counts, q, oi[i, :on[i]], od[i, :on[i]], "c4")
    idx.close()


def test_c5_pq_full_10m_x_960_bench_batch(wv, oracle):
    """configs[4] as bench.py --workload pq times it: 10M x 960 U[0,1) rows,
    PQ m=240 x ks=256 trained on the first 100k rows, ADC flat search of a
    B = 256 batch through the default minima-only search (k_pq_adc2 block
    minima -> candidate blocks -> k_pq_cand, flagged queries replayed), and a
    1024 batch both that way and through the full-matrix form (pq_cand = 0),
    which at 10M rows splits the batch into query groups sized to the free HBM
    and replays group i on the aux stream beside group i+1's k_pq_adc2.
    Codes of sampled rows against the oracle encoder, then 8 queries per run
    (spread over the groups) against the oracle's flatSearch over the index's
    full code array."""
    torch = pytest.importorskip("torch")
    from concurrent.futures import ThreadPoolExecutor
    from weaviate_amd import _lib
    lib = _lib.load()
    n, d, m, ks, limit, k, B = 10_000_000, 960, 240, 256, 100_000, 10, 256
    idx = device_index(wv, torch, "l2-squared", 2, n, d,
                       pq={"segments": m, "centroids": ks, "trainingLimit": limit, "rescore": False})
    idx.pq_fit(seed=1)
    centers = idx.pq_centers()
    codes = idx.pq_codes(n)
    rows = np.arange(0, n, n // 64)[:64]
    data_rows = np.concatenate([oracle.gen_matrix(2, 1, int(r), 1, d) for r in rows])
    ecodes = np.stack([oracle.pq_encode(centers, x) for x in data_rows])
    np.testing.assert_array_equal(codes[rows], ecodes)
    present = np.ones(n, np.uint8)
    dummy = np.zeros(1, np.float32)
    queries = oracle.gen_matrix(2, 2, 0, 1024, d)
    res = {}
    # the bench's batch and path (the int8 route, cand 2 here), the VALU minima
    # route at B and 1024, and the full-matrix multi-group form
    for cand, nb in ((2, B), (1, B), (1, 1024), (0, 1024)):
        idx.set_option("pq8", 1 if cand == 2 else 0)
        idx.set_option("pq_cand", min(cand, 1))
        qd = torch.empty((nb, d), dtype=torch.float32, device="cuda")
        _lib.check(lib.wv_gen_device(0, 2, 2, 0, nb, d, qd.data_ptr(), None))
        oi_d = torch.empty((nb, k), dtype=torch.int64, device="cuda")
        od_d = torch.empty((nb, k), dtype=torch.float32, device="cuda")
        on_d = torch.empty(nb, dtype=torch.int32, device="cuda")
        _lib.check(lib.wv_index_search_device(idx._h, qd.data_ptr(), nb, d, k, 0, oi_d.data_ptr(), od_d.data_ptr(),
                                              on_d.data_ptr(), None, None))
        torch.cuda.synchronize()
        group = idx.stats()["last_group_queries"]
        if cand == 0:
            assert 0 < group < nb, f"the multi-group path did not run (group of {group} queries)"
        res[cand, nb] = (oi_d.cpu().numpy().view(np.uint64), od_d.cpu().numpy(), on_d.cpu().numpy())
        sample = np.linspace(0, nb - 1, 8).astype(np.int64) + (3 if cand == 0 else 0)
        sample = np.minimum(sample, nb - 1)
        with ThreadPoolExecutor(min(8, oracle_threads())) as ex:
            exp = list(ex.map(lambda q: oracle.pq_flat_search(oracle.L2, 1, centers, codes, dummy, present,
                                                              queries[q], k, k, False), sample))
        for i, q in enumerate(sample):
            assert_rows(*res[cand, nb], q, exp[i][0], exp[i][1], f"c5 cand={cand} B={nb} (groups of {group})")
    # a query's result depends neither on the batch, the group it ran in nor the search form
    for other in ((2, B), (1, 1024), (0, 1024)):
        for a, b in zip(res[1, B], res[other]):
            np.testing.assert_array_equal(np.asarray(a), np.asarray(b)[:B])
    for a, b in zip(res[1, 1024], res[0, 1024]):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b))
    idx.close()


def test_c5_pq_960_m240_ks256(wv, oracle):
    """configs[4] shape: d=960, m=240 segments (ds=4) x 256 centroids, k-means
    on a 100k training sample (trainingLimit 100000 of 120k rows): codebook,
    codes, ADC distances and flat searches (the 32-segment LUT chunks in LDS)."""
    n, d, m, ks, limit, k = 120_000, 960, 240, 256, 100_000, 10
    data = oracle.gen_matrix(2, 1, 0, n, d)
    idx = wv.FlatIndex(distance="l2-squared", variant="avx256",
                       pq={"segments": m, "centroids": ks, "trainingLimit": limit, "rescore": False})
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    idx.pq_fit(seed=7)
    got = idx.pq_centers()
    exp = oracle.pq_fit(data[:limit], m, ks, seed=7, variant=oracle.AVX256, nthreads=oracle_threads())
    np.testing.assert_array_equal(got.view(np.uint32), exp.view(np.uint32))
    codes = idx.pq_codes(n)
    sample = np.arange(0, n, 97)
    ecodes = np.stack([oracle.pq_encode(exp, data[i]) for i in sample])
    np.testing.assert_array_equal(codes[sample], ecodes)
    queries = oracle.gen_matrix(2, 2, 0, 8, d)
    gd = idx.pq_distance(queries[0], codes[:2000])
    ed = np.array([oracle.pq_distance(oracle.L2, exp, queries[0], c) for c in codes[:2000]], np.float32)
    np.testing.assert_array_equal(gd.view(np.uint32), ed.view(np.uint32))
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    present = np.ones(n, np.uint8)
    for q in range(len(queries)):
        oi, od = oracle.pq_flat_search(oracle.L2, 1, exp, codes, data, present, queries[q], k, k, False)
        assert_rows(ids, dists, counts, q, oi, od, "c5")
    idx.close()


@pytest.mark.parametrize("variant", ["avx256", "avx512"])
def test_float_hamming_nan_inf_zero(wv, oracle, variant):
    """hamming_256/512 (distancer/c/hamming_avx{256,512}_amd64.c): SIMD lanes
    compare with _CMP_NEQ_OQ (NaN counts as equal), the scalar tail with !=
    (NaN counts as different); +-0 equal, +-Inf ordinary values.  Special
    values in SIMD and tail positions, both provider and flat search."""
    rng = np.random.default_rng(5)
    specials = np.array([np.nan, 0.0, -0.0, np.inf, -np.inf, 1.0], np.float32)
    for d in [3, 8, 13, 32, 45, 64, 129, 200]:
        a = rng.choice(specials, size=(64, d)).astype(np.float32)
        b = rng.choice(specials, size=(64, d)).astype(np.float32)
        got = wv.single_dist_batch("hamming", a, b, variant=variant)
        exp = np.array([oracle.single_dist(oracle.HAMMING, VARIANTS[variant], a[i], b[i]) for i in range(64)],
                       np.float32)
        np.testing.assert_array_equal(got.view(np.uint32), exp.view(np.uint32), err_msg=f"d={d}")
    # flat search with the hamming provider (the all-rows exact path)
    n, d, k = 3000, 45, 10
    data = rng.choice(specials, size=(n, d)).astype(np.float32)
    queries = rng.choice(specials, size=(12, d)).astype(np.float32)
    idx = wv.FlatIndex(distance="hamming", variant=variant)
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    orc = oracle.OracleFlat(oracle.HAMMING, VARIANTS[variant], d, n)
    orc.add_batch(np.arange(n), data)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    for q in range(len(queries)):
        rc, oi, od = orc.search(queries[q], k)
        assert_rows(ids, dists, counts, q, oi, od, "hamming")
    idx.close()
