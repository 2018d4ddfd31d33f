"""GPU parity of the int8 block-key pass (q8_kernels.hip):
k_q8_blockkey feeds the block-key selection / exact pass / replay for
384 < d <= 1536.  Every query bit-exact against the oracle, the same results
as the bf16 keys (option q8 = 0), and the int8 block keys within the proof's
eps of the exact block minima."""
import numpy as np
import pytest

from test_gpu_flat import VARIANTS, assert_same, build_pair, gen

pytestmark = pytest.mark.gpu

ROUTE_INT8, ROUTE_BF16, ROUTE_W4 = 3, 1, 2


def check_block_keys(idx, oracle, kind, seed, n, d, metric, variant, queries, sample, data=None):
    qs = queries[sample]
    if metric == "cosine":
        qs = np.stack([oracle.normalize(x) for x in qs])
    if data is None:
        D = oracle.gen_dists(kind, seed, n, d, oracle.METRIC[metric], VARIANTS[variant], qs, 8)
    else:
        D = np.stack([[oracle.single_dist(oracle.METRIC[metric], VARIANTS[variant], q, x) for x in data] for q in qs])
    worst = 0.0
    for i, q in enumerate(sample):
        A, eps = idx.debug_blockkeys(int(q))
        nb = (n // 32) * 32
        bmin = D[i][:nb].reshape(-1, 32).min(axis=1).astype(np.float64)
        err = np.abs(A[: bmin.size].astype(np.float64) - bmin)
        worst = max(worst, float(err.max() / eps))
        assert (err <= eps).all(), f"q{q}: int8 block-key error {err.max()} > eps {eps}"
    return worst


@pytest.mark.parametrize("metric,kind,variant,n,d,k", [
    ("cosine", 0, "avx256", 30000, 768, 10),     # C3 shape: two blocks per ring slot
    ("l2-squared", 0, "avx256", 20000, 768, 10),
    ("dot", 0, "avx512", 20000, 640, 24),
    ("cosine", 0, "avx256", 20000, 400, 10),     # dpb8 512: zero-padded columns
    ("l2-squared", 1, "avx256", 20000, 512, 100),  # integer data: exact codes, ties -> replay
    ("cosine", 0, "avx512", 16000, 1024, 10),    # one block per slot
    ("l2-squared", 2, "avx256", 12000, 1100, 10),  # dpb8 1280
    ("dot", 0, "avx256", 12000, 1536, 100),
])
def test_q8_keys_match_oracle_and_bf16(wv, oracle, metric, kind, variant, n, d, k):
    data = gen(oracle, kind, 71, n, d)
    queries = gen(oracle, kind, 72, 300, d)
    idx, orc = build_pair(wv, oracle, metric, variant, data)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    assert idx.stats()["last_route"] == ROUTE_INT8
    for qi in range(len(queries)):
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], ctx=f"q{qi}")
    worst = check_block_keys(idx, oracle, kind, 71, n, d, metric, variant, queries, [0, 131, 299])
    print(f"{metric} d={d}: int8 max |A_block - min E| / eps = {worst:.4f}")
    idx.set_option("q8", 0)
    ids2, dists2, counts2 = idx.search_by_vector_batch(queries, k)
    assert idx.stats()["last_route"] in (ROUTE_BF16, ROUTE_W4)
    np.testing.assert_array_equal(counts, counts2)
    np.testing.assert_array_equal(ids, ids2)
    np.testing.assert_array_equal(dists.view(np.uint32), dists2.view(np.uint32))
    idx.close()


def test_q8_upsert_delete_allow_requantises_blocks(wv, oracle):
    """Rows written into existing blocks (upserts with a 50x larger norm,
    sparse ids) re-quantise the whole block (its scale grows); whole deleted
    blocks key +inf; allow lists; every query equals the oracle."""
    n, d, k = 9000, 768, 10
    rng = np.random.default_rng(5)
    data = gen(oracle, 0, 73, n, d)
    ids = np.arange(n, dtype=np.uint64) * 3  # sparse: blocks hold every third id
    idx = wv.FlatIndex(distance="l2-squared", variant="avx256")
    idx.add_batch(ids, data)
    orc = oracle.OracleFlat(oracle.METRIC["l2-squared"], VARIANTS["avx256"], d, int(ids.max()) + 1 + 3000)
    orc.add_batch(ids, data)
    up = rng.choice(n, 200, replace=False)
    newv = (gen(oracle, 0, 74, 200, d) * np.float32(50.0)).astype(np.float32)
    idx.add_batch(ids[up], newv)
    orc.add_batch(ids[up], newv)
    extra = np.arange(int(ids.max()) + 1, int(ids.max()) + 1 + 3000, dtype=np.uint64)[::7]
    ev = gen(oracle, 0, 75, len(extra), d)
    idx.add_batch(extra, ev)
    orc.add_batch(extra, ev)
    dele = ids[(ids >= 3 * 32 * 10) & (ids < 3 * 32 * 14)]  # whole 32-slot blocks
    idx.delete(*[int(x) for x in dele])
    orc.delete([int(x) for x in dele])
    queries = gen(oracle, 0, 76, 120, d)
    queries[:40] = data[up[:40]] * np.float32(50.0)  # near the upserted rows
    got = idx.search_by_vector_batch(queries, k)
    assert idx.stats()["last_route"] == ROUTE_INT8
    for qi in range(len(queries)):
        assert_same(orc.search(queries[qi], k), got[0][qi, :got[2][qi]], got[1][qi, :got[2][qi]], ctx=f"q{qi}")
    allow = wv.AllowList(int(x) for x in ids[::5])
    got = idx.search_by_vector_batch(queries, k, allow=allow)
    for qi in range(0, len(queries), 7):
        assert_same(orc.search(queries[qi], k, allow=set(int(x) for x in ids[::5])), got[0][qi, :got[2][qi]],
                    got[1][qi, :got[2][qi]], ctx=f"allow q{qi}")
    idx.close()


@pytest.mark.parametrize("metric", ["cosine", "l2-squared"])
def test_q8_heavy_tailed_rows_and_forced_replay(wv, oracle, metric):
    """A few huge coordinates per row (int8 scales dominated by outliers: wide
    bound, many candidate blocks, overflow into the second selection pass) and
    every query forced through the keyed replay: still bit-exact."""
    n, d, k = 20000, 512, 10
    rng = np.random.default_rng(6)
    data = gen(oracle, 0, 77, n, d)
    spikes = rng.integers(0, d, size=(n, 2))
    data[np.arange(n)[:, None], spikes] *= np.float32(40.0)
    queries = gen(oracle, 0, 78, 64, d)
    for force in (0, 1):
        idx, orc = build_pair(wv, oracle, metric, "avx256", data)
        idx.set_option("qs_force_flag", force)
        ids, dists, counts = idx.search_by_vector_batch(queries, k)
        assert idx.stats()["last_route"] == ROUTE_INT8
        for qi in range(len(queries)):
            assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], ctx=f"f{force} q{qi}")
        idx.close()


@pytest.mark.parametrize("metric,variant,d,k", [("cosine", "avx256", 768, 10), ("l2-squared", "avx512", 640, 24),
                                               ("dot", "avx256", 1024, 100), ("cosine", "avx256", 1536, 10)])
def test_q8_row_filter_equals_bf16_filter_and_unfiltered(wv, oracle, metric, variant, d, k):
    """The exact pass's row bound from the int8 plane (q8_filter 1, default),
    from the bf16 plane (q8_filter 0) and no row bound (exact_filter 0): the
    same results bit for bit, equal to the oracle."""
    n = 24000
    data = gen(oracle, 0, 79, n, d)
    queries = gen(oracle, 0, 80, 256, d)
    res = []
    for opts in ({}, {"q8_filter": 0}, {"exact_filter": 0}):
        idx, orc = build_pair(wv, oracle, metric, variant, data, options=opts)
        res.append(idx.search_by_vector_batch(queries, k))
        assert idx.stats()["last_route"] == ROUTE_INT8
        idx.close()
    for other in res[1:]:
        for a, b in zip(res[0], other):
            np.testing.assert_array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
    ids, dists, counts = res[0]
    for qi in range(0, len(queries), 16):
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"{metric} q{qi}")


@pytest.mark.parametrize("metric,kind,d,k", [("cosine", 0, 768, 10), ("l2-squared", 1, 512, 100), ("dot", 0, 640, 10)])
@pytest.mark.parametrize("variant_opt", [{"q8_stag": 1}, {"q8_pf": 2}])
def test_q8_staggered_epilogue_same_keys(wv, oracle, metric, kind, d, k, variant_opt):
    """q8_stag 1 (waves 4-7 reduce each block late) and q8_pf 2 (fragment reads
    two chunks ahead) write the same block keys as the default schedule:
    identical results and block keys, both equal to the oracle; corpus sizes
    that end mid-slot and mid-span."""
    n = 20000 + 37
    data = gen(oracle, kind, 81, n, d)
    queries = gen(oracle, kind, 82, 300, d)
    res, keys = [], []
    for opt in ({}, variant_opt):
        idx, orc = build_pair(wv, oracle, metric, "avx256", data, options=opt)
        res.append(idx.search_by_vector_batch(queries, k))
        assert idx.stats()["last_route"] == ROUTE_INT8
        keys.append([idx.debug_blockkeys(q)[0] for q in (0, 255, 299)])
        idx.close()
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
    for a, b in zip(keys[0], keys[1]):
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    ids, dists, counts = res[1]
    for qi in range(0, len(queries), 10):
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"{metric} q{qi}")


@pytest.mark.parametrize("metric,kind,d,k", [("cosine", 0, 768, 10), ("l2-squared", 1, 512, 100), ("dot", 0, 640, 10)])
@pytest.mark.parametrize("nq", [40, 64, 100, 300])
def test_q8_live_padding_waves_same_keys(wv, oracle, metric, kind, d, k, nq):
    """q8_live (default 1): in a batch that is not a multiple of 256 queries the
    waves holding only padding queries skip their MFMAs; every real query's
    keys and results equal the full schedule's (q8_live 0) and the oracle."""
    n = 20000 + 37
    data = gen(oracle, kind, 83, n, d)
    queries = gen(oracle, kind, 84, nq, d)
    res, keys = [], []
    probe = sorted({0, 31, 32, nq - 1})
    for opt in ({"q8_live": 0, "q8_gemv": 0}, {"q8_live": 1, "q8_gemv": 0}):
        idx, orc = build_pair(wv, oracle, metric, "avx256", data, options=opt)
        res.append(idx.search_by_vector_batch(queries, k))
        assert idx.stats()["last_route"] == ROUTE_INT8
        keys.append([idx.debug_blockkeys(q)[0] for q in probe])
        idx.close()
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
    for a, b in zip(keys[0], keys[1]):
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    ids, dists, counts = res[1]
    for qi in range(0, nq, 7):
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"{metric} q{qi}")


def test_q8_prio_same_keys(wv, oracle):
    """q8_prio 1 (waves 4-7 at s_setprio 1) changes the issue order only."""
    n, d, k = 20000 + 37, 768, 10
    data = gen(oracle, 0, 85, n, d)
    queries = gen(oracle, 0, 86, 512, d)
    res = []
    for opt in ({"q8_prio": 0}, {"q8_prio": 1}):
        idx, orc = build_pair(wv, oracle, "cosine", "avx256", data, options=opt)
        res.append(idx.search_by_vector_batch(queries, k) + (idx.debug_blockkeys(300)[0],))
        idx.close()
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))


# ---------------------------------------------------------------------------
# BQ block minima on the integer matrix cores (k_q8_blockkey<..., BQ> over
# +-1 code planes): hamming = (64 words - sum s_q s_x) / 2, exact
# ---------------------------------------------------------------------------
ROUTE_BQ_INT8, ROUTE_BQ_VALU = 6, 7


@pytest.mark.parametrize("metric,kind,n,d,k,rescore", [
    ("cosine", 0, 20000, 1536, 10, 200),   # C4 width: 24 words, one block per ring slot
    ("l2-squared", 0, 9000, 1000, 10, 64),  # 16 words, zero-padded columns 1024..
    ("dot", 0, 12000, 768, 5, 37),         # 12 words, two blocks per slot
    ("cosine", 1, 6000, 450, 10, 50),      # 8 words; all-positive data: every code 0, ties everywhere
    ("l2-squared", 2, 5000 + 77, 1100, 20, 20),  # 18 words, ragged corpus
])
def test_bq_int8_minima_equal_valu_and_oracle(wv, oracle, metric, kind, n, d, k, rescore):
    from test_gpu_flat import build_bq_pair
    data = gen(oracle, kind, 83, n, d)
    queries = gen(oracle, kind, 84, 300, d)
    idx, orc = build_bq_pair(wv, oracle, metric, "avx256", data, rescore)
    got = idx.search_by_vector_batch(queries, k)
    assert idx.stats()["last_route"] == ROUTE_BQ_INT8
    mins = [idx.debug_bqmin(q) for q in (0, 150, 299)]
    idx.set_option("bq8", 0)
    ref = idx.search_by_vector_batch(queries, k)
    assert idx.stats()["last_route"] == ROUTE_BQ_VALU
    for q, m in zip((0, 150, 299), mins):
        v = idx.debug_bqmin(q)
        np.testing.assert_array_equal(m[: v.size], v, err_msg=f"block minima q{q}")
        assert np.all(np.isinf(m[v.size:]))
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
    for q in range(0, len(queries), 12):
        assert_same(orc.search(queries[q], k), got[0][q, :got[2][q]], got[1][q, :got[2][q]], f"bq {metric} q{q}")
    idx.close()


def test_bq_int8_deletes_allow_upserts(wv, oracle):
    """Deleted rows, whole deleted 256-row blocks, upserts and allow lists: the
    +-1 plane follows the codes, the minima equal the VALU kernel's."""
    from test_gpu_flat import build_bq_pair
    n, d, k = 9000, 768, 10
    data = gen(oracle, 0, 85, n, d)
    idx, orc = build_bq_pair(wv, oracle, "cosine", "avx512", data, 64)
    dele = np.concatenate([np.arange(0, n, 7), np.arange(512, 1024)]).astype(np.uint64)
    idx.delete(*dele)
    orc.delete(dele)
    up = gen(oracle, 0, 86, 300, d)
    upids = np.arange(2000, 2300, dtype=np.uint64)
    idx.add_batch(upids, up)
    orc.add_batch(upids, up)
    queries = gen(oracle, 0, 87, 64, d)
    allow = np.arange(50, 7000, 3, dtype=np.uint64)
    for al in (None, wv.AllowList(allow)):
        got = idx.search_by_vector_batch(queries, k, allow=al)
        assert idx.stats()["last_route"] == ROUTE_BQ_INT8
        m0 = idx.debug_bqmin(5)
        idx.set_option("bq8", 0)
        ref = idx.search_by_vector_batch(queries, k, allow=al)
        v = idx.debug_bqmin(5)
        np.testing.assert_array_equal(m0[: v.size], v)
        idx.set_option("bq8", 1)
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
        for q in range(0, len(queries), 8):
            exp = orc.search(queries[q], k, allow=allow if al is not None else None)
            assert_same(exp, got[0][q, :got[2][q]], got[1][q, :got[2][q]], f"q{q}")
    idx.close()


@pytest.mark.parametrize("metric,kind,d,k", [("cosine", 0, 768, 10), ("l2-squared", 1, 512, 100), ("dot", 0, 640, 10),
                                           ("cosine", 0, 1024, 10), ("l2-squared", 0, 1536, 24)])
def test_q8_shape32_same_keys(wv, oracle, metric, kind, d, k):
    """q8_shape 32 (v_mfma_i32_32x32x32_i8, one query per lane in the block
    reduction) writes bit-identical block keys to the 16x16x64 kernel (the
    per-row values and the scale are the same; maxima commute with the
    monotone rounding), and the same results; corpus sizes end mid-slot."""
    n = 16000 + 45
    data = gen(oracle, kind, 92, n, d)
    queries = gen(oracle, kind, 93, 300, d)
    res, keys = [], []
    for shape in (16, 32):
        idx, orc = build_pair(wv, oracle, metric, "avx256", data, options={"q8_shape": shape})
        res.append(idx.search_by_vector_batch(queries, k))
        assert idx.stats()["last_route"] == ROUTE_INT8
        keys.append([idx.debug_blockkeys(q)[0] for q in (0, 255, 299)])
        idx.close()
    for a, b in zip(keys[0], keys[1]):
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
    ids, dists, counts = res[1]
    for qi in range(0, len(queries), 10):
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], f"{metric} q{qi}")


@pytest.mark.parametrize("metric,kind,variant,n,d,k", [
    ("cosine", 0, "avx256", 12000, 2048, 10),     # dpb8 2048: two column parts of 16 chunks
    ("l2-squared", 0, "avx512", 10000, 2048, 100),
    ("dot", 0, "avx256", 9000, 2500, 10),          # dpb8 2560 (parts of 20), zero-padded columns
    ("cosine", 0, "avx256", 8000, 3072, 10),       # dpb8 3072 (parts of 24)
    ("l2-squared", 1, "avx256", 8000, 3072, 24),   # integer data: ties -> replay without a bf16 plane
    ("cosine", 2, "avx512", 6000, 1600, 100),      # just above the bf16 planes' 1536
])
def test_q8_only_planes_above_1536_dims(wv, oracle, metric, kind, variant, n, d, k):
    """1536 < d <= 3072: int8 block-key planes without a bf16 plane
    (k_q8_blockkey_cp, 128-query groups, two column parts per block), the int8
    row filter in the exact pass, the unfiltered bounded replay.  Every query
    bit-exact against the oracle; block keys within eps; with deletes and an
    allow list too."""
    data = gen(oracle, kind, 171, n, d)
    queries = gen(oracle, kind, 172, 300, d)
    idx, orc = build_pair(wv, oracle, metric, variant, data)
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    assert idx.stats()["last_route"] == ROUTE_INT8
    for qi in range(len(queries)):
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], ctx=f"q{qi}")
    worst = check_block_keys(idx, oracle, kind, 171, n, d, metric, variant, queries, [0, 131, 299])
    print(f"{metric} d={d}: int8-only max |A_block - min E| / eps = {worst:.4f}")
    dele = list(range(5, n, 11)) + list(range(64, 160))  # scattered rows and whole blocks
    idx.delete(*dele)
    orc.delete(dele)
    allow = list(range(1, n, 3))
    ids, dists, counts = idx.search_by_vector_batch(queries[:64], k)
    ida, da, ca = idx.search_by_vector_batch(queries[:64], k, allow=wv.AllowList(allow))
    assert idx.stats()["last_route"] == ROUTE_INT8
    for qi in range(64):
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], ctx=f"d{qi}")
        assert_same(orc.search(queries[qi], k, allow=allow), ida[qi, :ca[qi]], da[qi, :ca[qi]], ctx=f"a{qi}")
    idx.close()


def test_q8_only_nonfinite_row_leaves_block_keys(wv, oracle):
    """A stored NaN above 1536 dims (no bf16 plane to flag it) sends the index
    to the all-rows path, which keeps the reference's NaN semantics."""
    n, d, k = 3000, 2048, 10
    data = gen(oracle, 0, 181, n, d)
    queries = gen(oracle, 0, 182, 20, d)
    idx, orc = build_pair(wv, oracle, "l2-squared", "avx256", data)
    idx.search_by_vector_batch(queries, k)
    assert idx.stats()["last_route"] == ROUTE_INT8
    bad = data[7].copy()
    bad[100] = np.nan
    idx.add_batch(np.array([n], dtype=np.uint64), bad[None, :])
    orc2 = oracle.OracleFlat(oracle.METRIC["l2-squared"], VARIANTS["avx256"], d, n + 1)
    orc2.add_batch(np.arange(n, dtype=np.uint64), data)
    orc2.add_batch(np.array([n], dtype=np.uint64), bad[None, :])
    ids, dists, counts = idx.search_by_vector_batch(queries, k)
    assert idx.stats()["last_route"] != ROUTE_INT8
    for qi in range(len(queries)):
        assert_same(orc2.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], ctx=f"n{qi}")
    idx.close()


@pytest.mark.parametrize("metric,kind,variant,n,d,k", [
    ("cosine", 0, "avx256", 30000, 768, 10),
    ("l2-squared", 0, "avx256", 20000, 400, 10),    # dpb8 512: zero-padded columns
    ("dot", 0, "avx512", 12000, 1024, 24),
    ("l2-squared", 1, "avx256", 20000, 512, 100),   # integer data: ties -> replay
    ("cosine", 0, "avx256", 9000, 1536, 10),        # NC 24: one query group per wave
])
@pytest.mark.parametrize("nq", [1, 7, 16, 17, 32])
def test_q8_gemv_small_batches_match_blockkey(wv, oracle, metric, kind, variant, n, d, k, nq):
    """Batches of <= 32 queries take k_q8_gemv (the int8 plane streamed through
    registers, no 256-query padding): the block keys must be bit-identical to
    k_q8_blockkey's, the results equal to the oracle's, with deletions and an
    allow list."""
    data = gen(oracle, kind, 191, n, d)
    queries = gen(oracle, kind, 192, nq, d)
    idx, orc = build_pair(wv, oracle, metric, variant, data)
    gone = list(range(11, n, 37))
    idx.delete(*gone)
    orc.delete(gone)
    res, keys = {}, {}
    for g in (1, 0):
        idx.set_option("q8_gemv", g)
        res[g] = idx.search_by_vector_batch(queries, k)
        dpb8 = -(-d // 128) * 128 if d <= 768 else -(-d // 256) * 256
        gemv = g and (nq <= 16 or dpb8 <= 1024)  # two query groups per wave need NC <= 16
        assert idx.stats()["last_route"] == (9 if gemv else ROUTE_INT8)
        keys[g] = [idx.debug_blockkeys(q)[0] for q in range(nq)]
    for q in range(nq):
        np.testing.assert_array_equal(keys[1][q].view(np.uint32), keys[0][q].view(np.uint32), err_msg=f"keys q{q}")
    for a, b in zip(res[1], res[0]):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b))
    ids, dists, counts = res[1]
    for qi in range(nq):
        assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]], ctx=f"q{qi}")
    idx.set_option("q8_gemv", 1)
    allow = list(range(3, n, 5))
    ids, dists, counts = idx.search_by_vector_batch(queries, k, allow=wv.AllowList(allow))
    for qi in range(nq):
        assert_same(orc.search(queries[qi], k, allow=allow), ids[qi, :counts[qi]], dists[qi, :counts[qi]],
                    ctx=f"a{qi}")
    idx.close()


@pytest.mark.parametrize("metric,kind,n,d,k,rescore", [
    ("cosine", 0, 30000, 1536, 10, 200),   # C4 width: most queries answered without the replay
    ("dot", 0, 12000, 768, 64, 100),       # k at the fast path's cap
    ("l2-squared", 2, 9000 + 5, 1000, 10, 40),  # ragged corpus
    ("cosine", 1, 6000, 450, 10, 50),      # every code 0: one hamming value, the replay decides
    ("l2-squared", 3, 8000, 512, 10, 30),  # small-integer data: exact-distance ties
])
def test_bq_fast_equals_replay_and_oracle(wv, oracle, metric, kind, n, d, k, rescore):
    """k_bq_fast: queries whose rescored result no hamming tie
    can change skip the R-heap replay.  Results with the fast path on equal
    the replay-only results bit for bit and the oracle (flat/index.go:460-532),
    also under an allow list."""
    from test_gpu_flat import build_bq_pair
    if kind == 3:  # signed small integers: codes vary, exact distances tie
        data = gen(oracle, 1, 85, n, d) - np.float32(64)
        queries = gen(oracle, 1, 86, 160, d) - np.float32(64)
    else:
        data = gen(oracle, kind, 85, n, d)
        queries = gen(oracle, kind, 86, 160, d)
    idx, orc = build_bq_pair(wv, oracle, metric, "avx256", data, rescore)
    allow = wv.AllowList(range(0, n, 3))
    for al in (None, allow):
        idx.set_option("bq_fast", 1)
        got = idx.search_by_vector_batch(queries, k, allow=al)
        assert idx.stats()["last_route"] == ROUTE_BQ_INT8
        idx.set_option("bq_fast", 0)
        ref = idx.search_by_vector_batch(queries, k, allow=al)
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
        if al is None:
            for q in range(0, len(queries), 10):
                assert_same(orc.search(queries[q], k), got[0][q, :got[2][q]], got[1][q, :got[2][q]],
                            f"bq fast {metric} q{q}")
    idx.close()
