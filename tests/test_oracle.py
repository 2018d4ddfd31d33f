"""CPU: pin the oracle (oracle/oracle.c) against the reference.

* golden vectors produced by the reference's own compiled C kernels
  (tests/golden/distances.npz, tools/make_golden.py);
* live comparison with oracle/_ref/libref.so when it is present;
* known answers from the reference's Go tests (distancer/*_test.go,
  priorityqueue/queue_test.go, binary_quantization_test.go).
"""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")
K2F = {"l2_256": ("or_l2_256",), "l2_512": ("or_l2_512",), "dot_256": ("or_dot_256",), "dot_512": ("or_dot_512",),
       "hamming_256": ("or_hamming_f32",), "hamming_512": ("or_hamming_f32",)}


def bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def test_oracle_matches_reference_golden_distances(oracle):
    g = np.load(os.path.join(GOLD, "distances.npz"))
    a, b, offs = g["a"], g["b"], g["offsets"]
    lib = oracle.lib()
    for kname, (fname,) in K2F.items():
        exp = g[kname]
        got = np.array([getattr(lib, fname)(oracle.f(np.ascontiguousarray(a[offs[i]:offs[i + 1]])),
                                            oracle.f(np.ascontiguousarray(b[offs[i]:offs[i + 1]])),
                                            int(offs[i + 1] - offs[i])) for i in range(len(exp))], np.float32)
        np.testing.assert_array_equal(bits(got), bits(exp), err_msg=kname)
    wa, wb, wo, wout = g["bw_a"], g["bw_b"], g["bw_offsets"], g["bw_out"]
    got = np.array([oracle.hamming_bitwise(wa[wo[i]:wo[i + 1]], wb[wo[i]:wo[i + 1]]) for i in range(len(wout))],
                   np.float32)
    np.testing.assert_array_equal(got, wout)


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(__file__), "..", "oracle", "_ref",
                                                    "libref.so")), reason="reference kernels not built here")
def test_oracle_matches_reference_live(oracle):
    if not oracle.host_has_avx512():
        pytest.skip("host cannot run the AVX-512 reference build")
    rng = np.random.default_rng(7)
    for n in list(range(1, 300)) + [767, 768, 769, 1536]:
        a = (rng.standard_normal(n) * rng.uniform(0.01, 50)).astype(np.float32)
        b = rng.standard_normal(n).astype(np.float32)
        for kname, (fname,) in K2F.items():
            exp = oracle.ref_kernel(kname, a, b)
            got = getattr(oracle.lib(), fname)(oracle.f(a), oracle.f(b), n)
            assert bits(got) == bits(exp), (kname, n)


def test_known_answers(oracle):
    """distancer/{l2,dot_product,cosine_dist,hamming}_test.go"""
    sd = lambda m, a, b: oracle.single_dist(m, 1, np.array(a, np.float32), np.array(b, np.float32))  # noqa: E731
    assert sd(oracle.L2, [3, 4, 5], [3, 4, 5]) == 0
    assert sd(oracle.L2, [3, 4, 5], [1.5, 2, 2.5]) == np.float32(12.5)
    assert sd(oracle.L2, [10, 11], [13, 15]) == 25
    assert sd(oracle.DOT, [3, 4, 5], [3, 4, 5]) == -50
    assert sd(oracle.DOT, [0, 1, 0, 2, 0, 3], [1, 0, 2, 0, 3, 0]) == 0
    assert sd(oracle.DOT, [3, 4, 5], [-3, -4, -5]) == 50
    n = oracle.normalize
    v1 = n(np.array([0.1, 0.3, 0.7], np.float32))
    assert oracle.single_dist(oracle.COSINE, 1, v1, n(np.array([0.1, 0.3, 0.7], np.float32))) == 0
    assert oracle.single_dist(oracle.COSINE, 1, v1, n(np.array([0.2, 0.6, 1.4], np.float32))) == 0
    assert abs(oracle.single_dist(oracle.COSINE, 1, v1, n(np.array([0.2, 0.2, 0.2], np.float32))) - 0.173) < 0.01
    assert abs(oracle.single_dist(oracle.COSINE, 1, v1, n(np.array([-0.1, -0.3, -0.7], np.float32))) - 2) < 0.01
    assert sd(oracle.HAMMING, [3, 4, 5], [3, 4, 5]) == 0
    assert sd(oracle.HAMMING, [3, 4, 5], [1.5, 2, 2.5]) == 3
    assert sd(oracle.HAMMING, [10, 11], [10, 15]) == 1
    assert sd(oracle.HAMMING, [10, 11, 15, 25, 31], [10, 15, 16, 25, 30]) == 3
    # TestNoNegativeDistance (cosine_dist_test.go:100): cosine distance is clamped at 0
    rng = np.random.default_rng(0)
    base = n((rng.random(1536, np.float32) - 0.5))
    for _ in range(20):
        v = n(base + ((rng.random(1536, np.float32) - 0.5) * 1e-5).astype(np.float32))
        assert oracle.single_dist(oracle.COSINE, 1, base, v) >= 0


def test_priority_queue_max_order(oracle):
    """priorityqueue/queue_test.go TestPriorityQueueMax 'insert': pops max first."""
    import ctypes as C
    values = {0: 0.0, 1: 0.23, 2: 0.8, 3: 0.222, 4: 0.88, 5: 1.0}
    for perm_seed in range(5):
        order = np.random.default_rng(perm_seed).permutation(list(values))
        ids = (C.c_uint64 * 8)()
        ds = (C.c_float * 8)()

        class H(C.Structure):
            _fields_ = [("id", C.POINTER(C.c_uint64)), ("dist", C.POINTER(C.c_float)), ("len", C.c_int)]
        h = H(C.cast(ids, C.POINTER(C.c_uint64)), C.cast(ds, C.POINTER(C.c_float)), 0)
        lib = oracle.lib()
        lib.or_heap_insert.argtypes = [C.POINTER(H), C.c_uint64, C.c_float]
        lib.or_heap_pop.argtypes = [C.POINTER(H), C.POINTER(C.c_uint64), C.POINTER(C.c_float)]
        for i in order:
            lib.or_heap_insert(C.byref(h), int(i), values[int(i)])
        out = []
        for _ in range(6):
            a, b = C.c_uint64(), C.c_float()
            lib.or_heap_pop(C.byref(h), C.byref(a), C.byref(b))
            out.append(a.value)
        assert out == [5, 4, 2, 1, 3, 0]


def test_bq_fixed_values_and_bit_order(oracle):
    """binary_quantization_test.go:102-146"""
    g = np.load(os.path.join(GOLD, "bq.npz"))
    for v, bit in zip(g["fixed_in"], g["fixed_bits"]):
        code = oracle.bq_encode(np.array([v], np.float32))
        assert int(code[0] & 1) == int(bit)
    x = (2.0 * np.random.default_rng(42).random(1000, np.float32) - 1.0).astype(np.float32)
    code = oracle.bq_encode(x)
    assert code.size == 16
    for i, v in enumerate(x):
        assert bool((int(code[i // 64]) >> (i % 64)) & 1) == bool(v < 0)
    for i in range(1000, 1024):
        assert not (int(code[i // 64]) >> (i % 64)) & 1


def test_oracle_flat_search_matches_golden(oracle):
    """Restated heap scan with restated kernels == restated heap scan with the
    reference's compiled kernels (tie-heavy integer data)."""
    g = np.load(os.path.join(GOLD, "flat_search.npz"))
    for name in ["l2_int", "dot_int", "cos_u", "l2_dup"]:
        corpus, queries, metric = g[f"{name}_corpus"], g[f"{name}_queries"], int(g[f"{name}_metric"])
        orc = oracle.OracleFlat(metric, oracle.AVX256, corpus.shape[1], corpus.shape[0])
        orc.add_batch(np.arange(corpus.shape[0]), corpus)
        for k in (1, 5, 10, 33):
            ids, dd, cnt = g[f"{name}_k{k}_ids"], g[f"{name}_k{k}_dists"], g[f"{name}_k{k}_counts"]
            for qi in range(len(queries)):
                rc, oi, od = orc.search(queries[qi], k)
                assert rc == 0
                n = int(cnt[qi])
                np.testing.assert_array_equal(oi, ids[qi, :n], err_msg=f"{name} k{k} q{qi}")
                np.testing.assert_array_equal(bits(od), bits(dd[qi, :n]))


def wide_corpus(oracle, g, name):
    """A flat_search_wide.npz corpus: regenerated from its generator parameters
    (tools/make_golden.py flat_search_wide) and checked against its checksum."""
    kind, seed, n, d = (int(x) for x in g[f"{name}_gen"])
    corpus = oracle.gen_matrix(kind, seed, 0, n, d)
    if int(g[f"{name}_dup7"]):
        corpus[1::7] = corpus[0::7][: len(corpus[1::7])]
    assert int(corpus.view(np.uint32).astype(np.uint64).sum()) == int(g[f"{name}_checksum"])
    return corpus


def test_oracle_flat_search_matches_wide_golden(oracle):
    """The same at 512 / 768 / 1024 dims (rows the GPU searches on the int8
    block-key route): restated kernels + heap == the reference's compiled
    kernels + restated heap."""
    g = np.load(os.path.join(GOLD, "flat_search_wide.npz"))
    for name in ["cos_768", "l2_int_512", "dot_1024"]:
        corpus, queries, metric = wide_corpus(oracle, g, name), g[f"{name}_queries"], int(g[f"{name}_metric"])
        orc = oracle.OracleFlat(metric, oracle.AVX256, corpus.shape[1], corpus.shape[0])
        orc.add_batch(np.arange(corpus.shape[0]), corpus)
        for k in (1, 10, 33):
            ids, dd, cnt = g[f"{name}_k{k}_ids"], g[f"{name}_k{k}_dists"], g[f"{name}_k{k}_counts"]
            for qi in range(len(queries)):
                rc, oi, od = orc.search(queries[qi], k)
                assert rc == 0
                n = int(cnt[qi])
                np.testing.assert_array_equal(oi, ids[qi, :n], err_msg=f"{name} k{k} q{qi}")
                np.testing.assert_array_equal(bits(od), bits(dd[qi, :n]))
    # the integer case holds exact ties inside the top 33
    d = g["l2_int_512_k33_dists"]
    assert any(len(np.unique(r)) < len(r) for r in d)


def test_tie_order_is_heap_order_not_sorted(oracle):
    """The reference result is NOT a (dist, id) sort under ties:
    make sure the fixtures exercise that."""
    g = np.load(os.path.join(GOLD, "flat_search.npz"))
    ids, dd = g["l2_dup_k33_ids"], g["l2_dup_k33_dists"]
    differs = 0
    for qi in range(ids.shape[0]):
        order = np.lexsort((ids[qi], dd[qi]))
        differs += int(not np.array_equal(order, np.arange(ids.shape[1])))
    assert differs > 0


def test_search_by_distance_filter(oracle):
    import ctypes as C
    ids = np.arange(10, dtype=np.uint64)
    d = np.array([0.1, 0.2, 0.3, 0.3000005, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9], np.float32)
    oi = np.zeros(10, np.uint64)
    od = np.zeros(10, np.float32)
    n = oracle.lib().or_filter_by_distance(ids.ctypes.data_as(oracle.pu), oracle.f(d), 10, C.c_float(0.3),
                                           oi.ctypes.data_as(oracle.pu), oracle.f(od))
    assert n == 4  # 0.3000005 is within 1e-6 (usecases/floatcomp.InDelta)


def test_generator_is_counter_based(oracle):
    a = oracle.gen_matrix(0, 5, 100, 4, 8)
    b = oracle.gen_matrix(0, 5, 0, 104, 8)[100:]
    np.testing.assert_array_equal(a, b)
    assert a.min() >= -1 and a.max() < 1
    ints = oracle.gen_matrix(1, 5, 0, 100, 8)
    assert np.all(ints == np.round(ints)) and ints.max() <= 127


def test_bq_baseline_matches_oracle_bq(oracle):
    """The threaded BQ CPU baseline (bench cpu_baseline leg) = the BQ oracle,
    with the reference's own hamming_bitwise_256 / dot kernels when built."""
    n, d, k, R = 1500, 130, 10, 40
    data = oracle.gen_matrix(0, 41, 0, n, d)
    queries = oracle.gen_matrix(0, 42, 0, 6, d)
    orc = oracle.OracleFlatBQ(oracle.COSINE, oracle.AVX256, d, n, R)
    orc.add_batch(np.arange(n), data)
    qn = np.stack([oracle.normalize(q) for q in queries])
    uses = [False] + ([True] if oracle.ref_lib() is not None and oracle.host_has_avx512() else [])
    for use_ref in uses:
        ids, dd, cnt = oracle.cpu_baseline_bq(oracle.COSINE, oracle.AVX256, orc.store, orc.codes, qn, k, R, 3, use_ref)
        for q in range(len(queries)):
            rc, oi, od = orc.search(queries[q], k)
            assert rc == 0
            np.testing.assert_array_equal(ids[q, :cnt[q]], oi)
            np.testing.assert_array_equal(dd[q, :cnt[q]].view(np.uint32), od.view(np.uint32))


@pytest.mark.parametrize("bits", [8, 1])
def test_rq_search_gen_matches_oracle_flat_rq(oracle, bits):
    """The bench's full-size rq self-check (or_rq_search_gen: regenerated rows,
    host codes) equals OracleFlatRQ on a stored copy of the same corpus."""
    n, d, k, R = 2500, 136, 10, 40
    data = oracle.gen_matrix(0, 5, 0, n, d)
    qs = oracle.gen_matrix(0, 6, 0, 6, d)
    for metric in (oracle.COSINE, oracle.L2, oracle.DOT):
        ids, dd, cnt = oracle.rq_search_gen(bits, 0, 5, n, d, metric, oracle.AVX256, qs, k, R, 4)
        o = oracle.OracleFlatRQ(bits, metric, oracle.AVX256, d, n, R)
        o.add_batch(np.arange(n, dtype=np.uint64), data)
        for i in range(len(qs)):
            rc, oi, od = o.search(qs[i], k)
            assert rc == 0 and cnt[i] == len(oi)
            np.testing.assert_array_equal(ids[i, :cnt[i]], oi)
            np.testing.assert_array_equal(dd[i, :cnt[i]].view(np.uint32), od.view(np.uint32))
