"""CPU: the rotational-quantization oracle (oracle/rq.c: flat's "rq-8" and
"rq-1" modes) against what the reference's own tests assert
(compressionhelpers/fast_rotation_test.go, rotational_quantization_test.go,
binary_rotational_quantization_test.go) and against the reference's compiled
dot_byte_256 kernel (distancer/c/dot_byte_avx256.c).  The Go PCG swap / sign /
rounding streams are restated from the Go standard library and are
parity-unpinned (no Go toolchain here)."""
import ctypes as C

import numpy as np
import pytest


def _recursive_fwht(x, normalize):
    """fast_rotation_test.go:250-261 fastWalshHadamardTransform (normalises at
    the leaves), float32."""
    x = x.astype(np.float32)
    if len(x) == 2:
        a, b = x[0], x[1]
        return np.array([np.float32(normalize) * (a + b), np.float32(normalize) * (a - b)], np.float32)
    m = len(x) // 2
    lo = _recursive_fwht(x[:m], normalize)
    hi = _recursive_fwht(x[m:], normalize)
    return np.concatenate([lo + hi, lo - hi]).astype(np.float32)


@pytest.mark.parametrize("dim,norm", [(64, 0.125), (256, 0.0625)])
def test_fwht_equals_recursive(oracle, dim, norm):  # TestFastWalshHadamardTransform64/256
    rng = np.random.default_rng(7212334)
    for _ in range(200):
        x = np.where(rng.random(dim) < 0.5, -1.0, 1.0).astype(np.float32)
        want = _recursive_fwht(x, norm)
        got = x.copy()
        (oracle.lib().or_fwht64 if dim == 64 else oracle.lib().or_fwht256)(oracle.f(got))
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("d", [1, 2, 63, 64, 65, 128, 200, 256, 300, 768, 960, 1536])
def test_output_length_and_swaps(oracle, d):  # TestFastRotationOutputLength, randomSwaps (fast_rotation.go:46-70)
    r = oracle.RQ(8, oracle.DOT, d)
    assert r.D % 64 == 0 and r.D >= d and r.D - d < 64
    sI, sJ, sg, _ = r.tables()
    for rd in range(3):
        both = np.concatenate([sI[rd], sJ[rd]])
        assert sorted(both.tolist()) == list(range(r.D))  # every entry swapped exactly once
        assert np.all(sI[rd] < sJ[rd]) and np.all(np.diff(sI[rd].astype(int)) > 0)  # sorted by I
        assert set(np.unique(sg[rd]).tolist()) <= {-1.0, 1.0}


def test_brq_pads_to_256_and_rounding_range(oracle):  # binary_rotational_quantization.go:40-58
    r = oracle.RQ(1, oracle.COSINE, 100)
    assert r.D == 256
    _, _, _, rd = r.tables()
    assert np.all(rd >= 0) and np.all(rd < 1) and len(np.unique(rd)) > 200


@pytest.mark.parametrize("d", [96, 128, 768, 1000])
def test_rotation_preserves_norm_and_distance(oracle, d):  # TestFastRotationPreservesNorm / Distance
    rng = np.random.default_rng(d)
    r = oracle.RQ(8, oracle.L2, d)
    for _ in range(20):
        x = rng.standard_normal(d).astype(np.float32)
        y = rng.standard_normal(d).astype(np.float32)
        rx, ry = r.rotate(x), r.rotate(y)
        assert abs(np.linalg.norm(rx) - np.linalg.norm(x)) < 1e-4 * np.linalg.norm(x)
        assert abs(np.linalg.norm(rx - ry) - np.linalg.norm(x - y)) < 1e-4 * np.linalg.norm(x - y)


def test_rq8_encode_restore(oracle):  # TestRQEncodeRestore
    rng = np.random.default_rng(7542)
    for _ in range(10):
        d = 2 + int(rng.integers(1000))
        r = oracle.RQ(8, oracle.L2, d, seed=int(rng.integers(1 << 63)))
        s = 1000 * rng.random()
        x = ((2 * rng.random(d) - 1) * s).astype(np.float32)
        c = r.encode(x)
        lower = np.frombuffer(c[0:4][::-1].tobytes(), np.float32)[0]
        step = np.frombuffer(c[4:8][::-1].tobytes(), np.float32)[0]
        restored = lower + step * c[16:].astype(np.float32)
        eps = 0.1 * s * np.sqrt(d) / 128
        assert np.max(np.abs(r.rotate(x) - restored)) < eps


def test_rq8_handles_abnormal_vectors(oracle):  # TestRQHandlesAbnormalVectorsGracefully
    r = oracle.RQ(8, oracle.DOT, 97)
    zero = np.zeros(16 + r.D, np.uint8)
    for n in (0, 15, 572):
        np.testing.assert_array_equal(r.encode(np.zeros(n, np.float32)), zero)
    x = np.arange(243, dtype=np.float32)
    np.testing.assert_array_equal(r.encode(x[: r.D]), r.encode(x))


@pytest.mark.parametrize("metric", ["cosine", "dot", "l2"])
def test_rq8_distance_estimate(oracle, metric):  # TestRQDistanceEstimate (dim 2, seed 42, eps 1e-3)
    m = {"cosine": oracle.COSINE, "dot": oracle.DOT, "l2": oracle.L2}[metric]
    a = np.float32(1.0 / np.sqrt(2.0))
    q = np.array([1.0, 0.0], np.float32)
    x = np.array([a, a], np.float32)
    r = oracle.RQ(8, m, 2, seed=42)
    est = r.distance(r.encode(x), r.encode(q))
    target = oracle.single_dist(m, oracle.AVX256, q, x)
    assert abs(est - target) < 1e-3


def test_rq8_byte_dot_matches_reference_kernel(oracle):
    """dotByteImpl (compressionhelpers/distance_amd64.go:22 -> dot_byte_256)
    against the reference's compiled kernel: the rq-8 estimator's integer part."""
    ref = oracle.ref_lib()
    if ref is None or not hasattr(ref, "dot_byte_256"):
        pytest.skip("reference kernels not built")
    fn = ref.dot_byte_256
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(3)
    for n in (1, 7, 31, 32, 33, 64, 127, 768, 960, 1536):
        a = rng.integers(0, 256, n).astype(np.uint8)
        b = rng.integers(0, 256, n).astype(np.uint8)
        res = C.c_uint32(0)
        ln = C.c_long(n)
        fn(a.ctypes.data, b.ctypes.data, C.addressof(res), C.addressof(ln))
        assert res.value == int(np.dot(a.astype(np.uint64), b.astype(np.uint64)))


@pytest.mark.parametrize("metric", ["cosine", "dot", "l2"])
def test_rq8_estimates_concentrate(oracle, metric):  # TestRQDistancerRandomVectorsWithScaling (loose form)
    m = {"cosine": oracle.COSINE, "dot": oracle.DOT, "l2": oracle.L2}[metric]
    rng = np.random.default_rng(11)
    d = 256
    r = oracle.RQ(8, m, d)
    for _ in range(50):
        q = rng.standard_normal(d).astype(np.float32)
        x = rng.standard_normal(d).astype(np.float32)
        q /= np.linalg.norm(q)
        x /= np.linalg.norm(x)
        est = r.distance(r.encode(x), r.encode(q))
        target = oracle.single_dist(m, oracle.AVX256, q, x)
        assert abs(est - target) < 0.02


@pytest.mark.parametrize("metric", ["cosine", "dot", "l2"])
def test_brq_distance_estimates(oracle, metric):  # TestBRQDistanceEstimates (unit vectors, loose bound)
    m = {"cosine": oracle.COSINE, "dot": oracle.DOT, "l2": oracle.L2}[metric]
    rng = np.random.default_rng(5)
    d = 768
    r = oracle.RQ(1, m, d)
    errs = []
    for _ in range(100):
        q = rng.standard_normal(d).astype(np.float32)
        x = rng.standard_normal(d).astype(np.float32)
        q /= np.linalg.norm(q)
        x = x / np.linalg.norm(x) + 0.5 * q
        est = r.distance(r.encode(x), r.encode_query(q))
        target = oracle.single_dist(m, oracle.AVX256, q, x)
        errs.append(est - target)
    errs = np.array(errs)
    assert abs(errs.mean()) < 0.02 and np.abs(errs).max() < 0.2


def test_brq_zero_query_and_zero_code(oracle):  # encodeQuery abs == 0 -> RQMultiBitCode{}; Encode l1 == 0
    r = oracle.RQ(1, oracle.L2, 300)
    st, sq, dim, planes = r.encode_query(np.zeros(300, np.float32))
    assert (st, sq, dim) == (0.0, 0.0, 0) and not planes.any()
    np.testing.assert_array_equal(r.encode(np.zeros(300, np.float32)), np.zeros(1 + r.W, np.uint64))
    x = np.ones(300, np.float32)
    c = r.encode(x)
    sqn = np.frombuffer(np.uint32(int(c[0]) >> 32).tobytes(), np.float32)[0]
    # zero query: distance = l2 * (|x|^2 + 0) + cos - 0
    assert r.distance(c, (st, sq, dim, planes)) == sqn


def test_rq_flat_search_consistent(oracle):
    """The restated searchByVectorQuantized returns the fp32-rescored top-k of
    the R best quantized candidates: with R >= n it equals the exact search."""
    rng = np.random.default_rng(9)
    n, d, k = 300, 64, 10
    X = rng.standard_normal((n, d)).astype(np.float32)
    for bits in (8, 1):
        idx = oracle.OracleFlatRQ(bits, oracle.COSINE, oracle.AVX256, d, n, rescore_limit=n)
        ex = oracle.OracleFlat(oracle.COSINE, oracle.AVX256, d, n)
        idx.add_batch(range(n), X)
        ex.add_batch(range(n), X)
        for qi in range(5):
            q = rng.standard_normal(d).astype(np.float32)
            rc, ids, dd = idx.search(q, k)
            rc2, ids2, dd2 = ex.search(q, k)
            assert rc == 0 and rc2 == 0
            np.testing.assert_array_equal(ids, ids2)
            np.testing.assert_array_equal(dd, dd2)
