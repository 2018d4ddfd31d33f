"""CPU: the product-quantizer oracle (oracle/pq.c) against the invariants the
reference's own tests assert (kmeans/kmeans_test.go, kmeans_encoder_test.go,
product_quantization_test.go).  The Go PCG stream itself is parity-unpinned
(no Go toolchain / stdlib here)."""
import numpy as np
import pytest


def test_one_center(oracle):  # kmeans_test.go:269-280 TestOneCenter
    data = np.array([[1, 0], [0, 1], [1, 1], [0, 0]], np.float32)
    c = oracle.pq_fit(data, 1, 1, seed=7)
    np.testing.assert_array_equal(c[0, 0], [0.5, 0.5])


def test_few_data_points_zero_wcss(oracle):  # kmeans_test.go:254-267 TestFewDataPoints
    rng = np.random.default_rng(1)
    data = rng.random((10, 8), dtype=np.float32)
    c = oracle.pq_fit(data, 1, 10, seed=3)[0]
    for x in data:
        assert min(oracle.single_dist(oracle.L2, oracle.AVX256, x, cc) for cc in c) == 0.0


def test_correctness_across_segments(oracle):  # kmeans_test.go:174-205
    data = np.array([[0.99, 0.99, -0.99, 0.99], [1.01, 1.01, -1.01, 1.01],
                     [-0.99, -0.99, 0.99, -0.99], [-1.01, -1.01, 1.01, -1.01]], np.float32)
    c = oracle.pq_fit(data, 2, 2, seed=11)

    def contains(cs, q):
        return any(oracle.single_dist(oracle.L2, oracle.AVX256, x, np.array(q, np.float32)) < 1e-12 for x in cs)
    assert contains(c[0], [1, 1]) and contains(c[0], [-1, -1])
    assert contains(c[1], [-1, 1]) and contains(c[1], [1, -1])


def test_graph_pruning_equals_brute_force(oracle):  # kmeans_test.go:143-160
    rng = np.random.default_rng(2)
    data = rng.standard_normal((1000, 8)).astype(np.float32)
    for seed in (1, 99):
        a = oracle.pq_fit(data, 1, 32, seed=seed)
        b = oracle.pq_fit(data, 1, 32, seed=seed, brute_force=True)
        np.testing.assert_array_equal(a, b)


def test_not_enough_data(oracle):  # kmeans.go:459-461
    with pytest.raises(ValueError):
        oracle.pq_fit(np.zeros((5, 4), np.float32), 1, 8, seed=0)


def test_encoder_encodes_to_nearest_centroid(oracle):  # kmeans_encoder_test.go:26-53
    vectors = np.array([[0, 5], [0.1, 4.9], [0.01, 5.1], [10.1, 7], [5.1, 2], [5.0, 2.1]], np.float32)
    c = oracle.pq_fit(vectors, 1, 3, seed=5)
    for v in vectors:
        code = oracle.pq_encode(c, v)[0]
        best = oracle.single_dist(oracle.L2, oracle.AVX256, v, c[0, code])
        assert all(oracle.single_dist(oracle.L2, oracle.AVX256, v, cc) >= best for cc in c[0])


def test_random_subset_is_a_subset(oracle):  # kmeans.go:238-274: both branches, distinct indices
    for n, k in [(1000, 256), (300, 256), (10, 10), (100000, 256)]:
        s = oracle.random_subset(123, n, k)
        assert len(set(s.tolist())) == k and s.min() >= 0 and s.max() < n
        np.testing.assert_array_equal(s, oracle.random_subset(123, n, k))  # deterministic for a seed


def test_adc_equals_lut_sum_and_wrap(oracle):  # product_quantization.go:85-104, Step/Wrap
    rng = np.random.default_rng(4)
    data = rng.standard_normal((600, 16)).astype(np.float32)
    c = oracle.pq_fit(data, 4, 16, seed=9)
    q = rng.standard_normal(16).astype(np.float32)
    code = oracle.pq_encode(c, data[0])
    for metric in (oracle.L2, oracle.DOT, oracle.COSINE):
        s = np.float32(0)
        for seg in range(4):
            a, b = q[seg * 4:(seg + 1) * 4], c[seg, code[seg]]
            acc = np.float32(0)
            for j in range(4):
                t = (a[j] - b[j]) * (a[j] - b[j]) if metric == oracle.L2 else a[j] * b[j]
                acc = np.float32(acc + np.float32(t))
            s = np.float32(s + acc)
        want = s if metric == oracle.L2 else -s if metric == oracle.DOT else max(np.float32(1) - s, np.float32(0))
        assert oracle.pq_distance(metric, c, q, code) == np.float32(want)


def test_pq_cpu_baseline_equals_oracle_search(oracle):
    rng = np.random.default_rng(6)
    data = rng.random((800, 16), dtype=np.float32)
    c = oracle.pq_fit(data, 4, 16, seed=3)
    codes = np.stack([oracle.pq_encode(c, x) for x in data])
    qs = rng.random((5, 16), dtype=np.float32)
    ids, dd, cnt = oracle.cpu_baseline_pq(oracle.L2, c, codes, qs, 10, 2)
    for i in range(5):
        oi, od = oracle.pq_flat_search(oracle.L2, 1, c, codes, data, np.ones(800, np.uint8), qs[i], 10, 10, False)
        np.testing.assert_array_equal(ids[i, :cnt[i]], oi)
        np.testing.assert_array_equal(dd[i, :cnt[i]], od)
