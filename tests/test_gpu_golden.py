"""The HIP path against the reference-scored fixtures directly (no oracle in
the loop): tests/golden/distances.npz holds the outputs of the reference's
own amd64 C kernels (l2_256/512, dot_256/512, hamming_256/512,
hamming_bitwise; tools/make_golden.py), tests/golden/flat_search.npz the
searchByVector results over reference-kernel-scored corpora, including the
heap-order tie fixtures (flat/index.go:423-448, priorityqueue/queue.go).

Provider mapping (distancer/*.go): l2-squared = l2 kernel; dot = -dot kernel;
cosine-dot = max(0, 1 - dot kernel); hamming = the float hamming kernel.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
# fixture metric ints (wv_knn.h WV_METRIC_*: 0 l2, 1 dot, 2 cosine) -> Provider names
METRIC_NAME = {0: "l2-squared", 1: "dot", 2: "cosine"}


def bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


@pytest.mark.parametrize("variant", ["avx256", "avx512"])
def test_distance_batch_matches_reference_kernels(wv, variant):
    g = np.load(os.path.join(GOLD, "distances.npz"))
    a, b, offs = g["a"], g["b"], g["offsets"]
    suffix = "256" if variant == "avx256" else "512"
    l2, dot, ham = g["l2_" + suffix], g["dot_" + suffix], g["hamming_" + suffix]
    one = np.float32(1.0)
    for i in range(len(l2)):
        x = a[offs[i]:offs[i + 1]][None, :]
        y = b[offs[i]:offs[i + 1]][None, :]
        got = {m: wv.single_dist_batch(m, x, y, variant=variant)[0] for m in ("l2-squared", "dot", "cosine", "hamming")}
        cos = one - dot[i]
        exp = {"l2-squared": l2[i], "dot": -dot[i], "cosine": np.float32(0.0) if cos < 0 else cos, "hamming": ham[i]}
        for m in got:
            assert bits(got[m]) == bits(exp[m]), (m, variant, i, int(offs[i + 1] - offs[i]), got[m], exp[m])


def test_hamming_bitwise_matches_reference_kernel(wv):
    g = np.load(os.path.join(GOLD, "distances.npz"))
    wa, wb, wo, wout = g["bw_a"], g["bw_b"], g["bw_offsets"], g["bw_out"]
    for i in range(len(wout)):
        got = wv.hamming_bitwise_batch(wa[wo[i]:wo[i + 1]][None, :], wb[wo[i]:wo[i + 1]][None, :])
        assert got[0] == wout[i], (i, got[0], wout[i])


@pytest.mark.parametrize("name", ["l2_int", "dot_int", "cos_u", "l2_dup"])
@pytest.mark.parametrize("batched", [True, False])
def test_flat_search_matches_reference_fixtures(wv, name, batched):
    """Every id, every distance bit and the heap's tie order, per k."""
    g = np.load(os.path.join(GOLD, "flat_search.npz"))
    corpus, queries = g[f"{name}_corpus"], g[f"{name}_queries"]
    metric = METRIC_NAME[int(g[f"{name}_metric"])]
    idx = wv.FlatIndex(distance=metric, variant="avx256", dims=0)
    idx.add_batch(np.arange(corpus.shape[0], dtype=np.uint64), corpus)
    try:
        for k in (1, 5, 10, 33):
            ids, dd, cnt = g[f"{name}_k{k}_ids"], g[f"{name}_k{k}_dists"], g[f"{name}_k{k}_counts"]
            if batched:
                gi, gd, gc = idx.search_by_vector_batch(queries, k)
            for qi in range(len(queries)):
                if batched:
                    oi, od = gi[qi, :gc[qi]], gd[qi, :gc[qi]]
                else:
                    oi, od = idx.search_by_vector(queries[qi], k)
                n = int(cnt[qi])
                assert len(oi) == n, (name, k, qi)
                np.testing.assert_array_equal(np.asarray(oi, np.uint64), ids[qi, :n], err_msg=f"{name} k{k} q{qi}")
                np.testing.assert_array_equal(bits(od), bits(dd[qi, :n]), err_msg=f"{name} k{k} q{qi}")
    finally:
        idx.close()


@pytest.mark.parametrize("name", ["cos_768", "l2_int_512", "dot_1024"])
def test_flat_search_matches_wide_reference_fixtures(wv, oracle, name):
    """Reference-kernel-scored fixtures at 512 / 768 / 1024 dims: the search
    runs on the int8 block-key route (k_q8_blockkey keys, int8 row filter,
    reference-order exact pass) and must return every id, distance bit and
    tie position of the fixture (tools/make_golden.py flat_search_wide)."""
    from test_oracle import wide_corpus
    g = np.load(os.path.join(GOLD, "flat_search_wide.npz"))
    corpus, queries = wide_corpus(oracle, g, name), g[f"{name}_queries"]
    metric = METRIC_NAME[int(g[f"{name}_metric"])]
    idx = wv.FlatIndex(distance=metric, variant="avx256", dims=0)
    idx.add_batch(np.arange(corpus.shape[0], dtype=np.uint64), corpus)
    try:
        # both int8 key routes: the small-batch streaming kernel (k_q8_gemv,
        # route 9, the default at this batch size) and k_q8_blockkey (route 3)
        for gemv, routes in ((1, (9, 3)), (0, (3,))):
          idx.set_option("q8_gemv", gemv)
          for k in (1, 10, 33):
            ids, dd, cnt = g[f"{name}_k{k}_ids"], g[f"{name}_k{k}_dists"], g[f"{name}_k{k}_counts"]
            gi, gd, gc = idx.search_by_vector_batch(queries, k)
            assert idx.stats()["last_route"] in routes, (gemv, k)
            for qi in range(len(queries)):
                n = int(cnt[qi])
                assert gc[qi] == n, (name, k, qi)
                np.testing.assert_array_equal(gi[qi, :n], ids[qi, :n], err_msg=f"{name} k{k} q{qi}")
                np.testing.assert_array_equal(bits(gd[qi, :n]), bits(dd[qi, :n]), err_msg=f"{name} k{k} q{qi}")
    finally:
        idx.close()
