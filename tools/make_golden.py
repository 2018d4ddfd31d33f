#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Runs in the CPU container only (needs /root/reference for oracle/_ref):
  * distances.npz   -- inputs and outputs of the reference's OWN compiled
                       distance kernels (distancer/c/*_amd64.c built by
                       oracle/Makefile into oracle/_ref/libref.so);
  * flat_search.npz -- flat-index searches over tie-heavy integer data, scored
                       by the reference's compiled kernels and ranked by the
                       restated NewMax heap scan (oracle/baseline.c with
                       use_ref=1);
  * flat_search_wide.npz -- the same at 512 / 768 / 1024 dims (the int8
                       block-key route), corpora as generator parameters;
  * bq.npz          -- BinaryQuantizer.Encode known answers from
                       compressionhelpers/binary_quantization_test.go:102-146.

Usage: make -C oracle && make -C oracle ref && python tools/make_golden.py
"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as orc  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")
LENGTHS = [1, 2, 3, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 40, 63, 64, 65, 100, 127, 128, 129, 130, 160, 200,
           255, 256, 257, 300, 511, 512, 513, 768, 960, 1536]
KERNELS = ["l2_256", "l2_512", "dot_256", "dot_512", "hamming_256", "hamming_512"]


def distances():
    r = orc.ref_lib()
    assert r is not None, "build oracle/_ref first (make -C oracle ref)"
    rng = np.random.default_rng(20260215)
    a_all, b_all, offs, lens = [], [], [0], []
    for n in LENGTHS:
        for kind in range(3):
            if kind == 0:
                a = rng.standard_normal(n).astype(np.float32)
                b = rng.standard_normal(n).astype(np.float32)
            elif kind == 1:  # wide dynamic range
                a = (rng.standard_normal(n) * np.exp(rng.uniform(-8, 8, n))).astype(np.float32)
                b = (rng.standard_normal(n) * np.exp(rng.uniform(-8, 8, n))).astype(np.float32)
            else:  # partly equal, for hamming
                a = rng.integers(-3, 4, n).astype(np.float32)
                b = a.copy()
                b[rng.integers(0, n, max(1, n // 3))] += 1
            a_all.append(a)
            b_all.append(b)
            offs.append(offs[-1] + n)
            lens.append(n)
    out = {k: np.zeros(len(lens), np.float32) for k in KERNELS}
    for i, n in enumerate(lens):
        for k in KERNELS:
            out[k][i] = orc.ref_kernel(k, a_all[i], b_all[i])
    # bitwise hamming through the reference kernel
    words = [1, 2, 3, 4, 5, 7, 8, 9, 16, 17, 24, 25, 33]
    wa, wb, woff, wout = [], [], [0], []
    lookup = (C.c_uint8 * 32)(*([0, 1, 1, 2, 1, 2, 2, 3, 1, 2, 2, 3, 2, 3, 3, 4] * 2))
    consts = (C.c_uint64 * 5)(0x5555555555555555, 0x3333333333333333, 0x0F0F0F0F0F0F0F0F, 0x0101010101010101,
                              0x0F0F0F0F0F0F0F0F)
    for w in words:
        for _ in range(3):
            x = rng.integers(0, 2**64, w, dtype=np.uint64)
            y = rng.integers(0, 2**64, w, dtype=np.uint64)
            res = C.c_uint64()
            ln = C.c_long(w)
            r.hamming_bitwise_256(x.ctypes.data_as(C.c_void_p), y.ctypes.data_as(C.c_void_p), C.byref(res),
                                  C.byref(ln), lookup, consts)
            wa.append(x)
            wb.append(y)
            woff.append(woff[-1] + w)
            wout.append(float(np.float32(res.value)))
    np.savez_compressed(os.path.join(OUT, "distances.npz"), a=np.concatenate(a_all), b=np.concatenate(b_all),
                        offsets=np.array(offs, np.int64), lengths=np.array(lens, np.int64),
                        bw_a=np.concatenate(wa), bw_b=np.concatenate(wb), bw_offsets=np.array(woff, np.int64),
                        bw_out=np.array(wout, np.float32), **out)


def flat_search():
    """Tie-heavy searches: integer data -> exact equal distances."""
    res = {}
    for name, metric, kind, n, d, seed in [("l2_int", orc.L2, 1, 600, 12, 5), ("dot_int", orc.DOT, 1, 500, 9, 6),
                                           ("cos_u", orc.COSINE, 0, 400, 20, 7), ("l2_dup", orc.L2, 1, 300, 4, 8)]:
        corpus = orc.gen_matrix(kind, seed, 0, n, d)
        if name == "l2_dup":
            corpus = np.concatenate([corpus[:30]] * 10)
        queries = orc.gen_matrix(kind, seed + 100, 0, 12, d)
        store = corpus.copy()
        q = queries.copy()
        if metric == orc.COSINE:
            orc.lib().or_normalize_rows(orc.f(store), store.shape[0], d)
            orc.lib().or_normalize_rows(orc.f(q), q.shape[0], d)
        for k in (1, 5, 10, 33):
            ids, dd, cnt = orc.cpu_baseline(metric, orc.AVX256, store, q, k, 4, use_ref=True)
            res[f"{name}_k{k}_ids"] = ids
            res[f"{name}_k{k}_dists"] = dd
            res[f"{name}_k{k}_counts"] = cnt
        res[f"{name}_corpus"] = corpus
        res[f"{name}_queries"] = queries
        res[f"{name}_metric"] = np.array(metric)
    np.savez_compressed(os.path.join(OUT, "flat_search.npz"), **res)


def flat_search_wide():
    """Rows wide enough for the int8 block-key route (384 < d <= 1536): the
    corpus is kept as its generator parameters (oracle.gen_matrix: the
    counter-based generator the GPU tests share) plus a checksum of its bits,
    the queries and the reference-kernel-scored results are stored."""
    res = {}
    for name, metric, kind, n, d, seed in [("cos_768", orc.COSINE, 0, 4000, 768, 11),
                                           ("l2_int_512", orc.L2, 1, 3000, 512, 12),
                                           ("dot_1024", orc.DOT, 0, 2000, 1024, 13)]:
        corpus = orc.gen_matrix(kind, seed, 0, n, d)
        queries = orc.gen_matrix(kind, seed + 100, 0, 12, d)
        if name == "l2_int_512":  # near-duplicate rows: exact ties inside the candidate blocks
            corpus[1::7] = corpus[0::7][: len(corpus[1::7])]
        store = corpus.copy()
        q = queries.copy()
        if metric == orc.COSINE:
            orc.lib().or_normalize_rows(orc.f(store), store.shape[0], d)
            orc.lib().or_normalize_rows(orc.f(q), q.shape[0], d)
        for k in (1, 10, 33):
            ids, dd, cnt = orc.cpu_baseline(metric, orc.AVX256, store, q, k, 4, use_ref=True)
            res[f"{name}_k{k}_ids"] = ids
            res[f"{name}_k{k}_dists"] = dd
            res[f"{name}_k{k}_counts"] = cnt
        res[f"{name}_gen"] = np.array([kind, seed, n, d], np.int64)
        res[f"{name}_dup7"] = np.array(1 if name == "l2_int_512" else 0)
        res[f"{name}_checksum"] = np.array(int(corpus.view(np.uint32).astype(np.uint64).sum()), np.uint64)
        res[f"{name}_queries"] = queries
        res[f"{name}_metric"] = np.array(metric)
    np.savez_compressed(os.path.join(OUT, "flat_search_wide.npz"), **res)


def wide_corpus(g, name):
    """The corpus of a flat_search_wide.npz case, regenerated and checked."""
    kind, seed, n, d = (int(x) for x in g[f"{name}_gen"])
    corpus = orc.gen_matrix(kind, seed, 0, n, d)
    if int(g[f"{name}_dup7"]):
        corpus[1::7] = corpus[0::7][: len(corpus[1::7])]
    assert int(corpus.view(np.uint32).astype(np.uint64).sum()) == int(g[f"{name}_checksum"])
    return corpus


def bq():
    # binary_quantization_test.go:102-123 fixed values
    fixed_in = np.array([-1, 1, 0, np.nan, np.inf, -np.inf], np.float32)
    fixed_bits = np.array([1, 0, 0, 0, 0, 1], np.uint8)  # -1->1, 1->0, 0->0, NaN->0, +Inf->0, -Inf->1
    np.savez_compressed(os.path.join(OUT, "bq.npz"), fixed_in=fixed_in, fixed_bits=fixed_bits)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    distances()
    flat_search()
    flat_search_wide()
    bq()
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))
