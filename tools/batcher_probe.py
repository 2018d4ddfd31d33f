"""Repeat the batcher's concurrent filtered-caller scenario and report every
mismatch against the one-query calls (kind of list, ids missing / extra,
whether they are in the caller's list).  GPU debugging aid."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import weaviate_amd as wv  # noqa: E402
from weaviate_amd import _lib  # noqa: E402

sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402
from test_gpu_multi_allow import _allow_lists  # noqa: E402

n, d, k = 20000, int(sys.argv[1]) if len(sys.argv) > 1 else 128, 10
data = oracle.gen_matrix(0, 75, 0, n, d)
queries = oracle.gen_matrix(0, 76, 0, 64, d)
bad = 0
for trial in range(int(os.environ.get("TRIALS", "4"))):
    idx = wv.FlatIndex(distance="cosine", variant="avx256")
    idx.add_batch(np.arange(n, dtype=np.uint64), data)
    idx.set_option("batch_window_us", 3000)
    for kv in sys.argv[2:]:
        kk, vv = kv.split("=")
        idx.set_option(kk, int(vv))
    allows = _allow_lists(wv, n, len(queries), k, seed=5)
    exp = [idx.search_by_vector_batch(queries[i:i + 1], k, allow=allows[i]) for i in range(len(queries))]
    for rnd in range(3):
        order = np.random.default_rng(rnd).permutation(len(queries))
        with ThreadPoolExecutor(32) as ex:
            res = dict(zip(order, ex.map(lambda i: idx.search_by_vector(queries[i], k, allow=allows[i]), order)))
        for i in range(len(queries)):
            ri, rd = res[i]
            ei, ed, ec = exp[i]
            if not np.array_equal(ri, ei[0, :ec[0]]):
                bad += 1
                al = set() if allows[i] is None else set(int(x) for x in allows[i].ids)
                miss = [int(x) for x in ei[0, :ec[0]] if int(x) not in set(int(y) for y in ri)]
                extra = [int(x) for x in ri if int(x) not in set(int(y) for y in ei[0, :ec[0]])]
                print(f"trial {trial} round {rnd} q{i} kind {i % 9} list {len(al)} missing {miss} "
                      f"(in list {[m in al for m in miss]}) extra {extra} (in list {[e in al for e in extra]})",
                      flush=True)
    print("trial", trial, "batcher", idx.batcher_stats(), flush=True)
    idx.close()
print("mismatches", bad, sys.argv[2:])
