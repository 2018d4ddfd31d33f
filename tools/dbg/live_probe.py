import os, sys, json
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as orc
import weaviate_amd as wv
n, d, k = 30000, 768, 10
data = orc.gen_matrix(0, 71, 0, n, d)
queries = orc.gen_matrix(0, 72, 0, 300, d)
idx = wv.FlatIndex(distance="cosine", variant="avx256")
idx.add_batch(np.arange(n, dtype=np.uint64), data)
for nq in (256, 300, 64):
    for live in (0, 1):
        for prio in (0, 1):
            idx.set_option("q8_live", live); idx.set_option("q8_prio", prio)
            ids, dd, cnt = idx.search_by_vector_batch(queries[:nq], k)
            A, eps = idx.debug_blockkeys(0)
            print(json.dumps({"nq": nq, "live": live, "prio": prio, "cnt0": int(cnt[0]), "cnt_min": int(cnt.min()),
                              "route": idx.stats()["last_route"], "key0": [float(x) for x in A[:4]],
                              "inf_keys": int(np.isinf(A).sum()), "nb": int(len(A)), "ids0": ids[0, :3].tolist()}), flush=True)
