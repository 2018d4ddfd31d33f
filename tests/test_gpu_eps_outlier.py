"""The ε cliff (VERDICT r5 "ε is still index-global"): the int8 block keys'
error bound ε(q) uses the corpus-wide maxima N, H, R (qs_eps,
weaviate_amd/csrc/qs_kernels.hip), so ONE row with a 1000× norm widens every
query's candidate window for the life of the index.  This test pins what that
costs and that results stay exact: the same corpus with and without the
outlier row, searched on the int8 route, equals the oracle (flat/index.go:578-619
with the reference heap) bit for bit, and the replayed-query and scanned-row
counts of both are written to gpurun_out/eps_cliff.json.
No bound is asserted on the ratio: ε is per index, not per block."""
import json
import os

import numpy as np
import pytest

from test_gpu_flat import assert_same, build_pair, gen

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("metric", ["dot", "l2-squared"])
def test_outlier_row_keeps_results_exact(wv, oracle, metric):
    n, d, k, nq = 120000, 512, 10, 48
    data = gen(oracle, 0, 191, n, d)
    queries = gen(oracle, 0, 192, nq, d)
    out = {}
    for name, scale in (("clean", 1.0), ("outlier", 1000.0)):
        x = data.copy()
        x[77777] *= np.float32(scale)
        idx, orc = build_pair(wv, oracle, metric, "avx256", x, options={"timing": 1})
        idx.search_by_vector_batch(queries, k)  # warm
        before = idx.stats()["replayed_queries"]
        ids, dists, counts = idx.search_by_vector_batch(queries, k)
        st = idx.stats()
        out[name] = {"route": st.get("last_route"), "replayed_queries": st["replayed_queries"] - before,
                     "scan_rows": st.get("last_scan_rows"), "total_ms": st.get("last_total_ms")}
        for qi in range(nq):
            assert_same(orc.search(queries[qi], k), ids[qi, :counts[qi]], dists[qi, :counts[qi]],
                        f"{metric} {name} q{qi}")
    os.makedirs("gpurun_out", exist_ok=True)
    path = os.path.join("gpurun_out", "eps_cliff.json")
    rec = json.load(open(path)) if os.path.exists(path) else {}
    rec[metric] = {"rows": n, "dims": d, "k": k, "queries": nq, "outlier_row_norm_scale": 1000.0, **out}
    json.dump(rec, open(path, "w"), indent=1)
    print(metric, out)
