#!/bin/bash
# ASan + UBSan host build of the LSM segment reader and a mutation fuzz run over
# the reference's segment files (tests/golden/lsm).  CPU only.
set -e
REPO="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${TMPDIR:-/tmp}/wv_lsm_fuzz"
mkdir -p "$OUT"
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer \
    -x c++ "$REPO/tools/lsm_fuzz.cpp" -o "$OUT/lsm_fuzz"
# vectors-bucket seeds written by the oracle's segment writer (v0 and v1, with
# tombstones), beside the reference's own segment files
python3 - "$OUT" "$REPO" <<'PY'
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[2], "oracle"))
import lsm
out = sys.argv[1]
rng = np.random.default_rng(1)
for i, (n, d, ver) in enumerate([(6, 4, 1), (9, 3, 0), (4, 16, 1)]):
    e = lsm.vector_entries(range(n), rng.standard_normal((n, d)).astype(np.float32))
    e += lsm.vector_entries([n + 1], None)
    open(f"{out}/seed{i}.db", "wb").write(lsm.write_segment(sorted(e, key=lambda t: t[0]), version=ver))
PY
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 "$OUT/lsm_fuzz" "$OUT" "${1:-20000}" "$REPO"/tests/golden/lsm/*.db "$OUT"/seed*.db
