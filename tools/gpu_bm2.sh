#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-bm2}; mkdir -p $O
for bm in 0 1; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$bm -o run --output-format csv -- python3 tools/qs_probe.py --n 1000000 --d 128 --k 100 --batch 10000 --metric l2-squared --kind 1 --verify 0 --configs "exact_bm=$bm" > $O/c2_$bm.log 2>&1 || { cat $O/c2_$bm.log; exit 1; }
python3 - "$O/p$bm/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r["Percentage"]) > 0.5: print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), r["Percentage"])
PY
done
