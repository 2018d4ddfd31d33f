#!/bin/bash
# C2 with the capped selection: block-major exact A/B, bench c1 / c2 lines, c2 kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-cap2}; mkdir -p $O
timeout -k 10 300 python -u tools/qs_probe.py --n 1000000 --d 128 --k 100 --batch 10000 --metric l2-squared --kind 1 --verify 0 --configs "exact_bm=0;exact_bm=1;exact_bm=0;exact_bm=1" > $O/c2_bm.log 2>&1 || { cat $O/c2_bm.log; exit 1; }
cat $O/c2_bm.log
for w in c2 c1; do
  timeout -k 10 300 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --workload c2 --no-cpu-baseline > $O/bench_c2_prof.json 2> $O/bench_c2_prof.err || exit $?
python3 - "$O/prof_c2/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r["Percentage"]) > 0.5: print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), r["Percentage"])
PY
