#!/bin/bash
# final-tree evidence: smoke, default bench (cpu baseline), kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-final2}; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_c3_prof.json 2> $O/bench_c3_prof.err || exit $?
python3 - "$O/prof_c3/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r["Percentage"]) > 0.3: print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), r["Percentage"])
PY
