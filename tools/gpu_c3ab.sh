#!/bin/bash
# usage: gpu_c3ab.sh OUT "TESTS" "OPTS1" "OPTS2" ...  -- optional pytest files, then C3 bench
# variants (space-separated --option key=value lists; "-" = defaults), each under rocprofv3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; shift; mkdir -p $O
T="$1"; shift
if [ -n "$T" ] && [ "$T" != "-" ]; then
  timeout -k 10 900 python -u -m pytest $T -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for v in "$@"; do
  i=$((i+1)); opts=""
  if [ "$v" != "-" ]; then for kv in $v; do opts="$opts --option $kv"; done; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline $BENCH_EXTRA $opts > $O/bench_$i.json 2> $O/bench_$i.err || { tail $O/bench_$i.err; exit 1; }
  python3 - $O/bench_$i.json $O/prof_$i/run_kernel_stats.csv "$v" <<'PY'
import json, sys, csv
r = json.load(open(sys.argv[1]))
print("variant", sys.argv[3], "qps", round(r["value"]), "ms", round(r["ms_per_step"], 2), "key", r["roofline"].get("kernel"),
      round(r["roofline"].get("launch_ms", 0), 2), "frac", round(r["roofline"].get("frac", 0), 3), "verified", r.get("verified"),
      "replayed", r["config"].get("replayed_queries"))
rows = list(csv.DictReader(open(sys.argv[2])))
for x in rows[:12]:
    print("   ", x["Name"][:60], x["Calls"], round(float(x["AverageNs"]) / 1e6, 3))
PY
done
