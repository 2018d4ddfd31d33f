#!/bin/bash
# BQ on the integer matrix cores: parity tests, then C4 with int8 vs VALU minima
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-bq8}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_q8.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in "-" "bq8=0"; do
  opts=""; [ "$v" != "-" ] && opts="--option $v"
  n=$(echo "$v" | tr '=' '_')
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_bq_$n -o run --output-format csv -- python3 bench.py --workload bq --no-cpu-baseline $opts > $O/bench_bq_$n.json 2> $O/bench_bq_$n.err || { tail $O/bench_bq_$n.err; exit 1; }
  python3 tools/kstats.py $O/bench_bq_$n.json $O/prof_bq_$n/run_kernel_stats.csv "$v" || true
done
