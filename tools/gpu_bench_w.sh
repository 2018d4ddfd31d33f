#!/bin/bash
# Bench (+ rocprofv3 kernel stats) for the named workloads. Usage: bash tools/gpu_bench_w.sh <tag> <w1,w2,..> [bench args]
TAG=${1:-w}; WL=${2:-pq}; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG; mkdir -p $O
for W in ${WL//,/ }; do
  timeout -k 10 300 python -u bench.py --workload $W "$@" > $O/bench_$W.json 2> $O/bench_$W.err; rc=$?
  echo "bench $W rc=$rc"; cat $O/bench_$W.json; tail -3 $O/bench_$W.err
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$W -o run --output-format csv -- python3 bench.py --workload $W --no-cpu-baseline "$@" > $O/bench_prof_$W.json 2> $O/bench_prof_$W.err; rc=$?
  echo "prof $W rc=$rc"; head -6 $O/prof_$W/run_kernel_stats.csv | cut -c1-160
  [ $rc -eq 0 ] || exit $rc
done
