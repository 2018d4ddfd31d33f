#!/bin/bash
# BQ bench (+ rocprofv3 kernel stats) on the GPU box. Usage: bash tools/gpu_bench_bq.sh <tag> [bench args]
TAG=${1:-bq}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u bench.py --workload bq "$@" > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json; tail -3 $O/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload bq --no-cpu-baseline "$@" > $O/bench_prof.json 2> $O/bench_prof.err; rc=$?
echo "prof rc=$rc"; head -6 $O/prof/run_kernel_stats.csv
exit $rc
