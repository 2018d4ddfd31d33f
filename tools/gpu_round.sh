#!/bin/bash
# One GPU call: gpu tests -> bench -> rocprofv3 kernel-trace stats of the bench.
# Usage (on the GPU box): bash tools/gpu_round.sh <tag> [bench args...]
TAG=${1:-r}; shift
BARGS="$@"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py $BARGS > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline $BARGS > $O/bench_prof.json 2> $O/bench_prof.err; rc=$?
echo "prof rc=$rc"; cat $O/bench_prof.json
find $O/prof -name '*kernel_stats.csv' | head -3
exit $rc
