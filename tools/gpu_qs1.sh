#!/bin/bash
# first GPU pass of the block-key path: smoke -> gpu tests -> bench -> kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-qs1}; mkdir -p $O
timeout -k 10 120 python -u tools/qs_smoke.py > $O/smoke.log 2>&1; rc=$?
cat $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json; tail -3 $O/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_prof.json 2> $O/bench_prof.err; rc=$?
echo "prof rc=$rc"
find $O/prof -name '*kernel_stats.csv' -exec head -12 {} \;
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -v --maxfail=15 --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/gpu_tests.log | tail -25
exit $rc
