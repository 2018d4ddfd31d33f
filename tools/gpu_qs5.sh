#!/bin/bash
# verify (c3/c2 vs GEMV) -> gpu tests -> c3 bench with cpu baseline
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-qs5}; mkdir -p $O
bash tools/gpu_qs3.sh ${1:-qs5} || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err; rc=$?
echo "bench rc=$rc"; cat $O/bench_c3.json; exit $rc
