#!/bin/bash
# selected GPU test files on the current tree: bash tools/gpu_tests.sh <tag> <pytest args...>
TAG=${1:-t}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread "$@" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/tests.log | tail -40; tail -30 $O/tests.log
exit $rc
