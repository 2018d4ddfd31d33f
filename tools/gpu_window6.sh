#!/bin/bash
# serving with the batch window (the leader waits until the callers of the last
# cycle are back): C3 at 64 / 256 / 1024 callers, windows 0 / 300 / 1000 us
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-win6}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_batcher.py tests/test_gpu_multi_allow.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for cfg in "256 0" "256 300" "256 1000" "64 0" "1024 0" "1024 1000" "1 1000"; do
set -- $cfg
timeout -k 10 150 tools/serve_bench 10000000 $1 6 $2 > $O/c3_$1_w$2.json 2> $O/c3_$1_w$2.err || { tail $O/c3_$1_w$2.err; exit 1; }
cat $O/c3_$1_w$2.json
done
timeout -k 10 120 tools/serve_bench 1000000 256 6 0 5 100 > $O/f5_all.json 2> $O/f5_all.err || { tail $O/f5_all.err; exit 1; }
cat $O/f5_all.json
