#!/bin/bash
# the full-size sharded C5 test (4 shards as threads) + C2's replay clock diagnostics
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3e}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_threads.py -m gpu -x -v -k "c5_sharded" --timeout 500 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --workload c2 --no-cpu-baseline --no-verify --steps 1 --warmup 0 --option replay_dbg=1 > $O/c2_dbg.out 2> $O/c2_dbg.err || { tail $O/c2_dbg.err; exit 1; }
grep "k_blk_replay dbg" $O/c2_dbg.out | head -40
