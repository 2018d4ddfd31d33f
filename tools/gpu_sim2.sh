#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-sim}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_multi_compressed.py tests/test_gpu_sharded_flat.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
timeout -k 10 300 python -u tools/shard_sim.py --world 8 --reps 5 > $O/sim_fwd.json 2> $O/sim_fwd.err; rc=$?
echo "fwd rc=$rc"; cat $O/sim_fwd.json; [ $rc -eq 0 ] || { tail $O/sim_fwd.err; exit $rc; }
