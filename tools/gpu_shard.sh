#!/bin/bash
# sharded exact path: GPU sharded tests (threads, flat), then the 8-shard simulation at B = 8192
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-shard}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded_flat.py tests/test_gpu_sharded_threads.py -k "not c5_sharded" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 tools/shard_sim.py --batch 8192 > $O/w8_b8192.json 2> $O/w8_b8192.err || { tail -5 $O/w8_b8192.err; exit 1; }
python3 -c "import json; r=json.load(open('$O/w8_b8192.json')); print({k: r[k] for k in ('flagged','equal_to_single','phase1_max','phase2_max','merge','replay_max','merge_rec','compute_ms')})"
