#!/bin/bash
# sharded hnsw flat search over PQ / SQ codes (ShardedQuantSearch, ranks as threads)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-quant}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_threads.py tests/test_gpu_pq.py tests/test_gpu_hnsw_flat.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|Error|error" $O/tests.log | tail -30; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
# the sharded PQ protocol at world 1 through RCCL (bench --sharded: equals the single-index search)
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519 \
  bench.py --workload pq --sharded --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_pq_sharded1.json 2> $O/bench_pq_sharded1.err || { tail $O/bench_pq_sharded1.err; exit 1; }
python3 -c "import json; r=json.load(open('$O/bench_pq_sharded1.json')); print('pq sharded w1', round(r['value']), r['ms_per_step'], r.get('sharded_equals_single'), r['roofline'].get('kernel'), r['roofline'].get('launch_ms'))"
