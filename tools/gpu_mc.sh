#!/bin/bash
# multi-shard tests + the bench's N>1 path at world 1 (bq, pq, c3 small)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-mc}; mkdir -p $O
[ -n "$SKIPT" ] && rc=0 || { timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_multi_compressed.py tests/test_gpu_multi.py > $O/tests.log 2>&1; rc=$?; }
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/tests.log | tail -40; [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
for w in bq pq; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29561 bench.py --workload $w --sharded --steps 3 --warmup 1 --no-cpu-baseline --rows 2000000 > $O/bench_$w.json 2> $O/bench_$w.err; rc=$?
  echo "bench $w rc=$rc"; cat $O/bench_$w.json | head -c 1500; echo; [ $rc -eq 0 ] || { tail -20 $O/bench_$w.err; exit $rc; }
  grep -h "equals the single" $O/bench_$w.err
done
