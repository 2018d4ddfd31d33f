#!/bin/bash
# round-3 final check, part B: the sharded tests (query chunks), rq-8 through the
# N > 1 code path at world 1, then every workload's bench under rocprof (with its
# CPU baseline)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-final3b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_threads.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --workload rq8 --sharded --no-cpu-baseline --steps 2 --warmup 1 > $O/bench_rq8_sharded1.out 2> $O/bench_rq8_sharded1.err || { tail $O/bench_rq8_sharded1.err; exit 1; }
grep '^{' $O/bench_rq8_sharded1.out > $O/bench_rq8_sharded1.json
python3 -c "import json; r=json.load(open('$O/bench_rq8_sharded1.json')); print('rq8 sharded w1', round(r['value']), round(r['ms_per_step'],2), r.get('sharded_equals_single'), r.get('verified'))"
for w in c3 c2 c1 bq pq rq8 rq1; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail $O/bench_$w.err; exit 1; }
  python3 -c "import json; r=json.load(open('$O/bench_$w.json')); print('$w', round(r['value']), round(r['ms_per_step'],2), r['roofline'].get('kernel'), r['roofline'].get('frac'), r.get('verified'), (r.get('cpu_baseline') or {}).get('value'))"
done
