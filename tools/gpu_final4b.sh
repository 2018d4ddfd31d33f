#!/bin/bash
# round-4 closing check, part B: every workload's bench under rocprof (with its
# CPU baseline), C3 through the N > 1 code path at world 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-final4b}; mkdir -p $O
for w in ${WL:-c3 c2 c1 bq pq rq8 rq1}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail $O/bench_$w.err; exit 1; }
  python3 -c "import json; r=json.load(open('$O/bench_$w.json')); print('$w', round(r['value']), round(r['ms_per_step'],2), r['roofline'].get('kernel'), r['roofline'].get('frac'), r.get('verified'), (r.get('cpu_baseline') or {}).get('value'))"
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29537 \
  bench.py --workload c3 --sharded --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_c3_sharded1.out 2> $O/bench_c3_sharded1.err || { tail $O/bench_c3_sharded1.err; exit 1; }
grep '^{' $O/bench_c3_sharded1.out > $O/bench_c3_sharded1.json
python3 -c "import json; r=json.load(open('$O/bench_c3_sharded1.json')); print('c3 sharded w1', round(r['value']), round(r['ms_per_step'],2), r.get('sharded_equals_single'), r.get('verified'))"
