#!/bin/bash
# round-3 final check, part A: the whole GPU suite, smoke(), the default bench
# (C3) under rocprof, and the N > 1 code path at world 1 over RCCL (c3, rq-8)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-final3a}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
echo "smoke ok"; tail -2 $O/smoke.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
python3 -c "import json; r=json.load(open('$O/bench_c3.json')); print('c3', round(r['value']), round(r['ms_per_step'],2), r['roofline']['frac'], r.get('verified'), r['cpu_baseline'].get('value'))"
for w in c3 rq8; do
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --workload $w --sharded --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_${w}_sharded1.out 2> $O/bench_${w}_sharded1.err || { tail $O/bench_${w}_sharded1.err; exit 1; }
grep '^{' $O/bench_${w}_sharded1.out > $O/bench_${w}_sharded1.json
python3 -c "import json; r=json.load(open('$O/bench_${w}_sharded1.json')); print('$w sharded w1', round(r['value']), round(r['ms_per_step'],2), r.get('sharded_equals_single'), r.get('verified'))"
done
