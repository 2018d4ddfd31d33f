#!/bin/bash
# register-heap replays (k_blk_replay, k_bq_replay_w) + whole-round span counts:
# the full GPU suite, then C2 / C4 / d = 1024 benches under rocprof (C4 also with the LDS heap)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-heap}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json,sys; r=json.load(open('$1')); print('$2', round(r['value']), 'qps', round(r['ms_per_step'],2), 'ms', r['roofline'].get('launch_ms'), r['roofline'].get('frac'), r.get('verified'))"; }
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail $O/bench_$n.err; exit 1; }
  summ $O/bench_$n.json $n
  python3 tools/kstats.py $O/prof_$n/run_kernel_stats.csv > $O/ks_$n.txt 2>&1; head -7 $O/ks_$n.txt
}
run c2 --workload c2
run bq --workload bq
run bq_lds --workload bq --option reg_heap=0
run d1024 --dims 1024
run pq --workload pq
run pq_adc2 --workload pq --option pq_adc3=0
run rq8 --workload rq8
