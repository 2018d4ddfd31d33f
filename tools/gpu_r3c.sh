#!/bin/bash
# packed-record replay heaps (k_blk_replay, k_bq_replay, k_replay_scan) + BQ replay
# instantiations + k_pq_adc3 bound experiments: the whole GPU suite, C2 / C4 / rq-8
# benches under rocprof, the adc3 probe
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3c}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail $O/bench_$n.err; exit 1; }
  python3 -c "import json; r=json.load(open('$O/bench_$n.json')); print('$n', round(r['value']), round(r['ms_per_step'],2), r['roofline'].get('frac'), r.get('verified'))"
  python3 tools/kstats.py $O/prof_$n/run_kernel_stats.csv > $O/ks_$n.txt 2>&1; head -5 $O/ks_$n.txt
}
run c2 --workload c2
run bq --workload bq
run rq8 --workload rq8
exit 0
