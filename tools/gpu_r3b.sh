#!/bin/bash
# round-3 checkpoint: the whole GPU suite, the headline + workload benches under rocprof
# (C3, C2, C4 BQ, C5 PQ via k_pq_adc3, d = 1024 / 1536 block keys), then the PMC
# traffic passes of k_pq_adc3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3b}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json,sys; r=json.load(open('$1')); print('$2', round(r['value']), 'qps', round(r['ms_per_step'],2), 'ms', r['roofline'].get('launch_ms'), r['roofline'].get('frac'), r.get('verified'))"; }
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- python3 bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail $O/bench_$n.err; exit 1; }
  summ $O/bench_$n.json $n
  python3 tools/kstats.py $O/prof_$n/run_kernel_stats.csv > $O/ks_$n.txt 2>&1; head -5 $O/ks_$n.txt
}
run c3
run c2 --workload c2
run bq --workload bq
run pq --workload pq
run d1024 --dims 1024 --no-cpu-baseline
run d1536 --dims 1536 --no-cpu-baseline
bash tools/pmc_traffic.sh $O/pmc_pq --workload pq && python3 tools/pmc_summary.py $O/pmc_pq > $O/pmc_pq_summary.txt 2>&1; grep adc3 $O/pmc_pq_summary.txt
