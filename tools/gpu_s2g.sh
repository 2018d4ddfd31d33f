#!/bin/bash
# evidence run: default bench (c3, B=4096, cpu baseline) + kernel stats + PMC traffic; c1 / c2 benches;
# PMC traffic of the bq / pq / rq dominant kernels and the LDS counters of k_pq_adc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s2g}; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit $?; cat $O/bench_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_c3_prof.json 2> $O/bench_c3_prof.err || exit $?
bash tools/pmc_traffic.sh $O/pmc_c3 || exit $?
python3 tools/pmc_summary.py $O/pmc_c3 > $O/pmc_c3_summary.txt; cat $O/pmc_c3_summary.txt
for w in c1 c2; do
  timeout -k 10 300 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || exit $?; cat $O/bench_$w.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --workload c2 --no-cpu-baseline > $O/bench_c2_prof.json 2> $O/bench_c2_prof.err || exit $?
for w in bq pq rq8; do
  bash tools/pmc_traffic.sh $O/pmc_$w --workload $w || exit $?
  python3 tools/pmc_summary.py $O/pmc_$w > $O/pmc_${w}_summary.txt; cat $O/pmc_${w}_summary.txt
done
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $O/pmc_pq_lds/lds -o run --output-format csv -- python3 bench.py --workload pq --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc_pq_lds.log 2>&1 || exit $?
python3 tools/pmc_summary.py $O/pmc_pq_lds > $O/pmc_pq_lds_summary.txt; cat $O/pmc_pq_lds_summary.txt
