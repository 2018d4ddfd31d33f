#!/bin/bash
# k_pq_adc2: PQ parity tests (incl. the full C5 shape) + bench pq + kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-pq2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pq.py tests/test_gpu_hnsw_flat.py "tests/test_gpu_scale.py::test_c5_pq_960_m240_ks256" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --workload pq > $O/bench_pq.json 2> $O/bench_pq.err || { tail $O/bench_pq.err; exit 1; }
cat $O/bench_pq.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_pq -o run --output-format csv -- python3 bench.py --workload pq --no-cpu-baseline > $O/bench_pq_prof.json 2> $O/bench_pq_prof.err || exit $?
bash tools/pmc_traffic.sh $O/pmc_pq --workload pq || exit $?
python3 tools/pmc_summary.py $O/pmc_pq > $O/pmc_pq_summary.txt; cat $O/pmc_pq_summary.txt
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE -d $O/pmc_pq_lds/lds -o run --output-format csv -- python3 bench.py --workload pq --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc_pq_lds.log 2>&1 || exit $?
python3 tools/pmc_summary.py $O/pmc_pq_lds > $O/pmc_pq_lds_summary.txt; cat $O/pmc_pq_lds_summary.txt
