#!/bin/bash
# k_pq_adc4 (16-byte LUT reads): PQ parity tests, adc3/adc4 A/B on C5, C5 bench with adc4 under rocprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-pq4}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pq.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u tools/pq_probe.py pq_adc3=1 pq_adc3=2 pq_adc3=1 pq_adc3=2 > $O/probe.txt 2>&1; rc=$?
cat $O/probe.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_pq -o run --output-format csv -- python3 bench.py --workload pq --no-cpu-baseline --option pq_adc3=2 > $O/pq.json 2> $O/pq.err || { tail $O/pq.err; exit 1; }
python3 -c "import json; r=json.load(open('$O/pq.json')); print('pq', round(r['value']), round(r['ms_per_step'],3), r.get('verified'), r.get('roofline'))"
python3 tools/kstats.py $O/prof_pq/run_kernel_stats.csv | head -6
