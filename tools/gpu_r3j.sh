#!/bin/bash
8-lanes-per-row exact distances in k_blk_replay: replay parity tests, the C2
full-size test and the C2 bench under rocprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_scale.py tests/test_gpu_sharded_threads.py -m gpu -x -v  --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --workload c2 > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
python3 -c "import json; r=json.load(open('$O/bench_c2.json')); print('c2', round(r['value']), round(r['ms_per_step'],2), r['roofline']['frac'], r.get('verified'))"
python3 tools/kstats.py $(ls $O/prof_c2/*/run_kernel_stats.csv $O/prof_c2/run_kernel_stats.csv 2>/dev/null) > $O/kstats.txt; head -9 $O/kstats.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
python3 -c "import json; r=json.load(open('$O/bench_c3.json')); print('c3', round(r['value']), round(r['ms_per_step'],2), r['roofline']['frac'], r.get('verified'))"
python3 tools/kstats.py $(ls $O/prof_c3/*/run_kernel_stats.csv $O/prof_c3/run_kernel_stats.csv 2>/dev/null) > $O/kstats_c3.txt; head -6 $O/kstats_c3.txt
