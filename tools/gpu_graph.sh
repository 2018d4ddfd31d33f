#!/bin/bash
# hipGraph replay: graph test, C1 with / without graphs, C3 (captured) verified
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-graph}; mkdir -p $O
timeout -k 10 300 python -u -m pytest "tests/test_gpu_flat.py::test_search_device_graph_replay" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --workload c1 --steps 200 --warmup 5 --no-cpu-baseline > $O/c1.json 2> $O/c1.err || { tail $O/c1.err; exit 1; }
timeout -k 10 300 python3 bench.py --workload c1 --steps 200 --warmup 5 --no-cpu-baseline --option graph=0 > $O/c1_nograph.json 2> $O/c1_nograph.err || { tail $O/c1_nograph.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c1 -o run --output-format csv -- python3 bench.py --workload c1 --steps 200 --warmup 5 --no-cpu-baseline > $O/c1_prof.json 2> $O/c1_prof.err || { tail $O/c1_prof.err; exit 1; }
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
for f in c1 c1_nograph c1_prof c3; do python3 -c "import json; r=json.load(open('$O/$f.json')); print('$f', round(r['value']), round(r['ms_per_step'],4), r.get('verified'), r['roofline'].get('launch_ms'))"; done
python3 tools/kstats.py $O/prof_c1/run_kernel_stats.csv > $O/kernel_stats_c1.txt && head -14 $O/kernel_stats_c1.txt
