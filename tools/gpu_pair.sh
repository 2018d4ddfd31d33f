#!/bin/bash
# int8 key kernel change check: q8 + filter parity tests, the C3 probe, C3 bench under rocprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-pair}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_q8.py tests/test_gpu_filter.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/qs_probe.py --verify 0 --batch 8192 --configs "${PROBE:-q8=1}" > $O/probe.txt 2>&1 || { tail $O/probe.txt; exit 1; }
cat $O/probe.txt | grep -v amdgpu.ids
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; r=json.load(open('$O/bench.json')); print('c3', round(r['value']), round(r['ms_per_step'],2), r['roofline'].get('launch_ms'), r['roofline'].get('frac'), r.get('verified'), r['config'].get('replayed_queries'))"
python3 tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kernel_stats.txt && head -12 $O/kernel_stats.txt
