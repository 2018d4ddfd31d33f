#!/bin/bash
# int8 block keys: parity tests, then C3 with int8 keys vs bf16 keys under rocprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-q8}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_q8.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3q8 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_c3q8.json 2> $O/bench_c3q8.err || { tail $O/bench_c3q8.err; exit 1; }
python3 -c "import json; r=json.load(open('$O/bench_c3q8.json')); print('c3 q8', round(r['value']), round(r['ms_per_step'],2), r['roofline'].get('launch_ms'), r['roofline'].get('frac'), r.get('verified'), r['config'].get('replayed_queries'))"
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-verify --option q8=0 > $O/bench_c3bf.json 2> $O/bench_c3bf.err || { tail $O/bench_c3bf.err; exit 1; }
python3 -c "import json; r=json.load(open('$O/bench_c3bf.json')); print('c3 bf16', round(r['value']), round(r['ms_per_step'],2), r['roofline'].get('launch_ms'), r['roofline'].get('frac'), r['config'].get('replayed_queries'))"
