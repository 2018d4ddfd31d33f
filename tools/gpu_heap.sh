#!/bin/bash
# read-ahead heap sifts: replay / tie / golden / sharded / BQ tests, C2 + C4 benches with the replay split
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-heap}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_golden.py tests/test_gpu_sharded_flat.py tests/test_gpu_sharded_threads.py tests/test_gpu_q8.py "tests/test_gpu_scale.py::test_c2_full_integer_k100" -k "not c5_sharded" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --workload c2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { tail $O/c2.err; exit 1; }
python3 -c "import json; r=json.load(open('$O/c2.json')); print('c2', round(r['value']), round(r['ms_per_step'],3), r.get('verified'), r['config'].get('replayed_queries'))"
python3 tools/kstats.py $O/prof_c2/run_kernel_stats.csv | grep "replay" | head -3
timeout -k 10 300 python3 bench.py --workload c2 --steps 1 --warmup 0 --no-cpu-baseline --no-verify --option replay_dbg=1 > $O/dbg.txt 2> $O/dbg.err; grep "k_blk_replay dbg" $O/dbg.txt | head -4
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_bq -o run --output-format csv -- python3 bench.py --workload bq --no-cpu-baseline > $O/bq.json 2> $O/bq.err || { tail $O/bq.err; exit 1; }
python3 -c "import json; r=json.load(open('$O/bq.json')); print('bq', round(r['value']), round(r['ms_per_step'],3), r.get('verified'))"
python3 tools/kstats.py $O/prof_bq/run_kernel_stats.csv | grep -v "k_prepare\|k_gen\|encode\|unpack" | head -6
