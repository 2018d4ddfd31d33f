#!/bin/bash
# filtering select, chunk vote: exact-path tests, C3 / C2 / 1.25M with both select forms
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-self2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_q8.py tests/test_gpu_sharded_flat.py -k "not 10m_rows" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for SF in 1 0; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3_sf$SF -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify --option sel_filter=$SF > $O/c3_sf$SF.json 2> $O/c3_sf$SF.err || { tail $O/c3_sf$SF.err; exit 1; }
  python3 tools/kstats.py $O/prof_c3_sf$SF/run_kernel_stats.csv | grep "select" | head -3
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2_sf$SF -o run --output-format csv -- python3 bench.py --workload c2 --no-cpu-baseline --no-verify --option sel_filter=$SF > $O/c2_sf$SF.json 2> $O/c2_sf$SF.err || { tail $O/c2_sf$SF.err; exit 1; }
  python3 tools/kstats.py $O/prof_c2_sf$SF/run_kernel_stats.csv | grep "select" | head -3
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_s_sf$SF -o run --output-format csv -- python3 bench.py --n 1250000 --no-cpu-baseline --no-verify --option sel_filter=$SF > $O/s_sf$SF.json 2> $O/s_sf$SF.err || { tail $O/s_sf$SF.err; exit 1; }
  python3 tools/kstats.py $O/prof_s_sf$SF/run_kernel_stats.csv | grep "select" | head -3
done
