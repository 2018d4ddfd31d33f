#!/bin/bash
# filtering select: exact-path GPU tests, the 8-shard simulation, C3 / C2 with both select forms
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-self}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_q8.py tests/test_gpu_filter.py tests/test_gpu_sharded_flat.py tests/test_gpu_sharded_threads.py -k "not c5_sharded and not 10m_rows" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 tools/shard_sim.py --batch 8192 > $O/w8_b8192.json 2> $O/w8_b8192.err || { tail -5 $O/w8_b8192.err; exit 1; }
python3 -c "import json; r=json.load(open('$O/w8_b8192.json')); print({k: r[k] for k in ('flagged','equal_to_single','phase1_max','phase2_max','merge','replay_max','merge_rec','compute_ms')})"
for SF in 1 0; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3_sf$SF -o run --output-format csv -- python3 bench.py --no-cpu-baseline --option sel_filter=$SF > $O/c3_sf$SF.json 2> $O/c3_sf$SF.err || { tail $O/c3_sf$SF.err; exit 1; }
  python3 -c "import json; r=json.load(open('$O/c3_sf$SF.json')); print('c3 sf$SF', round(r['value']), round(r['ms_per_step'],2), r.get('verified'), r['config'].get('replayed_queries'))"
  python3 tools/kstats.py $O/prof_c3_sf$SF/run_kernel_stats.csv | grep -v "k_prepare\|k_block_q8\|k_rows_split\|k_gen" | head -6
  timeout -k 10 400 python3 bench.py --workload c2 --no-cpu-baseline --option sel_filter=$SF > $O/c2_sf$SF.json 2> $O/c2_sf$SF.err || { tail $O/c2_sf$SF.err; exit 1; }
  python3 -c "import json; r=json.load(open('$O/c2_sf$SF.json')); print('c2 sf$SF', round(r['value']), round(r['ms_per_step'],3), r.get('verified'), r['config'].get('replayed_queries'))"
done
