#!/bin/bash
# replay rework check: targeted GPU tests -> full GPU tests -> c3/c2 bench -> per-rank (1.25M shard) bench + rocprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -x -q --timeout 120 --timeout-method thread -k "replay" > $O/t_replay.log 2>&1; rc=$?
echo "replay tests rc=$rc"; tail -3 $O/t_replay.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/t_replay.log | head -20; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit $?; cat $O/bench_c3.json
timeout -k 10 300 python -u bench.py --workload c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit $?; cat $O/bench_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_n8 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --n 1250000 > $O/bench_n8shard.json 2> $O/bench_n8shard.err || exit $?
cat $O/bench_n8shard.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --workload c2 --no-cpu-baseline > $O/bench_c2_prof.json 2> $O/bench_c2_prof.err || exit $?
