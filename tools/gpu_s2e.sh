#!/bin/bash
# parallel replay check: sharded + dynamic tests -> full GPU tests -> shard simulation W=8 (B 2048/4096) -> c3 bench B 2048/4096
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s2e}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded_flat.py tests/test_dynamic.py -x -q --timeout 120 --timeout-method thread > $O/t_shard.log 2>&1; rc=$?
echo "shard tests rc=$rc"; tail -3 $O/t_shard.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/t_shard.log | head -30; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
for b in 2048 4096; do
  timeout -k 10 300 python -u tools/shard_sim.py --world 8 --batch $b > $O/sim_w8_b$b.json 2> $O/sim_w8_b$b.err || { echo "sim failed"; tail -5 $O/sim_w8_b$b.err; exit 1; }
  cat $O/sim_w8_b$b.json
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch $b > $O/bench_c3_b$b.json 2> $O/bench_c3_b$b.err || exit $?; cat $O/bench_c3_b$b.json
done
