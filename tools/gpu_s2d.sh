#!/bin/bash
# sharded two-phase check: sharded tests -> full GPU tests -> shard simulation (W=8, 4, 2) -> c3 bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s2d}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded_flat.py -x -q --timeout 120 --timeout-method thread > $O/t_shard.log 2>&1; rc=$?
echo "shard tests rc=$rc"; tail -3 $O/t_shard.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/t_shard.log | head -30; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
for w in 8 4 2; do
  timeout -k 10 300 python -u tools/shard_sim.py --world $w > $O/sim_w$w.json 2> $O/sim_w$w.err || { echo "sim w$w failed"; tail -5 $O/sim_w$w.err; exit 1; }
  cat $O/sim_w$w.json
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit $?; cat $O/bench_c3.json
