#!/bin/bash
# full GPU tests -> c3 bench B 2048 / 4096 -> PMC traffic passes (c3) -> kernel stats of the 8-shard simulation
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s2f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
for b in 2048 4096; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch $b > $O/bench_c3_b$b.json 2> $O/bench_c3_b$b.err || exit $?; cat $O/bench_c3_b$b.json
done
bash tools/pmc_traffic.sh $O/pmc || exit $?
python3 tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt; cat $O/pmc_summary.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_sim -o run --output-format csv -- python3 tools/shard_sim.py --world 8 --reps 2 > $O/sim_prof.json 2> $O/sim_prof.err || exit $?
cat $O/sim_prof.json
