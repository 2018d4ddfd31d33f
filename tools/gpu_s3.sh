#!/bin/bash
# evidence run at the C3 default B=8192: bench (cpu baseline), kernel stats, PMC traffic,
# clock / MFMA-busy counters, 8-shard simulation
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s3}; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit $?; cat $O/bench_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_c3_prof.json 2> $O/bench_c3_prof.err || exit $?
bash tools/pmc_traffic.sh $O/pmc_c3 || exit $?
python3 tools/pmc_summary.py $O/pmc_c3 > $O/pmc_c3_summary.txt; cat $O/pmc_c3_summary.txt
bash tools/pmc_qs3.sh $O/pmcqs3 8192 || exit $?
cat $O/pmcqs3/summary.txt
timeout -k 10 400 python -u tools/shard_sim.py --world 8 --batch 8192 > $O/shard_w8_b8192.json 2> $O/shard.err || exit $?; cat $O/shard_w8_b8192.json
