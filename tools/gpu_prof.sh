#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py (args passed through) + host CPU facts
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-prof}; shift; mkdir -p $O
cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $O/bench_prof.json 2> $O/bench_prof.err; rc=$?
echo "prof rc=$rc"; cat $O/bench_prof.json
find $O/prof -name '*kernel_stats.csv' -exec head -14 {} \;
exit $rc
