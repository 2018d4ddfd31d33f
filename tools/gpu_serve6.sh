#!/bin/bash
# serving measurements (tools/serve_bench, C++ caller threads through the
# micro-batcher): C3 unfiltered at 256 callers, 1M rows with 5 % allow lists
# (all callers filtered, then half), the filtered run also under rocprofv3
# kernel + memory-copy traces
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-serve6}; mkdir -p $O
timeout -k 10 120 tools/serve_bench 10000000 256 8 > $O/c3_256.json 2> $O/c3_256.err || { tail $O/c3_256.err; exit 1; }
cat $O/c3_256.json
timeout -k 10 120 tools/serve_bench 1000000 256 8 0 5 100 > $O/f5_all.json 2> $O/f5_all.err || { tail $O/f5_all.err; exit 1; }
cat $O/f5_all.json
timeout -k 10 120 tools/serve_bench 1000000 256 8 0 5 50 > $O/f5_half.json 2> $O/f5_half.err || { tail $O/f5_half.err; exit 1; }
cat $O/f5_half.json
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof_f5 -o run -- tools/serve_bench 1000000 256 4 0 5 100 > $O/prof_f5.log 2>&1 || { tail $O/prof_f5.log; exit 1; }
grep '"qps"' $O/prof_f5.log | tail -1
