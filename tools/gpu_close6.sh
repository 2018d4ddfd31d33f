#!/bin/bash
# closing check on the final tree: C3 bench line, serving at the library's default window
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-close6}; mkdir -p $O
timeout -k 10 420 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 1; }
tail -c 400 $O/bench_c3.json
timeout -k 10 150 tools/serve_bench 10000000 256 8 > $O/serve_c3_256.json 2> $O/serve_c3_256.err || { tail $O/serve_c3_256.err; exit 1; }
cat $O/serve_c3_256.json
timeout -k 10 150 tools/serve_bench 10000000 512 6 > $O/serve_c3_512.json 2> $O/serve_c3_512.err || { tail $O/serve_c3_512.err; exit 1; }
cat $O/serve_c3_512.json
timeout -k 10 120 tools/serve_bench 1000000 256 6 1000 5 50 > $O/f5_half.json 2> $O/f5_half.err || { tail $O/f5_half.err; exit 1; }
cat $O/f5_half.json
