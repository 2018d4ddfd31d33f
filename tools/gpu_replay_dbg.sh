#!/bin/bash
# C2 replay clock diagnostics (k_blk_replay DBG instantiation)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3g}; mkdir -p $O
timeout -k 10 300 python3 bench.py --workload c2 --no-cpu-baseline --no-verify --steps 1 --warmup 0 --option replay_dbg=1 > $O/c2_dbg.out 2> $O/c2_dbg.err || { tail $O/c2_dbg.err; exit 1; }
grep "k_blk_replay dbg" $O/c2_dbg.out | head -12
