#!/bin/bash
# per-kernel breakdown of medium C3 batches (B = 64 and 256, one process each,
# ab_q8.py's default option set) under rocprofv3 kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-small6}; mkdir -p $O
for B in ${BATCHES:-64 256}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/b$B -o run -- \
        python3 tools/ab_q8.py --batches $B --rounds 2 > $O/b$B.log 2>&1 || { cat $O/b$B.log | tail -20; exit 1; }
    tail -2 $O/b$B.log
    python3 tools/kstats.py $O/b$B 2>/dev/null | head -25 || true
done
