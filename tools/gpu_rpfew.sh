#!/bin/bash
# replay form for small batches: pooled (rp_few 16) vs one-launch 8-wave (rp_few 1024)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-rpfew}; mkdir -p $O
timeout -k 10 400 python -u tools/ab_q8.py --batches 64,128,256,512 --reps 10 --rounds 3 --sets '{"rp_few":16}' '{"rp_few":1024}' > $O/ab.jsonl 2> $O/ab.err; rc=$?
echo "ab rc=$rc"; cat $O/ab.jsonl; [ $rc -eq 0 ] || { tail $O/ab.err; exit $rc; }
