#!/bin/bash
# round-3 8-shard prediction for C3 at the bench batch (tools/shard_sim.py: the C3
# corpus as 8 shards on one GPU, every stage timed per shard), plus BQ's
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-ssim}; mkdir -p $O
timeout -k 10 600 python3 tools/shard_sim.py --batch 8192 > $O/w8_b8192.json 2> $O/w8_b8192.err || { tail -5 $O/w8_b8192.err; exit 1; }
cat $O/w8_b8192.json
timeout -k 10 600 python3 tools/shard_sim_bq.py > $O/bq_w8.json 2> $O/bq_w8.err || { tail -5 $O/bq_w8.err; exit 1; }
cat $O/bq_w8.json
