#!/bin/bash
# the N > 1 code path (wv_multi over RCCL, one process per GPU) at world 1 for
# every workload, under torch.distributed.run; --sharded also checks the
# result equals the single-index search
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-sh6}; mkdir -p $O
for w in c3 c2 c1 bq pq rq8 rq1; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --gpus 1 --sharded --no-cpu-baseline --steps 3 --warmup 1 --workload $w \
        > $O/$w.json 2> $O/$w.err || { echo "$w failed"; tail -5 $O/$w.err; exit 1; }
    python3 -c "import json; r=json.loads(open('$O/$w.json').read().strip().splitlines()[-1]); print('$w', round(r['value']), r['config'].get('sharded_check', r.get('sharded_check')), r['config'].get('parallelism'))"
done
