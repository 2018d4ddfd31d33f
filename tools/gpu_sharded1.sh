#!/bin/bash
# the N>1 bench protocol (ShardedFlatSearch / ShardedBQSearch over RCCL) at WORLD_SIZE 1 on one GPU
O=gpurun_out/${1:-sh1}; mkdir -p $O
run() {
  local name=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --sharded --no-cpu-baseline --steps 3 --warmup 1 "$@" > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }
  cat $O/$name.json; grep -h "equals" $O/$name.err || true
}
run c3
run c2 --workload c2
run c1 --workload c1
run bq --workload bq
