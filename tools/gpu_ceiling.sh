#!/bin/bash
# vendor-GEMM ceiling vs the block-key kernel on the same box
O=gpurun_out/${1:-ceil}; mkdir -p $O
timeout -k 10 200 python -u tools/gemm_ceiling.py > $O/gemm.json 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
cat $O/gemm.json
timeout -k 10 300 python -u tools/qs_probe.py --batch 8192 --verify 0 --configs "sel_dbg=0;sel_dbg=0" > $O/probe.log 2>&1 || { cat $O/probe.log; exit 1; }
cat $O/probe.log


