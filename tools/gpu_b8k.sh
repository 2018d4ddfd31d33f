#!/bin/bash
# block-key throughput at B = 4096 vs 8192 (C3)
O=gpurun_out/b8k; mkdir -p $O
timeout -k 10 300 python -u tools/qs_probe.py --batch 4096 --verify 0 --configs "sel_dbg=0;sel_dbg=0" > $O/b4096.log 2>&1 || { cat $O/b4096.log; exit 1; }
timeout -k 10 300 python -u tools/qs_probe.py --batch 8192 --configs "sel_dbg=0;sel_dbg=0" > $O/b8192.log 2>&1 || { cat $O/b8192.log; exit 1; }
cat $O/b4096.log $O/b8192.log
