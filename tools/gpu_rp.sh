#!/bin/bash
O=gpurun_out/${1:-rp}; mkdir -p $O
timeout -k 10 400 python -u tools/qs_probe.py --n 1000000 --d 128 --k 100 --batch 10000 --metric l2-squared --kind 1 --verify 0 --configs "replay_par=2;replay_par=3,rp_pool=8388608;replay_par=3,rp_pool=33554432;replay_par=1;replay_par=2" > $O/c2_rp.log 2>&1 || { cat $O/c2_rp.log; exit 1; }
cat $O/c2_rp.log
