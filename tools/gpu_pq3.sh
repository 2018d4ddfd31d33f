#!/bin/bash
O=gpurun_out/${1:-pqab}; mkdir -p $O
timeout -k 10 400 python -u tools/pq_probe.py > $O/probe.log 2>&1 || { cat $O/probe.log; exit 1; }
cat $O/probe.log
