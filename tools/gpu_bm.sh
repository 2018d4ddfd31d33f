#!/bin/bash
# block-major exact: parity tests, then C2 / C1 / C3 A/B in one process each
O=gpurun_out/${1:-bm}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_flat.py -k "block_major or search_matches_oracle or replay" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/qs_probe.py --n 1000000 --d 128 --k 100 --batch 10000 --metric l2-squared --kind 1 --verify 0 --configs "exact_bm=0;exact_bm=1;exact_bm=0;exact_bm=1" > $O/c2.log 2>&1 || { cat $O/c2.log; exit 1; }
cat $O/c2.log
timeout -k 10 300 python -u tools/qs_probe.py --n 100000 --d 128 --k 10 --batch 1000 --metric l2-squared --kind 0 --verify 0 --configs "exact_bm=0;exact_bm=1;exact_bm=0;exact_bm=1" > $O/c1.log 2>&1 || { cat $O/c1.log; exit 1; }
cat $O/c1.log
