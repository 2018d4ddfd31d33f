#!/bin/bash
# capped exact selection: flat / sharded / scale GPU tests, then C2 / C3 / C1 A/B (exact_cap 0/1) in one process each
O=gpurun_out/${1:-cap}; mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_flat.py tests/test_gpu_sharded_flat.py tests/test_gpu_scale.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/qs_probe.py --n 1000000 --d 128 --k 100 --batch 10000 --metric l2-squared --kind 1 --verify 0 --configs "exact_cap=0;exact_cap=1;exact_cap=0;exact_cap=1" > $O/c2.log 2>&1 || { cat $O/c2.log; exit 1; }
cat $O/c2.log
timeout -k 10 300 python -u tools/qs_probe.py --batch 8192 --verify 0 --configs "exact_cap=0;exact_cap=1;exact_cap=0;exact_cap=1" > $O/c3.log 2>&1 || { cat $O/c3.log; exit 1; }
cat $O/c3.log
timeout -k 10 300 python -u tools/qs_probe.py --n 100000 --d 128 --k 10 --batch 1000 --metric l2-squared --kind 0 --verify 0 --configs "exact_cap=0;exact_cap=1;exact_cap=0;exact_cap=1" > $O/c1.log 2>&1 || { cat $O/c1.log; exit 1; }
cat $O/c1.log
