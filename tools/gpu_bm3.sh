#!/bin/bash
# block-major exact on by default: GPU tests, C1 / C2 A/B, bench c1 / c2, full suite
O=gpurun_out/${1:-bm3}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/qs_probe.py --n 100000 --d 128 --k 10 --batch 1000 --metric l2-squared --kind 0 --verify 0 --configs "exact_bm=0;exact_bm=1;exact_bm=0;exact_bm=1;exact_bm=0;exact_bm=1" > $O/c1_bm.log 2>&1 || { cat $O/c1_bm.log; exit 1; }
cat $O/c1_bm.log
for w in c2 c1; do
  timeout -k 10 300 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
done
