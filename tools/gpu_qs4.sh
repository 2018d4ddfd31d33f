#!/bin/bash
# decomposition probe + c1/c2/c3 bench lines
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-qs4}; mkdir -p $O
timeout -k 10 300 python -u tools/qs_probe.py --verify 0 --configs "sel_dbg=0;sel_dbg=1;sel_dbg=2;sel_dbg=4;sel_dbg=6;sel_dbg=3;sel_dbg=5;sel_dbg=0" > $O/probe.log 2>&1; rc=$?
grep -v amdgpu.ids $O/probe.log; [ $rc -eq 0 ] || exit $rc
for w in c1 c2 c3; do
  timeout -k 10 300 python -u bench.py --workload $w $([ $w = c1 ] || echo --no-cpu-baseline) > $O/bench_$w.json 2> $O/bench_$w.err; rc=$?
  echo "bench $w rc=$rc"; cat $O/bench_$w.json; [ $rc -eq 0 ] || { tail -5 $O/bench_$w.err; exit $rc; }
done
