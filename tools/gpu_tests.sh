#!/bin/bash
# full GPU test suite + smoke on the current tree
O=gpurun_out/${1:-tests}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
