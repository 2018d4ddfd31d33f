#!/bin/bash
# BQ replay-free answers (k_bq_fast): every BQ GPU test, then C4 with bq_fast 0 / 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-bqfast}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -k "bq or BQ or c4" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
for v in ${BQV:-0 1}; do
timeout -k 10 400 python -u bench.py --workload bq --option bq_fast=$v --no-cpu-baseline > $O/bq_fast$v.json 2> $O/bq_fast$v.err; rc=$?
echo "bq_fast=$v rc=$rc"; python3 -c "import json,sys; d=json.loads(open('$O/bq_fast$v.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('verified'), d['roofline'].get('pipeline_ms'))"; [ $rc -eq 0 ] || { tail $O/bq_fast$v.err; exit $rc; }
done
