#!/bin/bash
# q8 tests, then option A/B timings on the C3 corpus
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-ab}; mkdir -p $O
if [ -z "$SKIPT" ]; then
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_q8.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
fi
timeout -k 10 300 python -u tools/ab_q8.py --batches 40,64,100,128,200,256 --sets '{"q8_live":0}' '{"q8_live":1}' > $O/ab_live.jsonl 2> $O/ab_live.err; rc=$?
echo "ab live rc=$rc"; cat $O/ab_live.jsonl; [ $rc -eq 0 ] || { tail $O/ab_live.err; exit $rc; }
timeout -k 10 300 python -u tools/ab_q8.py --batches 8192 --reps 6 --rounds 4 --sets '{"q8_prio":0}' '{"q8_prio":1}' > $O/ab_prio.jsonl 2> $O/ab_prio.err; rc=$?
echo "ab prio rc=$rc"; cat $O/ab_prio.jsonl; [ $rc -eq 0 ] || { tail $O/ab_prio.err; exit $rc; }
