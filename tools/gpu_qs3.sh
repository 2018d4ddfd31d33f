#!/bin/bash
# block-key path: smoke -> C3 probe + verify -> C2-shaped probe + verify
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-qs3}; mkdir -p $O
timeout -k 10 120 python -u tools/qs_smoke.py > $O/smoke.log 2>&1; rc=$?
cat $O/smoke.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/qs_probe.py --configs "sel_dbg=0" > $O/probe_c3.log 2>&1; rc=$?
grep -v amdgpu.ids $O/probe_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/qs_probe.py --configs "sel_dbg=0" --n 1000000 --d 128 --k 100 --batch 10000 --metric l2-squared --kind 1 > $O/probe_c2.log 2>&1; rc=$?
grep -v amdgpu.ids $O/probe_c2.log; exit $rc
