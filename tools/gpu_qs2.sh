#!/bin/bash
# block-key path: smoke -> timing probe variants
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-qs2}; shift; mkdir -p $O
timeout -k 10 120 python -u tools/qs_smoke.py > $O/smoke.log 2>&1; rc=$?
cat $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/qs_probe.py "$@" > $O/probe.log 2>&1; rc=$?
cat $O/probe.log | grep -v amdgpu.ids
exit $rc
