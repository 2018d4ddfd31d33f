#!/bin/bash
# round-6 PMC records: C3 int8 key pass (clock, MFMA busy, LDS, HBM), the PQ int8 route's traffic
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-pmc6}; mkdir -p $O
bash tools/pmc_q8.sh $O/c3 8192 "q8=1" > $O/c3.txt 2>&1; rc=$?
cat $O/c3.txt | cut -c1-300; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_traffic.sh $O/pq --workload pq > $O/pq.txt 2>&1; rc=$?
cat $O/pq.txt; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py $O/pq > $O/pq_summary.txt; grep -E "q8_blockkey|pq" $O/pq_summary.txt | cut -c1-400
