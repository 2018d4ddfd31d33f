#!/bin/bash
# k_pq_adc4 as the default: PQ parity tests; adc4 / adc4-without-DMA / adc3 timing (debug library)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-pq4b}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pq.py tests/test_gpu_sharded_threads.py -k "pq or PQ" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
WV_LIB_PATH=weaviate_amd/libwvknn_dbg.so timeout -k 10 500 python3 -u tools/pq_probe.py ${PROBE:-pq_adc3=2 pq_adc3=5 pq_adc3=1 pq_adc3=3 pq_adc3=2 pq_adc3=5} > $O/probe.txt 2>&1; rc=$?
cat $O/probe.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
