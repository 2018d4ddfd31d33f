#!/bin/bash
O=gpurun_out/${1:-pq4}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pq.py tests/test_gpu_hnsw_flat.py "tests/test_gpu_scale.py::test_c5_pq_960_m240_ks256" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/pq_probe.py > $O/probe.log 2>&1 || { cat $O/probe.log; exit 1; }
cat $O/probe.log
