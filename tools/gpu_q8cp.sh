#!/bin/bash
# int8-only planes above 1536 dims: parity tests, then 10M x {1024, 2048, 3072} cosine benches under rocprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-q8cp}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_q8.py -k "above_1536 or nonfinite" "tests/test_gpu_flat.py::test_gemv_small_batches" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for D in ${DIMS:-1024 2048 3072}; do
  N=10000000; [ $D -ge 3072 ] && N=${N3072:-10000000}
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof_d$D -o run --output-format csv -- python3 bench.py --dims $D --n $N --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_d$D.json 2> $O/bench_d$D.err || { tail $O/bench_d$D.err; exit 1; }
  python3 -c "import json; r=json.load(open('$O/bench_d$D.json')); ro=r['roofline']; print('d$D', round(r['value']), round(r['ms_per_step'],2), ro.get('kernel'), round(ro.get('launch_ms') or 0,2), round(ro.get('frac') or 0,3), round(ro.get('bf16_peak_equivalent_frac') or 0,3), r.get('verified'))"
  python3 tools/kstats.py $O/prof_d$D/run_kernel_stats.csv > $O/kernel_stats_d$D.txt; head -8 $O/kernel_stats_d$D.txt
done
