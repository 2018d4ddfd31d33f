#!/bin/bash
# k_qs_blockkey_w4 (d > 768) + the minima-only PQ search: parity tests, benches (d = 1024 / 1536 with
# kernel stats, C5 PQ with both search forms), then PMC passes of the d = 1024 kernel
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-w4}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_pq.py tests/test_gpu_hnsw_flat.py tests/test_gpu_scale.py -m gpu -x -v -k "above_768 or select_kernel or proof_bound or removed or pq" --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json,sys; r=json.load(open('$1')); print('$2', round(r['value']), 'qps', round(r['ms_per_step'],2), 'ms', r['roofline'].get('launch_ms'), r['roofline'].get('frac'), r.get('verified'))"; }
for D in 1024 1536; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$D -o run --output-format csv -- python3 bench.py --dims $D --no-cpu-baseline > $O/bench_$D.json 2> $O/bench_$D.err || { tail $O/bench_$D.err; exit 1; }
summ $O/bench_$D.json d=$D
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_pq -o run --output-format csv -- python3 bench.py --workload pq --no-cpu-baseline > $O/bench_pq.json 2> $O/bench_pq.err || { tail $O/bench_pq.err; exit 1; }
summ $O/bench_pq.json pq_cand
timeout -k 10 300 python3 bench.py --workload pq --no-cpu-baseline --option pq_cand=0 > $O/bench_pq0.json 2> $O/bench_pq0.err || { tail $O/bench_pq0.err; exit 1; }
summ $O/bench_pq0.json pq_matrix
# C2 (k = 100, integer ties): one-wave replay vs the pooled replay with a pool large enough for every flagged query
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --workload c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
summ $O/bench_c2.json c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2p -o run --output-format csv -- python3 bench.py --workload c2 --no-cpu-baseline --option replay_par=3 --option rp_pool=16777216 > $O/bench_c2p.json 2> $O/bench_c2p.err || { tail $O/bench_c2p.err; exit 1; }
summ $O/bench_c2p.json c2_pooled
i=0
for grp in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$O/pmc$i" -o run --output-format csv -- python3 tools/qs_probe.py --d 1024 --verify 0 --batch 8192 --configs "timing=1" > "$O/pmc$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$O/pmc$i.log"; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_summary.py "$O" > "$O/pmc_summary.txt" 2>&1; head -40 "$O/pmc_summary.txt"
