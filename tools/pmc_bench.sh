#!/bin/bash
# busy / wait / LDS / HBM counters of a bench workload's kernels, one
# rocprofv3 --pmc pass per counter group (no traces), summary per kernel.
# Usage on the GPU box: bash tools/pmc_bench.sh <outdir> [bench args...]
OUT=${1:-gpurun_out/pmcb}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
i=0
for grp in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_INSTS_VALU SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
