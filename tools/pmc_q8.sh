#!/bin/bash
# busy / wait / LDS / HBM counters of the int8 block-key kernel on C3 (B = 8192), one pass per group
OUT=${1:-gpurun_out/pmcq8}
B=${2:-8192}
CFG=${3:-q8=1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
i=0
for grp in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_INSTS_VALU SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- python3 tools/qs_probe.py --verify 0 --batch $B --configs "$CFG" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
cat "$OUT/summary.txt" | grep -E "q8_blockkey|blk_exact|blk_select" | cut -c1-600
