#!/bin/bash
# clock / MFMA-busy / wait counters for the block-key kernel at several DBG settings
OUT=${1:-gpurun_out/pmcqs2}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
for dbg in 0 6 3; do
  timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU -d "$OUT/d$dbg" -o run --output-format csv -- python3 tools/qs_probe.py --verify 0 --configs "sel_dbg=$dbg" > "$OUT/d$dbg.log" 2>&1 || { echo "dbg $dbg failed"; tail -5 "$OUT/d$dbg.log"; exit 1; }
  echo "dbg $dbg ok"
done
python3 tools/pmc_summary.py "$OUT"
