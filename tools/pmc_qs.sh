#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over tools/qs_probe.py.
# Usage on the GPU box: bash tools/pmc_qs.sh <outdir> [probe args...]
OUT=${1:-gpurun_out/pmcqs}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum,TCC_MISS_sum" \
           "SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VMEM,SQ_INSTS_SALU,SQ_INSTS_SMEM,GRBM_GUI_ACTIVE,GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc ${grp//,/ } -d "$OUT/p$i" -o run --output-format csv -- python3 tools/qs_probe.py --configs "sel_dbg=0" "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($grp) failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok: $grp"
done
python3 tools/pmc_summary.py "$OUT"
