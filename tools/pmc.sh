#!/bin/bash
# PMC passes over a reduced bench (2M rows: corpus 6 GB > Infinity Cache), one
# counter group per rocprofv3 run (gpurun/pool rules: no --pmc with traces).
# Usage (on the GPU box): bash tools/pmc.sh <outdir> [bench args...]
set -o pipefail
OUT=${1:-gpurun_out/pmc}; shift
ARGS=${@:---n 2000000 --steps 1 --warmup 1 --no-cpu-baseline}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
run() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1
}
run sq   SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE TCC_HIT TCC_MISS && \
run lds  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_UNALIGNED_STALL SQ_INSTS_SALU SQ_WAIT_INST_LDS
echo "pmc exit $?"
