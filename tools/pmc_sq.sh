#!/bin/bash
# SQ / LDS utilisation counters of the bench's kernels (one rocprofv3 pass per group).
OUT=${1:-gpurun_out/pmcsq}; shift
ARGS="$@"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT -d "$OUT/sq" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $ARGS > "$OUT/sq.log" 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL -d "$OUT/lds" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $ARGS > "$OUT/lds.log" 2>&1 || exit $?
echo "pmc sq ok"
