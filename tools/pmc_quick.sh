#!/bin/bash
# two PMC passes (SQ utilisation, FETCH_SIZE) over a reduced bench
OUT=${1:-gpurun_out/pmcq}; shift
ARGS=${@:---n 2000000 --steps 1 --warmup 1 --no-cpu-baseline}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d "$OUT/sq" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/sq.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT TCC_MISS -d "$OUT/lds" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/lds.log" 2>&1
echo "pmc exit $?"
