#!/bin/bash
# HBM traffic of the bench's dominant kernel from PMC counters: one rocprofv3
# pass per counter group (FETCH_SIZE, then WRITE_SIZE), as MI355X_MICROARCH.md
# prescribes (no --pmc with traces).  Usage on the GPU box:
#   bash tools/pmc_traffic.sh <outdir> [bench args...]
OUT=${1:-gpurun_out/pmc}; shift
ARGS="$@"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $ARGS > "$OUT/write.log" 2>&1 || exit $?
echo "pmc ok"
