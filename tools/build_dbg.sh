#!/bin/bash
# Timing-experiment build (never the product library): qs_runtime.hip with
# -DWV_QS_DBG (k_qs_blockkey / k_q8_blockkey DBG variants behind option sel_dbg,
# results wrong by design), runtime.hip + quant_runtime.hip with -DWV_PQ_DBG
# (PQ ADC timing variants behind option pq_adc3 = 3..5) linked with the product objects into
# weaviate_amd/libwvknn_dbg.so; load it with WV_LIB_PATH=weaviate_amd/libwvknn_dbg.so.
set -e
cd "$(dirname "$0")/.."
python -c "from weaviate_amd import build as b; b.build_library(verbose=False)"
B=weaviate_amd/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wno-unused-value -Wno-unused-result \
  -DWV_QS_DBG -Iinclude -c weaviate_amd/csrc/qs_runtime.hip -o $B/qs_runtime_dbg.o &
for u in runtime quant_runtime; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wno-unused-value -Wno-unused-result \
    -DWV_PQ_DBG -Iinclude -c weaviate_amd/csrc/$u.hip -o $B/${u}_dbg.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $B/runtime_dbg.o $B/qs_runtime_dbg.o $B/qs_exact.o $B/qs_replay.o \
  $B/quant_runtime_dbg.o -o weaviate_amd/libwvknn_dbg.so
echo built weaviate_amd/libwvknn_dbg.so
