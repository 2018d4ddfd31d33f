#!/bin/bash
# VGPR / spill summary of the select kernels (device-only compile, no link)
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Wno-unused-value -Wno-unused-result \
  -I/root/repo/include --cuda-device-only -c /root/repo/weaviate_amd/csrc/runtime.hip -o /tmp/rt_dev.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -A8 "Function Name: .*${1:-select_bf3}" | \
  grep -E "Function Name|VGPRs:|Spill" | sed 's/.*remark: *//' | paste - - - - -
