#!/bin/bash
# VGPR/SGPR/spill/occupancy report of the hot kernels (compile-time remarks, no GPU).
#   usage: tools/resource_usage.sh [kernel-name-regex]
cd "$(dirname "$0")/../kubernetes-scheduler_amd/csrc"
PAT=${1:-"k1_block_n32|k2_block_n32"}
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize \
  --cuda-device-only -c -o /tmp/yk.o yoda_kernels.hip -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk -v pat="$PAT" '/Function Name:/ {show = ($0 ~ pat)} show && /remark/ {sub(/.*remark: /, ""); print}' |
  grep -E "Function Name|VGPRs:|SGPRs:|Spill|Occupancy|LDS" 
