#!/bin/bash
# VGPR / SGPR / spill / LDS / occupancy report of the kernels file for gfx950 (compile only, no GPU):
#   bash scripts/resource_usage.sh [kernel-name-regex] [extra -D flags...]
R=$(cd "$(dirname "$0")/.." && pwd)
PAT=${1:-k_sweep}
shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-gpu-flush-denormals-to-zero \
  -mllvm -amdgpu-atomic-optimizer-strategy=None -I$R/include -I$R/goworld_amd/csrc "$@" --cuda-device-only -c \
  -Rpass-analysis=kernel-resource-usage $R/goworld_amd/csrc/gwaoi_kernels.hip -o /tmp/ru_$$.o 2>&1 |
  grep -A12 -E "Function Name: .*($PAT)" | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size|SGPRs:" 
rm -f /tmp/ru_$$.o
