#!/bin/bash
# VGPR / AGPR / spill summary of the fused kernels (kernel-resource-usage remarks)
cd "$(dirname "$0")/.."
F=${1:-avc_fused.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm --amdgpu-mfma-vgpr-form -mllvm -amdgpu-sched-strategy=max-ilp \
  -Rpass-analysis=kernel-resource-usage -c attack-vc_amd/csrc/$F -o /tmp/res_$$.o 2>&1 |
  grep -E "Function Name|VGPRs|AGPRs|Spill|Scratch" | sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//' |
  awk '/Function Name/{printf "\n%s", $3; next}{printf " | %s", $0}' | grep -E "${2:-Li0E}"
rm -f /tmp/res_$$.o
