#!/bin/bash
# register / spill summary of every kernel in one source: res_usage_file.sh <file.hip> [extra hipcc flags]
f=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm --amdgpu-mfma-vgpr-form -mllvm -amdgpu-sched-strategy=max-ilp "$@" -c $f -o /tmp/res_usage.o -Rpass-analysis=kernel-resource-usage 2>&1 | \
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis.*//' | \
  awk -F': ' '/^Function Name/ {fn=$2} /^VGPRs$/ {} $1=="VGPRs" {v=$2} $1=="AGPRs" {a=$2} $1=="ScratchSize [bytes/lane]" {sc=$2} $1=="SGPRs Spill" {ss=$2} $1=="VGPRs Spill" {print fn, "v="v, "a="a, "scratch="sc, "sgpr_spill="ss, "vgpr_spill="$2}'
