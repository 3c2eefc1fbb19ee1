#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for P in 0 1; do
AVC_PROFILE_ROLES=1 timeout -k 10 300 ./attack-vc_amd/avc_bench 256 128 50 1 1 $P 2>&1 | grep -v amdgpu.ids > gpurun_out/roles_$P.log || exit 1
done
cat gpurun_out/roles_0.log gpurun_out/roles_1.log
