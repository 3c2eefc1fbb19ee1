#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
AVC_PROFILE_ROLES=1 timeout -k 10 300 ./attack-vc_amd/avc_bench 256 128 50 1 1 2>&1 | grep -v amdgpu.ids | tee gpurun_out/roles.log
