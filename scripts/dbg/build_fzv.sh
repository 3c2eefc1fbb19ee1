#!/bin/bash
# libavc variant scripts/dbg/fzv$1 with -DAVC_FZ_ABLATE=$1
set -e
cd "$(dirname "$0")/../.."
C=attack-vc_amd/csrc; D=scripts/dbg/fzv$1; mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DAVC_FZ_ABLATE=$1 -c $C/avc_fused.hip -o $D/avc_fused.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libavc.so $C/avc_gemm.hip.o $D/avc_fused.o $C/avc_api.hip.o $C/avc_kernels.hip.o
rm $D/avc_fused.o
