#!/bin/bash
# libavc variant with AVC_FZ_ABLATE=4 (no cross-GEMM A prefetch) in scripts/dbg/fz4/
set -e
cd "$(dirname "$0")/../.."
C=attack-vc_amd/csrc; D=scripts/dbg/fz4; mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DAVC_FZ_ABLATE=4 -c $C/avc_fused.hip -o $D/avc_fused.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libavc.so $C/avc_gemm.hip.o $D/avc_fused.o $C/avc_api.hip.o $C/avc_kernels.hip.o
