#!/bin/bash
# Build libavc variants with se_head_v ablations (AVC_HEAD_ABLATE bits: 1 = no weight
# loads, 2 = no LDS input reads) into scripts/dbg/headN/, each with its own avc_bench.
set -e
cd "$(dirname "$0")/../.."
C=attack-vc_amd/csrc
for V in 1 2 3; do
  D=scripts/dbg/head$V; mkdir -p $D
  for f in avc_gemm avc_fused avc_api; do cp $C/$f.hip.o $D/ 2>/dev/null || true; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DAVC_HEAD_ABLATE=$V -c $C/avc_kernels.hip -o $D/avc_kernels.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libavc.so $C/avc_gemm.hip.o $C/avc_fused.hip.o $C/avc_api.hip.o $D/avc_kernels.o
  /opt/rocm/bin/hipcc -O2 -std=c++17 -o $D/avc_bench $C/avc_bench_main.cpp -L$D -lavc -Wl,-rpath,'$ORIGIN'
done
