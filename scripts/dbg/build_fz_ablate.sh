#!/bin/bash
# libavc variants with fused-engine timing ablations (AVC_FZ_ABLATE bits) in scripts/dbg/fzN/
set -e
cd "$(dirname "$0")/../.."
C=attack-vc_amd/csrc
for V in 1 2 3; do
  D=scripts/dbg/fz$V; mkdir -p $D
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DAVC_FZ_ABLATE=$V -c $C/avc_fused.hip -o $D/avc_fused.o &
done
wait
for V in 1 2 3; do
  D=scripts/dbg/fz$V
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libavc.so $C/avc_gemm.hip.o $D/avc_fused.o $C/avc_api.hip.o $C/avc_kernels.hip.o
  /opt/rocm/bin/hipcc -O2 -std=c++17 -o $D/avc_bench $C/avc_bench_main.cpp -L$D -lavc -Wl,-rpath,'$ORIGIN'
done
