#!/bin/bash
# scripts/dbg/build_variant.sh NAME "extra hipcc flags" : libavc + avc_bench with the fused
# kernel sources (avc_fused.hip, avc_vc.hip) compiled with extra flags, in scripts/dbg/NAME/
set -e
cd "$(dirname "$0")/../.."
C=attack-vc_amd/csrc; D=scripts/dbg/$1; mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $2 -c $C/avc_fused.hip -o $D/avc_fused.o &
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $2 -c $C/avc_vc.hip -o $D/avc_vc.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libavc.so $C/avc_gemm.hip.o $D/avc_fused.o $D/avc_vc.o $C/avc_api.hip.o $C/avc_kernels.hip.o
/opt/rocm/bin/hipcc -O2 -std=c++17 -o $D/avc_bench $C/avc_bench_main.cpp -L$D -lavc -Wl,-rpath,'$ORIGIN'
rm -f $D/*.o
