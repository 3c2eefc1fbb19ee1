#!/bin/bash
# build/ab/NAME: libavc + avc_bench with the fused kernel sources (avc_fused.hip,
# avc_vc.hip) compiled with extra hipcc flags $2, the other objects from the in-tree
# build; timed against the in-tree build by scripts/ab.sh.
set -e
cd "$(dirname "$0")/../.."
C=attack-vc_amd/csrc; D=build/ab/$1; mkdir -p $D
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -Wno-unused-value -mllvm --amdgpu-mfma-vgpr-form"  # + $2 (a -amdgpu-sched-strategy replaces the in-tree max-ilp)
/opt/rocm/bin/hipcc $F $2 -c $C/avc_fused.hip -o $D/avc_fused.o &
/opt/rocm/bin/hipcc $F $2 -c $C/avc_vc.hip -o $D/avc_vc.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libavc.so $C/avc_gemm.hip.o $D/avc_fused.o $D/avc_vc.o \
    $C/avc_kernels.hip.o $C/avc_pm.hip.o $C/avc_dsp.hip.o $C/avc_api.hip.o
/opt/rocm/bin/hipcc -O2 -std=c++17 -o $D/avc_bench $C/avc_bench_main.cpp -L$D -lavc -Wl,-rpath,'$ORIGIN'
rm -f $D/*.o
