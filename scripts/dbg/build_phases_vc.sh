#!/bin/bash
# libavc variant with per-phase cycle stamps in the fused Decoder kernels (-DAVC_FZ_PHASES) in scripts/dbg/phv/
set -e
cd "$(dirname "$0")/../.."
C=attack-vc_amd/csrc; D=scripts/dbg/${PHDIR:-phv}; mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm --amdgpu-mfma-vgpr-form -mllvm -amdgpu-sched-strategy=max-ilp -DAVC_FZ_PHASES -DFZ_PH_MAX=160 ${EXTRA:-} -c $C/avc_vc.hip -o $D/avc_vc.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libavc.so $C/avc_gemm.hip.o $C/avc_fused.hip.o $D/avc_vc.o $C/avc_long.hip.o $C/avc_pm.hip.o $C/avc_dsp.hip.o $C/avc_api.hip.o $C/avc_kernels.hip.o
/opt/rocm/bin/hipcc -O2 -std=c++17 -o $D/avc_bench $C/avc_bench_main.cpp -L$D -lavc -Wl,-rpath,'$ORIGIN'
rm $D/avc_vc.o
