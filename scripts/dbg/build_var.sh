#!/bin/bash
# libavc timing variant: avc_fused.hip (and optionally avc_vc.hip / avc_long.hip) rebuilt with
# extra flags, linked with the main build's other objects, into scripts/dbg/var/NAME/.
#   scripts/dbg/build_var.sh NAME "-DAVC_FZ_ABLATE=1" [sources...]
set -e
cd "$(dirname "$0")/../.."
C=attack-vc_amd/csrc; N=$1; X=$2; shift 2
SRCS=${@:-avc_fused.hip}
D=scripts/dbg/var/$N; mkdir -p $D
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -Wno-unused-value -mllvm --amdgpu-mfma-vgpr-form ${SCHED--mllvm -amdgpu-sched-strategy=max-ilp} -DAVC_SRC_HASH=\"var-$N\""
OBJS=""
for s in avc_gemm avc_kernels avc_fused avc_vc avc_long avc_pm avc_dsp avc_api; do
  if [[ " $SRCS " == *" $s.hip "* ]]; then
    /opt/rocm/bin/hipcc $FL $X -c $C/$s.hip -o $D/$s.o
    OBJS="$OBJS $D/$s.o"
  else
    OBJS="$OBJS $C/$s.hip.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libavc.so $OBJS
/opt/rocm/bin/hipcc -O2 -std=c++17 -o $D/avc_bench $C/avc_bench_main.cpp -L$D -lavc -Wl,-rpath,'$ORIGIN'
rm -f $D/*.o
echo built $D
