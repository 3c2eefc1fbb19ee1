#!/bin/bash
# Diagnostic ablation builds of libavc (see AVC_ABLATE in avc_kernels.hip) + a driver per build.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
D=attack-vc_amd/csrc
mkdir -p build/abl
for A in ${ABLS:-1 2 4 8}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -Wno-unused-result -Wno-unused-value -DAVC_ABLATE=$A \
      -Wl,-soname,libavc_abl$A.so -o build/abl/libavc_abl$A.so $D/avc_kernels.hip $D/avc_api.hip &
done
wait
for A in ${ABLS:-1 2 4 8}; do
  hipcc -O2 -std=c++17 -o build/abl/avc_bench_abl$A $D/avc_bench_main.cpp -Lbuild/abl -lavc_abl$A -Wl,-rpath,'$ORIGIN'
done
ls build/abl
