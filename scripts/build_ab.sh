#!/bin/bash
# A/B builds: libavc + avc_bench from a git revision (default HEAD) into build/ab/<name>/,
# so a working-tree change can be timed against it in the same gpurun call.
set -e
cd "$(dirname $0)/.."
REV=${1:-HEAD}; NAME=${2:-base}
OUT=build/ab/$NAME; SRC=$OUT/tree/attack-vc_amd/csrc
rm -rf $OUT; mkdir -p $SRC $OUT/tree/include
for f in $(git ls-tree --name-only $REV attack-vc_amd/csrc/); do git show $REV:$f > $OUT/tree/$f; done
git show $REV:include/avc.h > $OUT/tree/include/avc.h
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -Wno-unused-value"
for s in $SRC/*.hip; do
  X=""; case $(basename $s) in avc_fused.hip|avc_vc.hip) X="-mllvm --amdgpu-mfma-vgpr-form -mllvm -amdgpu-sched-strategy=max-ilp";; esac
  hipcc $F $X -c -o $OUT/$(basename $s .hip).o $s &
done; wait
hipcc --offload-arch=gfx950 -shared -o $OUT/libavc.so $OUT/*.o
hipcc -O2 -std=c++17 -o $OUT/avc_bench $SRC/avc_bench_main.cpp -L$OUT -lavc -Wl,-rpath,'$ORIGIN'
rm -rf $OUT/*.o
ls $OUT
