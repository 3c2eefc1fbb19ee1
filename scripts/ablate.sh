#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for b in attack-vc_amd/avc_bench ${ABL_BINS:-build/abl/avc_bench_abl5 build/abl/avc_bench_abl16 build/abl/avc_bench_abl32 build/abl/avc_bench_abl37}; do
  echo "=== $b"
  timeout -k 10 300 $b 256 128 100 1 1 > gpurun_out/abl_$(basename $b).log 2>&1
  rc=$?; cat gpurun_out/abl_$(basename $b).log | grep -v amdgpu.ids
  [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
done
