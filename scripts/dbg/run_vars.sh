#!/bin/bash
# Time libavc variants (scripts/dbg/var/*) with avc_bench: VARS="main noA ..." ARGS="256 128 200 1 1 1 0"
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in ${VARS:-main}; do
  if [ "$v" = main ]; then b=attack-vc_amd/avc_bench; else b=scripts/dbg/var/$v/avc_bench; fi
  echo "=== $v"
  timeout -k 10 300 $b ${ARGS:-256 128 200 1 1 1 0} > gpurun_out/var_$v.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/var_$v.log | grep -v "^fwd\|^bwd" | head -20
  [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
done
