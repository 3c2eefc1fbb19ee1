#!/bin/bash
# Long-engine iteration: GPU tests of the long / generic-length paths, an interleaved A/B of the
# T=400 emb attack against scripts/dbg/var/base (build it from an older checkout with
# scripts/dbg/build_var.sh base "" avc_long.hip, or name other variants in LZ_VARS), and the phase
# stamps of scripts/dbg/phl (scripts/dbg/build_phases_long.sh) when built.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${LZ_TESTS:-tests/test_gpu_long.py tests/test_gpu_lengths.py tests/test_gpu_lrelu.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lz_tests.log 2>&1
rc=$?; tail -2 gpurun_out/lz_tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAILED" gpurun_out/lz_tests.log | head; exit $rc; }
IFS=';' read -ra ARGL <<< "${LZ_ARGS:-256 400 200 1 1 1 0}"
for args in "${ARGL[@]}"; do
  echo "== avc_bench $args"
  VARS="${LZ_VARS:-base}" ARGS="$args" REPS=${LZ_REPS:-2} bash scripts/abv.sh || exit 1
done
if [ -x scripts/dbg/phl/avc_bench ]; then
  timeout -k 10 120 scripts/dbg/phl/avc_bench 256 400 3 1 0 1 ${LZ_ATTACK:-0} > gpurun_out/phl.log 2>&1 || exit 1
  python scripts/dbg/phases_long.py gpurun_out/phl.log
fi
