#!/bin/bash
# Round-2 measurement set, part 2: rocprofv3 kernel trace + PMC passes (scripts/pmc_fused.sh)
# of the graph-replayed native driver for emb bf16 / fp32, e2e, fb at T=128 and emb at T=400.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
for cfg in "1 0 128 20" "0 0 128 10" "1 1 128 10" "1 2 128 10" "1 0 400 10"; do
  set -- $cfg
  PREC=$1 ATTACK=$2 T=$3 ITERS=$4 bash scripts/pmc_fused.sh > gpurun_out/pmc_${1}_${2}_${3}.log 2>&1
  rc=$?; echo "pmc $cfg rc=$rc"; tail -2 gpurun_out/pmc_${1}_${2}_${3}.log
  [ $rc -eq 0 ] || exit $rc
done
echo ALL_OK
