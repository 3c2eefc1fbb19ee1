#!/bin/bash
# Round-4 PMC + kernel-trace set at HEAD: scripts/pmc_fused.sh (rocprofv3 kernel trace of the
# graph-replayed native driver + bounded PMC passes) for emb bf16 / fp32, e2e, fb at T=128 and
# emb / e2e / fb at T=400; then the PredictiveModel / mel2wav traces and HBM passes
# (scripts/r03_pm_prof.sh).  Any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
IFS=';' read -ra CFGS <<< "${PMC_CFGS:-1 0 128 20;0 0 128 10;1 1 128 10;1 2 128 10;1 0 400 10;1 1 400 6;1 2 400 6}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  PREC=$1 ATTACK=$2 T=$3 ITERS=$4 bash scripts/pmc_fused.sh > gpurun_out/pmc_${1}_${2}_${3}.log 2>&1
  rc=$?; echo "pmc $cfg rc=$rc"; tail -2 gpurun_out/pmc_${1}_${2}_${3}.log
  [ $rc -eq 0 ] || exit $rc
done
if [ "${PM_PROF:-1}" = 1 ]; then
  bash scripts/r03_pm_prof.sh > gpurun_out/pm_prof.log 2>&1
  rc=$?; echo "pm/mel2wav prof rc=$rc"; tail -3 gpurun_out/pm_prof.log; [ $rc -eq 0 ] || exit $rc
fi
echo ALL_OK
