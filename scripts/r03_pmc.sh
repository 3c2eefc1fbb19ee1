#!/bin/bash
# Round-3 PMC set at HEAD: rocprofv3 kernel trace + PMC passes (scripts/pmc_fused.sh) of the
# graph-replayed native driver -- emb bf16 / fp32, e2e, fb at T=128, emb / e2e at T=400.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
# PMC_CFGS: configs "PREC ATTACK T ITERS" separated by ';'
IFS=';' read -ra CFGS <<< "${PMC_CFGS:-1 0 128 20;0 0 128 10;1 1 128 10;1 2 128 10;1 0 400 10;1 1 400 6}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  PREC=$1 ATTACK=$2 T=$3 ITERS=$4 bash scripts/pmc_fused.sh > gpurun_out/pmc_${1}_${2}_${3}.log 2>&1
  rc=$?; echo "pmc $cfg rc=$rc"; tail -2 gpurun_out/pmc_${1}_${2}_${3}.log
  [ $rc -eq 0 ] || exit $rc
done
echo ALL_OK
