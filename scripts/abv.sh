#!/bin/bash
# A/B of the in-tree avc_bench against scripts/dbg/var/<V>/avc_bench, interleaved:
#   VARS="nostat ..." ARGS="256 128 300 1 1 1 0" REPS=2
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
for v in main ${VARS:-}; do
  if [ "$v" = main ]; then b=attack-vc_amd/avc_bench; else b=scripts/dbg/var/$v/avc_bench; fi
  timeout -k 10 300 $b ${ARGS:-256 128 300 1 1 1 0} > gpurun_out/abv_${v}_$rep.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/abv_${v}_$rep.log; exit $rc; }
  echo "r$rep $v: $(grep -m1 -o '"ms_per_iter": [0-9.]*' gpurun_out/abv_${v}_$rep.log) $(grep -o '"kernel": "[^"]*", "launches_per_iter": [0-9.]*, "avg_ms": [0-9.]*' gpurun_out/abv_${v}_$rep.log | sed 's/"launches_per_iter": [0-9.]*, //' | tr '\n' ' ')"
done; done
