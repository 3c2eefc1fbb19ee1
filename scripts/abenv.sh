#!/bin/bash
# A/B of one avc_bench binary under two environments, interleaved:
#   ENV_B="AVC_HEAD_W8=0" ARGS="256 128 300 1 1 1 0" REPS=2
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
for v in A B; do
  if [ $v = A ]; then e="${ENV_A:-AVC_NOOP=1}"; else e="${ENV_B:-AVC_NOOP=1}"; fi
  env $e timeout -k 10 300 attack-vc_amd/avc_bench ${ARGS:-256 128 300 1 1 1 0} > gpurun_out/abenv_${v}_$rep.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/abenv_${v}_$rep.log; exit $rc; }
  echo "r$rep $v ($e): $(grep -m1 -o '"ms_per_iter": [0-9.]*' gpurun_out/abenv_${v}_$rep.log) $(grep -o '"kernel": "[^"]*", "launches_per_iter": [0-9.]*, "avg_ms": [0-9.]*' gpurun_out/abenv_${v}_$rep.log | sed 's/"launches_per_iter": [0-9.]*, //' | tr '\n' ' ')"
done; done
