#!/bin/bash
# Round-5 A/B: selected GPU tests, then interleaved avc_bench timings of the in-tree build against
# scripts/dbg/var/<V> builds and env-switched runs of the in-tree build ("env:NAME=VAL" in VARS).
#   TESTS="..."|none  VARS="abl32 env:AVC_FWD_ADV=0"  WL="B T n steps warmup prec attack;..."  REPS=2
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
T="${TESTS:-none}"
if [ "$T" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --tb=short --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_ab.log | cut -c1-300; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_ab.log | head -30; exit $rc; }
fi
IFS=';' read -ra WLS <<< "${WL:-256 128 300 1 1 1 0}"
for wl in "${WLS[@]}"; do
  tag=$(echo $wl | tr ' ' '_')
  for rep in $(seq ${REPS:-2}); do
    for v in main ${VARS:-}; do
      envs=""; b=attack-vc_amd/avc_bench
      case "$v" in
        main) ;;
        env:*) envs="${v#env:}" ;;
        *) b=scripts/dbg/var/$v/avc_bench ;;
      esac
      vt=$(echo $v | tr ':=' '__')
      env $envs timeout -k 10 300 $b $wl > gpurun_out/ab_${tag}_${vt}_$rep.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/ab_${tag}_${vt}_$rep.log; exit $rc; }
      echo "[$wl] r$rep $v: $(grep -m1 -o "\"ms_per_iter\": [0-9.]*" gpurun_out/ab_${tag}_${vt}_$rep.log) $(grep -o '"ktime_kernel": "[^"]*", "launches_per_iter": [0-9.]*, "avg_us": [0-9.]*' gpurun_out/ab_${tag}_${vt}_$rep.log | sed 's/"launches_per_iter": [0-9.]*, //;s/"ktime_kernel": //;s/"avg_us": //' | tr '\n' ' ')"
    done
  done
done
echo AB_DONE
