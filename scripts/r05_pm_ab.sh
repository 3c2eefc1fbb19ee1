#!/bin/bash
# PredictiveModel A/B: bench.py --attack pm against libavc variants (AVC_LIB_PATH), interleaved.
#   VARS="pf2 pf3"  REPS=2
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for v in main ${VARS:-}; do
    lib=""; envs=""
    case "$v" in main) ;; env:*) envs="${v#env:}" ;; *) lib=scripts/dbg/var/$v/libavc.so ;; esac
    env $envs AVC_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --attack pm --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/pmab_$(echo $v | tr ":=" "__")_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/pmab_$(echo $v | tr ":=" "__")_$rep.log; exit $rc; }
    echo "r$rep $v: $(tail -1 gpurun_out/pmab_$(echo $v | tr ":=" "__")_$rep.log | grep -o '"value": [0-9.]*')"
  done
done
echo PMAB_DONE
