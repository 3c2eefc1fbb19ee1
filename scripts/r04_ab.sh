#!/bin/bash
# Round-4 A/B call: selected GPU tests, then interleaved avc_bench timings of the in-tree build
# against scripts/dbg/var/<V> variants for each workload in WL ("B T n steps warmup prec attack").
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
T="${TESTS:-tests/test_gpu_fused.py tests/test_gpu_parity.py}"
if [ "$T" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --tb=short --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_ab.log | cut -c1-300; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_ab.log | head -20; exit $rc; }
fi
IFS=';' read -ra WLS <<< "${WL:-256 128 300 1 1 1 0}"
for wl in "${WLS[@]}"; do
  tag=$(echo $wl | tr ' ' '_')
  for rep in $(seq ${REPS:-2}); do
    for v in main ${VARS:-}; do
      if [ "$v" = main ]; then b=attack-vc_amd/avc_bench; else b=scripts/dbg/var/$v/avc_bench; fi
      timeout -k 10 300 $b $wl > gpurun_out/ab_${tag}_${v}_$rep.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/ab_${tag}_${v}_$rep.log; exit $rc; }
      echo "[$wl] r$rep $v: $(grep -m1 -o "\"ms_per_iter\": [0-9.]*, \"checksum\": [-0-9.]*" gpurun_out/ab_${tag}_${v}_$rep.log) $(grep -o '"kernel": "[^"]*", "launches_per_iter": [0-9.]*, "avg_ms": [0-9.]*' gpurun_out/ab_${tag}_${v}_$rep.log | sed 's/"launches_per_iter": [0-9.]*, //;s/"kernel": //;s/"avg_ms": //' | tr '\n' ' ')"
    done
  done
done
echo AB_DONE
