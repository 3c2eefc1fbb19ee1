#!/bin/bash
# PredictiveModel A/B: the GPU tests on the in-tree build, then bench.py --attack pm alternating the
# in-tree libavc.so and scripts/dbg/var/<V>/libavc.so for V in VARS (copied over it in this scratch tree).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_predictive.py tests/test_gpu_modules.py tests/test_gpu_vsmask.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pm_t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pm_t.log; [ $rc -eq 0 ] || exit $rc
cp attack-vc_amd/libavc.so /tmp/libavc_main.so
for r in 1 2; do
  for v in main ${VARS:-base}; do
    if [ $v = main ]; then cp /tmp/libavc_main.so attack-vc_amd/libavc.so; else cp scripts/dbg/var/$v/libavc.so attack-vc_amd/libavc.so; fi
    timeout -k 10 180 python -u bench.py --attack ${ATTACK:-pm} --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > gpurun_out/pm_${v}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/pm_${v}_$r.log; exit $rc; }
    echo "r$r $v: $(grep -o '"value": [0-9.]*' gpurun_out/pm_${v}_$r.log | head -1)"
  done
done
cp /tmp/libavc_main.so attack-vc_amd/libavc.so
echo PM_AB_DONE
