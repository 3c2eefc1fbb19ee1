#!/bin/bash
# Fused-engine bring-up: its GPU tests first (each GPU step under its own limit; any
# failure ends the call), then the remaining GPU tests, then short benches.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export AVC_TUNE_FILE=$PWD/profiles/tune_gfx950.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1
rc=$?; echo "pytest fused rc=$rc"; tail -25 gpurun_out/pytest_fused.log; [ $rc -eq 0 ] || exit $rc
if [ "${ALL:-1}" = "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for P in bf16 fp32; do
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --precision $P --no-cpu-baseline > gpurun_out/bench_$P.log 2>&1
rc=$?; echo "bench $P rc=$rc"; tail -1 gpurun_out/bench_$P.log; [ $rc -eq 0 ] || exit $rc
done
echo DONE
