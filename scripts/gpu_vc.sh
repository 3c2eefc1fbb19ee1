#!/bin/bash
# VC path bring-up: its GPU tests (e2e / fb / inference), then the fused-engine tests
# (regression of the shared kernels).  Each GPU step under its own limit; any failure
# ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export AVC_TUNE_FILE=$PWD/profiles/tune_gfx950.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_vc.py -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_vc.log 2>&1
rc=$?; echo "pytest vc rc=$rc"; tail -40 gpurun_out/pytest_vc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1
rc=$?; echo "pytest fused rc=$rc"; tail -5 gpurun_out/pytest_fused.log; [ $rc -eq 0 ] || exit $rc
echo DONE
