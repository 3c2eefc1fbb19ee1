#!/bin/bash
# Round 6: selected GPU tests (SEL) first, verbose with prints, then (SUITE=1) the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
SEL="${SEL:-tests/test_gpu_bf16_lengths.py tests/test_gpu_sn.py}"
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r06_sel.log 2>&1
rc=$?; echo "sel rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r06_sel.log | tail -40
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r06_sel.log | head -30; exit $rc; }
if [ "${SUITE:-0}" = "1" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/r06_suite.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r06_suite.log | cut -c1-400
  [ $rc -eq 0 ] || { grep -E "^FAILED|Error:|AssertionError" gpurun_out/r06_suite.log | head -30; exit $rc; }
fi
echo TESTS_OK
