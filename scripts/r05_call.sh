#!/bin/bash
# Round-5 combined call: A/B -> measurement -> full GPU suite (each bounded).  A crash / timeout
# (rc 124, 134, 137, 139) ends the call; a plain test failure (rc 1) is reported at the end.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
if [ -n "${VARS:-}" ]; then TESTS=none bash scripts/r05_ab.sh; rc=$?; [ $rc -eq 0 ] || exit $rc; fi
if [ "${MEASURE:-1}" = "1" ]; then bash scripts/r05_measure.sh; rc=$?; [ $rc -eq 0 ] || exit $rc; fi
if [ "${SUITE:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest ${SUITE_SEL:-tests} -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/pytest_gpu.log | cut -c1-400
  [ $rc -eq 0 ] || { grep -E "^FAILED|Error:|AssertionError" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
fi
echo CALL_OK
