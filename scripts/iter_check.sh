#!/bin/bash
# Iteration check in one gpurun call: GPU parity suite, phase stamps of the working
# tree (scripts/dbg/ph), then the interleaved A/B timing against build/ab/*.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_iter.log | cut -c1-400; [ $rc -eq 0 ] || { grep -m5 -B5 "Error\|assert" gpurun_out/pytest_iter.log | head -60; exit $rc; }
if [ -x scripts/dbg/ph/avc_bench ]; then
  timeout -k 10 120 scripts/dbg/ph/avc_bench 256 128 3 1 0 1 0 > gpurun_out/ph.log 2>&1 || exit 1
  python3 scripts/dbg/phases.py gpurun_out/ph.log
fi
PRECS=${PRECS:-1} bash scripts/ab.sh
