#!/bin/bash
# Round 6 combined call: selected tests (SEL, verbose) -> bench lines (BENCHES: ';'-separated bench.py
# argument sets, each bounded) -> optionally the whole GPU suite.  The first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "${SEL:-}" ]; then
  timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r06_sel.log 2>&1
  rc=$?; echo "sel rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r06_sel.log | tail -40
  [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r06_sel.log | head -30; exit $rc; }
fi
if [ -n "${BENCHES:-}" ]; then
  IFS=';' read -ra BS <<< "$BENCHES"
  i=0
  for b in "${BS[@]}"; do
    i=$((i+1))
    timeout -k 10 600 python -u bench.py $b > gpurun_out/r06_bench_$i.log 2>&1
    rc=$?; echo "bench [$b] rc=$rc"; tail -1 gpurun_out/r06_bench_$i.log | cut -c1-700
    [ $rc -eq 0 ] || { tail -20 gpurun_out/r06_bench_$i.log; exit $rc; }
  done
fi
if [ "${SUITE:-0}" = "1" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/r06_suite.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r06_suite.log | cut -c1-400
  [ $rc -eq 0 ] || { grep -E "^FAILED|Error:|AssertionError" gpurun_out/r06_suite.log | head -30; exit $rc; }
fi
echo CALL_OK
