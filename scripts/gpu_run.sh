#!/bin/bash
# One gpurun call: GPU tests (selectable), smoke, and the default bench line.
# Every GPU step runs under its own time limit; the first failure / crash / timeout ends it.
#   TESTS="tests/test_gpu_lengths.py ..." (default: all -m gpu)   SMOKE=1   BENCH=1   EXTRA="cmd"
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
stop() { echo "STOP: $1 rc=$2"; exit "$2"; }

if [ "${TESTS:-all}" != "none" ]; then
  sel="${TESTS:-tests}"
  [ "$sel" = "all" ] && sel=tests
  timeout -k 10 1500 python -u -m pytest $sel -m gpu -x -v --timeout 400 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
  [ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; stop pytest $rc; }
fi

if [ "${SMOKE:-1}" = "1" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -4 gpurun_out/smoke.log
  [ $rc -eq 0 ] || stop smoke $rc
fi

if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
  [ $rc -eq 0 ] || { tail -20 gpurun_out/bench.log; stop bench $rc; }
fi

if [ -n "${EXTRA:-}" ]; then
  timeout -k 10 900 bash -c "$EXTRA" > gpurun_out/extra.log 2>&1
  rc=$?; echo "extra rc=$rc"; tail -30 gpurun_out/extra.log
  [ $rc -eq 0 ] || stop extra $rc
fi
echo ALL_OK
