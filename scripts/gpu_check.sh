#!/bin/bash
# One gpurun call: GPU parity tests, smoke, a short bench, a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout/abort ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
stop() { echo "STOP: $1 rc=$2"; exit "$2"; }
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
export AVC_TUNE_FILE=$PWD/gpurun_out/tune.txt
rm -f "$AVC_TUNE_FILE"

if [ "${TESTS:-1}" = "1" ]; then
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=5 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
# any failure ends the GPU work of this call (a failing kernel may have faulted the GPU)
[ $rc -eq 0 ] || stop pytest $rc

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || stop smoke $rc
fi

timeout -k 10 600 python bench.py --steps ${STEPS:-2} --warmup 1 --cpu-seconds 15 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -eq 0 ] || stop bench $rc

if [ "${BF16:-1}" = "1" ]; then
timeout -k 10 600 python bench.py --steps ${STEPS:-2} --warmup 1 --precision bf16 --no-cpu-baseline > gpurun_out/bench_bf16.log 2>&1
rc=$?; echo "bench bf16 rc=$rc"; tail -1 gpurun_out/bench_bf16.log
[ $rc -eq 0 ] || stop bench_bf16 $rc
fi

if [ "${PROF:-1}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_native -o run --output-format csv -- \
      ./attack-vc_amd/avc_bench 256 128 ${PROF_ITERS:-300} 1 1 > gpurun_out/prof_native.log 2>&1
  rc=$?; echo "rocprof native rc=$rc"; tail -2 gpurun_out/prof_native.log
  [ $rc -eq 0 ] || stop rocprof_native $rc
  find gpurun_out/prof_native -name "*stats*"
fi
if [ "${PROF_PY:-0}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_py -o run --output-format csv -- \
      python3 -c "import torch; x = torch.ones(1000, device='cuda'); print(float(x.sum()))" > gpurun_out/prof_py.log 2>&1
  rc=$?; echo "rocprof py rc=$rc"; tail -3 gpurun_out/prof_py.log
fi
echo DONE
