#!/bin/bash
# Per-dispatch kernel trace of the PredictiveModel forward (B=256): which layers the time goes to.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/pmtrace
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pmtrace -o run --output-format csv -- \
  python -u bench.py --attack pm --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/pmtrace.log 2>&1
rc=$?; echo "pmtrace rc=$rc"; tail -2 gpurun_out/pmtrace.log | cut -c1-300
find gpurun_out/pmtrace -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} gpurun_out/pmtrace_kernels.csv
exit $rc
