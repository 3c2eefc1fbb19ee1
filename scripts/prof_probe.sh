#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocprofv3 --version > gpurun_out/rocprof_version.txt 2>&1
hipcc --offload-arch=gfx950 -O2 -o /tmp/rocprof_probe scripts/rocprof_probe.hip || exit 1
echo "--- probe (plain kernel-trace, default output)"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/probe1 -o run -- /tmp/rocprof_probe > gpurun_out/probe1.log 2>&1
rc=$?; echo "probe1 rc=$rc"; tail -3 gpurun_out/probe1.log
[ $rc -eq 0 ] || exit $rc
echo "--- probe csv"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/probe2 -o run --output-format csv -- /tmp/rocprof_probe > gpurun_out/probe2.log 2>&1
rc=$?; echo "probe2 rc=$rc"; tail -3 gpurun_out/probe2.log
[ $rc -eq 0 ] || exit $rc
echo "--- avc_bench no graph, no autotune"
AVC_NO_GRAPH=1 AVC_AUTOTUNE=0 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/probe3 -o run --output-format csv -- ./attack-vc_amd/avc_bench 32 128 20 1 0 > gpurun_out/probe3.log 2>&1
rc=$?; echo "probe3 rc=$rc"; tail -3 gpurun_out/probe3.log
[ $rc -eq 0 ] || exit $rc
echo "--- avc_bench with graph"
AVC_AUTOTUNE=0 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/probe4 -o run --output-format csv -- ./attack-vc_amd/avc_bench 32 128 20 1 0 > gpurun_out/probe4.log 2>&1
rc=$?; echo "probe4 rc=$rc"; tail -3 gpurun_out/probe4.log
find gpurun_out/probe* -type f | head -30
