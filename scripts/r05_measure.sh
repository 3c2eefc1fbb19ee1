#!/bin/bash
# Round 5: in-graph kernel timing (avc_ktime) of the emb loop with and without a kernel-trace-only
# rocprofv3 attached, and the default bench line.  Each GPU step bounded; the first failure ends it.
#   WL="B T n steps warmup prec attack" (default the headline: 256 128 1500 1 1 1 0)   BENCH=0|1
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
WL="${WL:-256 128 1500 1 1 1 0}"
TAG="${TAG:-emb}"
timeout -k 10 300 attack-vc_amd/avc_bench $WL > gpurun_out/kt_${TAG}_plain.log 2>&1
rc=$?; echo "plain rc=$rc"; grep -E "ms_per_iter|ktime" gpurun_out/kt_${TAG}_plain.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/kt_${TAG}_trace
AVC_BENCH_KTIME=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${TAG}_trace -o run --output-format csv -- \
  attack-vc_amd/avc_bench $WL > gpurun_out/kt_${TAG}_traced.log 2>&1
rc=$?; echo "traced rc=$rc"; grep -E "ms_per_iter|ktime" gpurun_out/kt_${TAG}_traced.log; [ $rc -eq 0 ] || exit $rc
find gpurun_out/kt_${TAG}_trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kt_${TAG}_kernel_stats.csv
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_${TAG}.log | cut -c1-600; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}.log; exit $rc; }
fi
echo MEASURE_OK
