#!/bin/bash
# One gpurun call: tune (written to gpurun_out/tune_gfx950.txt), rocprofv3 trace + PMC passes
# for fp32 and bf16, then bench.py in both precisions with the same tile choices.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export AVC_TUNE_FILE=$PWD/gpurun_out/tune_gfx950.txt
[ "${KEEP_TUNE:-0}" = "1" ] || rm -f $AVC_TUNE_FILE
[ -f $AVC_TUNE_FILE ] || { [ -f profiles/tune_gfx950.txt ] && [ "${KEEP_TUNE:-0}" = "1" ] && cp profiles/tune_gfx950.txt $AVC_TUNE_FILE; }
PREC=0 bash scripts/pmc.sh || exit 1
PREC=1 bash scripts/pmc.sh || exit 1
timeout -k 10 600 python bench.py --steps ${STEPS:-2} --warmup 1 --cpu-seconds 15 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps ${STEPS:-2} --warmup 1 --precision bf16 --no-cpu-baseline > gpurun_out/bench_bf16.log 2>&1
rc=$?; echo "bench bf16 rc=$rc"; tail -1 gpurun_out/bench_bf16.log; [ $rc -eq 0 ] || exit $rc
echo DONE
