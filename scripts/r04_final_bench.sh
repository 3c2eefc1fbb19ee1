#!/bin/bash
# Round-4 measurement set: smoke + bench lines (emb default with CPU baseline and the
# fp32 comparison; e2e / fb; the T=400 long-engine lines; mel2wav; PredictiveModel).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/final4
O=gpurun_out/final4
run() {   # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; grep -o '{"metric".*' $O/$n.log > $O/$n.json || true
  [ $rc -eq 0 ] || { tail -20 $O/$n.log; exit $rc; }
}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
[ "${ONLY_EMB:-0}" = 1 ] && { run bench_emb 600 --steps 2 --warmup 1; echo ALL_OK; exit 0; }
run bench_emb 600 --steps 2 --warmup 1
run bench_e2e 600 --attack e2e --steps 1 --warmup 1 --no-fp32-compare
run bench_fb 600 --attack fb --steps 1 --warmup 1 --no-fp32-compare
run bench_emb_T400 400 --frames 400 --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-compare
run bench_e2e_T400 400 --attack e2e --frames 400 --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-compare
run bench_fb_T400 500 --attack fb --frames 400 --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-compare
run bench_mel2wav 300 --attack mel2wav --steps 2 --warmup 1
run bench_pm 300 --attack pm --steps 2 --warmup 1
echo ALL_OK
