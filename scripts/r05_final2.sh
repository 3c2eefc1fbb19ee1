#!/bin/bash
# Round-5 closing measurement set at HEAD, in two gpurun calls (each under the 20-minute limit):
#   STAGE=A  PMC + kernel traces (scripts/pmc_fused.sh) of the fused / long workloads, then the
#            PredictiveModel and mel2wav traces + HBM passes (scripts/r03_pm_prof.sh)
#   STAGE=B  the in-graph / kernel-trace reconciliation of the headline (scripts/r05_measure.sh) and
#            every bench line into gpurun_out/final5b/
# Any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/final5b; O=gpurun_out/final5b
if [ "${STAGE:-A}" = A ]; then
  IFS=';' read -ra CFGS <<< "${PMC_CFGS:-1 0 128 20;1 1 128 10;1 2 128 10;1 0 400 10;1 1 400 6;1 2 400 6}"
  for cfg in "${CFGS[@]}"; do
    set -- $cfg
    PREC=$1 ATTACK=$2 T=$3 ITERS=$4 bash scripts/pmc_fused.sh > gpurun_out/pmc_${1}_${2}_${3}.log 2>&1
    rc=$?; echo "pmc $cfg rc=$rc"; tail -1 gpurun_out/pmc_${1}_${2}_${3}.log
    [ $rc -eq 0 ] || exit $rc
  done
  bash scripts/r03_pm_prof.sh > gpurun_out/pm_prof.log 2>&1
  rc=$?; echo "pm/mel2wav prof rc=$rc"; tail -2 gpurun_out/pm_prof.log; [ $rc -eq 0 ] || exit $rc
  echo STAGE_A_OK
  exit 0
fi
BENCH=0 bash scripts/r05_measure.sh || exit $?
run() {   # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; grep -o '{"metric".*' $O/$n.log > $O/$n.json || true
  [ $rc -eq 0 ] || { tail -20 $O/$n.log; exit $rc; }
}
IFS=';' read -ra RUNS <<< "${RUNS:-emb;e2e;fb;emb_T400;e2e_T400;fb_T400;mel2wav;pm}"
for r in "${RUNS[@]}"; do
  case $r in
    emb) run bench_emb 600 --steps 2 --warmup 1 ;;
    e2e) run bench_e2e 600 --attack e2e --steps 1 --warmup 1 --no-fp32-compare ;;
    fb) run bench_fb 600 --attack fb --steps 1 --warmup 1 --no-fp32-compare ;;
    emb_T400) run bench_emb_T400 400 --frames 400 --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-compare ;;
    e2e_T400) run bench_e2e_T400 400 --attack e2e --frames 400 --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-compare ;;
    fb_T400) run bench_fb_T400 500 --attack fb --frames 400 --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-compare ;;
    mel2wav) run bench_mel2wav 300 --attack mel2wav --steps 2 --warmup 1 ;;
    pm) run bench_pm 300 --attack pm --steps 2 --warmup 1 ;;
  esac
done
echo FINAL_OK
