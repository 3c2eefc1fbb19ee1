#!/bin/bash
# Round-6 closing measurement set at HEAD, in three gpurun calls (each under the 20-minute limit):
#   STAGE=A  PMC + kernel traces (scripts/pmc_fused.sh) of the fused / long workloads, then the
#            PredictiveModel and mel2wav traces + HBM passes (scripts/r03_pm_prof.sh)
#   STAGE=B  the in-graph / kernel-trace reconciliation of the headline (scripts/r05_measure.sh) and
#            the fixed-length bench lines into gpurun_out/final6/
#   STAGE=C  PMC passes of the mixed-length workload (scripts/pmc_ragged.sh) and the --lengths lines
#            (ragged and per-length buckets)
# Any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/final6; O=gpurun_out/final6
run() {   # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; grep -o '{"metric".*' $O/$n.log > $O/$n.json || true
  [ $rc -eq 0 ] || { tail -20 $O/$n.log; exit $rc; }
}
case "${STAGE:-A}" in
A)
  IFS=';' read -ra CFGS <<< "${PMC_CFGS:-1 0 128 10;1 1 128 6;1 2 128 6;1 0 400 4;1 1 400 3;1 2 400 3}"
  for cfg in "${CFGS[@]}"; do
    set -- $cfg
    PREC=$1 ATTACK=$2 T=$3 ITERS=$4 bash scripts/pmc_fused.sh > gpurun_out/pmc_${1}_${2}_${3}.log 2>&1
    rc=$?; echo "pmc $cfg rc=$rc"; tail -1 gpurun_out/pmc_${1}_${2}_${3}.log
    [ $rc -eq 0 ] || exit $rc
  done
  if [ "${PM:-1}" = "1" ]; then
    bash scripts/r03_pm_prof.sh > gpurun_out/pm_prof.log 2>&1
    rc=$?; echo "pm/mel2wav prof rc=$rc"; tail -2 gpurun_out/pm_prof.log; [ $rc -eq 0 ] || exit $rc
  fi
  echo STAGE_A_OK ;;
B)
  BENCH=0 bash scripts/r05_measure.sh || exit $?
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
  echo STAGE_B_OK ;;
C)
  if [ "${PMC:-1}" = "1" ]; then
    LO=64 HI=600 bash scripts/pmc_ragged.sh > gpurun_out/pmc_ragged.log 2>&1
    rc=$?; echo "pmc ragged rc=$rc"; tail -1 gpurun_out/pmc_ragged.log; [ $rc -eq 0 ] || exit $rc
    LO=65 HI=128 bash scripts/pmc_ragged.sh > gpurun_out/pmc_ragged_short.log 2>&1
    rc=$?; echo "pmc ragged short rc=$rc"; tail -1 gpurun_out/pmc_ragged_short.log; [ $rc -eq 0 ] || exit $rc
  fi
  run bench_lengths 600 --lengths 64:600 --steps 1 --warmup 1
  # the per-length-bucket comparison at 64 utterances (one bucket per length: ~1.5 s each on the long engine)
  run bench_lengths_b64 300 --lengths 64:600 --batch 64 --steps 1 --warmup 1 --no-cpu-baseline
  run bench_lengths_b64_bucketed 600 --lengths 64:600 --batch 64 --bucketed --steps 1 --warmup 0 --no-cpu-baseline
  # every length in (64, 128]: the ragged batch on the fused runtime-length kernels
  run bench_lengths_65_128 600 --lengths 65:128 --steps 1 --warmup 1 --no-cpu-baseline
  run bench_lengths_65_128_bucketed 600 --lengths 65:128 --bucketed --steps 1 --warmup 1 --no-cpu-baseline
  [ -n "${EXTRA:-}" ] && run bench_extra 600 $EXTRA
  echo STAGE_C_OK ;;
esac
