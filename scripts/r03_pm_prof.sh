#!/bin/bash
# rocprofv3 kernel traces of the PredictiveModel (config 5) and mel2wav bench runs, and their PMC
# HBM passes (FETCH_SIZE, WRITE_SIZE; MFMA busy for the PredictiveModel).  Each pass bounded.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for w in pm mel2wav; do
  O=gpurun_out/prof_$w; rm -rf $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 bench.py --attack $w --steps 5 --warmup 1 --no-cpu-baseline > $O.trace.log 2>&1
  rc=$?; echo "$w trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O.trace.log; exit $rc; }
  i=0
  for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE SQ_WAVES"; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --pmc $C -d $O/pmc_$i -o run --output-format csv -- \
      python3 bench.py --attack $w --steps 2 --warmup 1 --no-cpu-baseline > $O.pmc_$i.log 2>&1
    rc=$?; echo "$w pmc $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O.pmc_$i.log; exit $rc; }
  done
done
echo ALL_OK
