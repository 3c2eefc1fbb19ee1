#!/bin/bash
# rocprofv3 kernel trace + HBM-traffic PMC passes of the mel2wav back end
# (bench.py --attack mel2wav, B=256 mels of 80x128, 100 Griffin-Lim iterations).
# Every pass is its own bounded run; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/dsp
rm -rf $OUT
ARGS="bench.py --attack mel2wav --steps 1 --warmup 0 --no-cpu-baseline --no-roofline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $ARGS \
    > $OUT.trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT.trace.log; exit $rc; }
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $C -d $OUT/pmc_$i -o run --output-format csv -- python3 $ARGS \
      > $OUT.pmc_$i.log 2>&1
  rc=$?; echo "pmc pass $i ($C) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT.pmc_$i.log; exit $rc; }
done
python3 scripts/dsp_summary.py --dir $OUT --round r01
