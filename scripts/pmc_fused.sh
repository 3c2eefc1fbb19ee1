#!/bin/bash
# rocprofv3 kernel trace + PMC counter passes of the fused-engine emb attack on the
# native driver (no Python in the profiled process).  PREC=0 fp32, PREC=1 bf16;
# ATTACK=0 emb (default), 1 e2e, 2 fb; T = frames (default 128).
# Every pass is its own bounded run; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
# no in-graph kernel stamps: their closing atomics lengthen every launch by ~9 us
export AVC_BENCH_KTIME=0
P=${PREC:-1}
A=${ATTACK:-0}
ITERS=${ITERS:-5}
TT=${T:-128}
OUT=gpurun_out/fz_p${P}_a${A}_T$TT
rm -rf $OUT
# 4 attack calls per run (steps): the persistent emb kernel (one dispatch per call) keeps 2 dispatches past
# fz_summary's 2 skipped ones; trace and counter runs use the same iterations per call
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    ./attack-vc_amd/avc_bench 256 $TT $ITERS 4 0 $P $A > $OUT.trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT.trace.log; exit $rc; }
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_$i -o run --output-format csv -- \
      ./attack-vc_amd/avc_bench 256 $TT $ITERS 4 0 $P $A > $OUT.pmc_$i.log 2>&1
  rc=$?; echo "pmc pass $i ($C) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT.pmc_$i.log; exit $rc; }
done
echo DONE
