#!/bin/bash
# rocprofv3 kernel trace + PMC counter passes of the mixed-length line's workload (bench.py --lengths
# LO:HI, bf16): one ragged embedding attack over B=256 utterances (scripts/ragged_prof.py), the same passes
# as scripts/pmc_fused.sh so scripts/fz_summary.py reads it.  Every pass is its own bounded run.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LO=${LO:-64}
HI=${HI:-600}
ITERS=${ITERS:-6}
OUT=gpurun_out/rg_${LO}_${HI}
rm -rf $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 scripts/ragged_prof.py $LO $HI $ITERS > $OUT.trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT.trace.log; exit $rc; }
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $C -d $OUT/pmc_$i -o run --output-format csv -- \
      python3 scripts/ragged_prof.py $LO $HI 4 > $OUT.pmc_$i.log 2>&1
  rc=$?; echo "pmc pass $i ($C) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT.pmc_$i.log; exit $rc; }
done
echo DONE
