#!/bin/bash
# rocprofv3 kernel trace + PMC counter passes on the native driver (no Python in the
# profiled process).  Tuning happens in an unprofiled run first (AVC_TUNE_FILE).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${PREC:-1}
ITERS=${ITERS:-20}
export AVC_TUNE_FILE=${AVC_TUNE_FILE:-$PWD/gpurun_out/tune_prof.txt}
AVC_PRINT_PLAN=1 timeout -k 10 300 ./attack-vc_amd/avc_bench 256 128 $ITERS 1 1 $P > gpurun_out/pmc_tune_p$P.log 2>&1 || { echo tune failed; exit 1; }
rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_p$P -o run --output-format csv -- \
    ./attack-vc_amd/avc_bench 256 128 $ITERS 1 0 $P > gpurun_out/prof_p$P.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C -d gpurun_out/pmc_p${P}_$i -o run --output-format csv -- \
      ./attack-vc_amd/avc_bench 256 128 5 1 0 $P > gpurun_out/pmc_p${P}_$i.log 2>&1
  rc=$?; echo "pmc pass $i ($C) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_p${P}_$i.log; exit $rc; }
done
echo DONE
