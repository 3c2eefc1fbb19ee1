#!/bin/bash
# Round-4 kernel traces of the bench workloads (graph replay included): rocprofv3 --kernel-trace
# --stats of avc_bench per attack at T=128 (B=256, bf16, n iterations).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out/trace
export TMPDIR=/tmp
N=${N:-100}
for a in ${ATTACKS:-0 1 2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/trace/a$a" -o a$a -- "$R/attack-vc_amd/avc_bench" 256 ${T:-128} $N 1 1 1 $a > "$R/gpurun_out/trace/a$a.log" 2>&1
  rc=$?; echo "attack $a rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$R/gpurun_out/trace/a$a.log"; exit $rc; }
done
echo TRACE_DONE
