#!/bin/bash
# Time the in-tree avc_bench against build/ab/*/avc_bench, interleaved (A B A B).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
ARGS=${ARGS:-256 128 300 1 1}
for P in ${PRECS:-0 1}; do
for rep in 1 2; do
for b in attack-vc_amd/avc_bench build/ab/*/avc_bench; do
  tag=$(echo $b | tr '/' '_')
  timeout -k 10 300 $b $ARGS $P > gpurun_out/ab_${tag}_p${P}_r$rep.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$b rc=$rc"; tail -5 gpurun_out/ab_${tag}_p${P}_r$rep.log; exit $rc; }
  echo "p$P r$rep $b: $(grep -m1 -o '"ms_per_iter": [0-9.]*' gpurun_out/ab_${tag}_p${P}_r$rep.log)"
done; done; done
