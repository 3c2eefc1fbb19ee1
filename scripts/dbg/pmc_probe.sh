#!/bin/bash
# Exploratory PMC passes on the emb bf16 driver (one pass per counter group, each bounded).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/rocprof_L.txt 2>&1; echo "list rc=$?"
i=0
IFS=';' read -ra GROUPS_ <<< "${GRPS:-TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum;TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum}"
for C in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/probe_$i -o run --output-format csv -- \
      ./attack-vc_amd/avc_bench 256 128 5 1 0 1 0 > gpurun_out/probe_$i.log 2>&1
  rc=$?; echo "pass $i ($C) rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/probe_$i.log; }
done
echo DONE
