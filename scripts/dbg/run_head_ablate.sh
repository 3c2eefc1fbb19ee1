#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for V in 0 1 2 3; do
  B=./attack-vc_amd/avc_bench; [ $V -gt 0 ] && B=./scripts/dbg/${PFX:-head}$V/avc_bench
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${PFX:-head}ab$V -o run --output-format csv -- $B 256 128 20 1 0 1 > gpurun_out/${PFX:-head}ab$V.log 2>&1 || exit 1
  echo "variant $V"; grep -h "se_head_v\|se_fwd_fused<1, 1>\|se_bwd" gpurun_out/${PFX:-head}ab$V/run_kernel_stats.csv | cut -d, -f1-5
done
