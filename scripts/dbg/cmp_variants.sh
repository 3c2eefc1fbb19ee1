#!/bin/bash
# Per-kernel times (avc_bench HIP-event profile) of the in-tree build and variants
# VARIANTS="a b" under scripts/dbg/, attack ATTACK (0 emb, 1 e2e, 2 fb), bf16.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for V in base ${VARIANTS}; do
  B=./attack-vc_amd/avc_bench; [ $V != base ] && B=./scripts/dbg/$V/avc_bench
  timeout -k 10 120 $B 256 128 300 1 1 1 ${ATTACK:-0} > gpurun_out/cmp_$V.log 2>&1 || { echo "$V failed"; tail -3 gpurun_out/cmp_$V.log; exit 1; }
  echo "== $V"; grep -h "utts_per_s\|\"kernel\"" gpurun_out/cmp_$V.log | sed -E 's/"(B|T|n_iters|steps|s|checksum)": [^,}]*,? ?//g'
done
