#!/bin/bash
# rocprofv3 kernel traces + PMC passes for the three attacks (bf16) and emb fp32.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
for cfg in "1 0" "0 0" "1 1" "1 2"; do
  set -- $cfg
  PREC=$1 ATTACK=$2 bash scripts/pmc_fused.sh || exit $?
done
echo ALLDONE
