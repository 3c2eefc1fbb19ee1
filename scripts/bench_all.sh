#!/bin/bash
# Short bench lines for the three attacks (no CPU baseline), each under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for A in ${ATTACKS:-emb e2e fb}; do
timeout -k 10 300 python bench.py --attack $A --steps ${STEPS:-1} --warmup 1 --no-cpu-baseline ${EXTRA:-} > gpurun_out/bench_$A.log 2>&1
rc=$?; echo "bench $A rc=$rc"; tail -1 gpurun_out/bench_$A.log | cut -c1-3000; [ $rc -eq 0 ] || exit $rc
done
echo DONE
