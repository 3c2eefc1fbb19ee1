#!/bin/bash
# Fused + VC GPU tests, then a short emb bench line (bf16) with per-kernel times.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_vc.py -x -q --tb=short --timeout 200 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_q.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for A in ${ATTACKS:-emb}; do
timeout -k 10 300 python bench.py --attack $A --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-compare > gpurun_out/bench_q_$A.log 2>&1
rc=$?; echo "bench $A rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/bench_q_$A.log; exit $rc; }
python - "$A" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_q_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], "utts/s", "frac", d["roofline"]["frac"], {k: v["avg_ms"] for k, v in d["roofline"]["per_kernel"].items()})
PY
done
