#!/bin/bash
# One development iteration on the GPU box: selected GPU tests, the phase-stamped driver
# (scripts/dbg/ph, if built) and a short emb bench line.  Every GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
T="${TESTS:-tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_vc.py}"
if [ "$T" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --tb=short --timeout 300 --timeout-method thread > gpurun_out/pytest_it.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_it.log | cut -c1-300; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_it.log | head -20; exit $rc; }
fi
if [ -x scripts/dbg/ph/avc_bench ] && [ "${PH:-1}" = 1 ]; then
  timeout -k 10 120 scripts/dbg/ph/avc_bench 256 128 20 1 1 1 ${PH_ATTACK:-0} > gpurun_out/ph.log 2>&1
  rc=$?; echo "phases rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
for A in ${ATTACKS-emb}; do
  timeout -k 10 300 python bench.py --attack $A --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-compare > gpurun_out/bench_q_$A.log 2>&1
  rc=$?; echo "bench $A rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/bench_q_$A.log; exit $rc; }
  python - "$A" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_q_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], "utts/s", "frac", d["roofline"]["frac"], {k: v["avg_ms"] for k, v in d["roofline"]["per_kernel"].items()})
PY
done
echo ALL_OK
