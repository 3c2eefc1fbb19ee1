set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
AVC_TOL_LOG=$PWD/gpurun_out/tol.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 120 scripts/dbg/ph/avc_bench 256 128 20 1 1 1 0 > gpurun_out/ph.log 2>&1
rc=$?; echo "phases rc=$rc"; [ $rc -eq 0 ] || exit $rc
python scripts/dbg/phases.py gpurun_out/ph.log
