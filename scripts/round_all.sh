#!/bin/bash
# One gpurun call at a milestone: full GPU test suite, smoke(), rocprofv3 trace + PMC of the
# emb bf16 attack and of the mel2wav back end, and the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_all.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; grep smoke: gpurun_out/smoke.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/smoke.log; exit $rc; }
PREC=1 ATTACK=0 bash scripts/pmc_fused.sh > gpurun_out/pmc_emb.log 2>&1
rc=$?; echo "pmc emb rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_emb.log; exit $rc; }
python3 scripts/prof_fused.py --prec 1 --attack 0 > /dev/null || exit 1
bash scripts/pmc_dsp.sh > gpurun_out/pmc_dsp.log 2>&1
rc=$?; echo "pmc dsp rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_dsp.log; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/bench_default.log gpurun_out/bench_default.json
timeout -k 10 300 python bench.py --attack mel2wav --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_mel2wav.log 2>&1
rc=$?; echo "bench mel2wav rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo DONE
