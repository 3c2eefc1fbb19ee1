#!/bin/bash
# Phase-stamp runs of scripts/dbg/<PH dirs> (emb bf16 unless ARGS), summaries via scripts/dbg/phases.py
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for d in ${PHS:-ph}; do
  timeout -k 10 120 scripts/dbg/$d/avc_bench ${ARGS:-256 128 20 1 1 1 0} > gpurun_out/ph_$d.log 2>&1
  rc=$?; echo "$d rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python scripts/dbg/phases.py gpurun_out/ph_$d.log
done
