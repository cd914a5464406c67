#!/bin/bash
# Round-5 session 26: GPU suite after removing the wave order; stage caps at 8 in flight
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_s26_suite.txt 2>&1 || { tail -30 gpurun_out/r5_s26_suite.txt; exit 1; }
tail -1 gpurun_out/r5_s26_suite.txt
for caps in 9,4 7,4 11,4 13,4 9,3; do
  STEPS=100 bash scripts/ab.sh "--warmup 10 --stage-caps $caps" - 2>&1 | cut -c1-120 || exit 1
done
for caps in 9,4 11,4; do
  STEPS=20 bash scripts/ab.sh "--warmup 5 --stage-caps $caps" - - 2>&1 | cut -c1-120 || exit 1
done
