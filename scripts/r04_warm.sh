#!/bin/bash
# Warm start across calls: GPU suite, the closed-loop cold/warm timing, and an A/B of the
# default (cold) pipeline against the previous tree's library (rmpc/librmpc_head.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/suite_r04w.txt 2>&1 || { tail -30 gpurun_out/suite_r04w.txt; exit 1; }
tail -3 gpurun_out/suite_r04w.txt
grep "warm start" gpurun_out/suite_r04w.txt
timeout -k 10 200 python scripts/closed_loop_warm.py > gpurun_out/closed_loop_warm.txt 2>&1 || { cat gpurun_out/closed_loop_warm.txt; exit 1; }
cat gpurun_out/closed_loop_warm.txt
H=RMPC_LIB_PATH=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc/librmpc_head.so
for r in 1 2; do
  STEPS=60 bash scripts/ab.sh "" - "$H" || exit 1
  STEPS=60 bash scripts/ab.sh "--inflight 1" - "$H" || exit 1
done
STEPS=40 bash scripts/ab.sh "--config cfg4" - "$H" || exit 1
