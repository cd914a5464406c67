#!/bin/bash
# Overlapped pipeline (RMPC_PIPE=1): GPU parity subset, then bench A/B (one batch alone, in flight)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
RMPC_DIAG=1 RMPC_PIPE=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "mpc or hybrid or rollout or warm or stream or inflight or side" > gpurun_out/r4_pipe_suite.txt 2>&1
rc=$?; tail -3 gpurun_out/r4_pipe_suite.txt; [ $rc = 0 ] || exit $rc
STEPS=50 bash scripts/ab.sh "--inflight 1" "-" "RMPC_PIPE=1" "RMPC_PIPE=1 RMPC_FAST_CAP=6" \
  "RMPC_PIPE=1 RMPC_FAST_CAP=5" "RMPC_PIPE=1 RMPC_FAST_CAP=4" || exit 1
STEPS=50 bash scripts/ab.sh "" "-" "RMPC_PIPE=1" || exit 1
