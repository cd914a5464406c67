#!/bin/bash
# Overlapped pipeline, polling A/B (one batch alone, config 3)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
STEPS=50 bash scripts/ab.sh "--inflight 1" "-" "RMPC_PIPE=1" "RMPC_PIPE=1 RMPC_PIPE_SLEEP=4" "RMPC_PIPE=1 RMPC_PIPE_SLEEP=16" \
  "RMPC_PIPE=1 RMPC_PIPE_NOWAIT=1" "RMPC_PIPE=1 RMPC_PIPE_SLEEP=16 RMPC_FAST_CAP=5" || exit 1
