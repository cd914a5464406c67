#!/bin/bash
# Straggler hand-off A/B (RMPC_STRAGGLE=it,lanes): one batch alone and three in flight, config 3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
STEPS=50 bash scripts/ab.sh "--inflight 1" "-" "RMPC_STRAGGLE=3,4" "RMPC_STRAGGLE=3,8" "RMPC_STRAGGLE=3,16" \
  "RMPC_STRAGGLE=2,8" "RMPC_STRAGGLE=4,8" "RMPC_STRAGGLE=5,8" "RMPC_STRAGGLE=3,8 RMPC_FAST_CAP=9" || exit 1
STEPS=50 bash scripts/ab.sh "" "-" "RMPC_STRAGGLE=3,8" "RMPC_STRAGGLE=4,8" "RMPC_STRAGGLE=3,16" || exit 1
STEPS=30 bash scripts/ab.sh "--config cfg5 --inflight 1 --no-drop-in" "-" "RMPC_STRAGGLE=3,8" || exit 1
