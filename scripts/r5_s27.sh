#!/bin/bash
# Round-5 session 27: zero-correction start at 8 in flight (RMPC_INIT_ZC, A/B)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS=100 bash scripts/ab.sh "--warmup 10" - "RMPC_INIT_ZC=1" - "RMPC_INIT_ZC=1" 2>&1 | cut -c1-150 || exit 1
STEPS=20 bash scripts/ab.sh "--warmup 5" - "RMPC_INIT_ZC=1" - "RMPC_INIT_ZC=1" 2>&1 | cut -c1-150 || exit 1
STEPS=50 bash scripts/ab.sh "--warmup 5 --config cfg5" - "RMPC_INIT_ZC=1" 2>&1 | cut -c1-150 || exit 1
STEPS=50 bash scripts/ab.sh "--warmup 5 --config cfg4" - "RMPC_INIT_ZC=1" 2>&1 | cut -c1-150 || exit 1
