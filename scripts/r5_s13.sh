#!/bin/bash
# Round-5 session 13: the generic kernel's LDS grid (one 121-KB workgroup per CU) in flight
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS=100 bash scripts/ab.sh "--warmup 10" - "RMPC_GENERIC_GRID=1" "RMPC_GENERIC_GRID=4" "RMPC_GENERIC_GRID=16" "RMPC_GENERIC_GRID=4 RMPC_GATE=0" 2>&1 | cut -c1-150 || exit 1
STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight 4" "RMPC_GENERIC_GRID=4" "GPU_MAX_HW_QUEUES=16 RMPC_GENERIC_GRID=4" 2>&1 | cut -c1-150 || exit 1
STEPS=20 bash scripts/ab.sh "--warmup 5" - "RMPC_GENERIC_GRID=4" 2>&1 | cut -c1-150 || exit 1
