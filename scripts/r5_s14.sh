#!/bin/bash
# Round-5 session 14: LDS fragmentation -- the tail's workgroup padded to the stage's LDS footprint
# (stage: 39424 dynamic + 408 static; tail: 37120 dynamic + 512 static -> pad 39320)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS=100 bash scripts/ab.sh "--warmup 10" - "RMPC_LDS_PAD=39320" "RMPC_LDS_PAD=39320 RMPC_GENERIC_GRID=1" "RMPC_LDS_PAD=39320 RMPC_GENERIC_GRID=1 RMPC_GATE=0" - 2>&1 | cut -c1-150 || exit 1
STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight 5" "GPU_MAX_HW_QUEUES=16 RMPC_LDS_PAD=39320 RMPC_GENERIC_GRID=1" 2>&1 | cut -c1-150 || exit 1
