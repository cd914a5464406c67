#!/bin/bash
# Round-5 session 10: batches in flight x admission gate with one hardware queue per stream
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for S in 3 4 5 6; do
  STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight $S" "GPU_MAX_HW_QUEUES=16" "GPU_MAX_HW_QUEUES=16 RMPC_GATE=0" 2>&1 | cut -c1-120 || exit 1
done
