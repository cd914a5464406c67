#!/bin/bash
# Round-5 session 9: batches in flight x admission gate
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for S in 3 4 5 6 8; do
  STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight $S" - "RMPC_GATE=0" 2>&1 | cut -c1-120 || exit 1
done
for S in 4 6; do
  STEPS=20 bash scripts/ab.sh "--warmup 5 --inflight $S" - - 2>&1 | cut -c1-120 || exit 1
done
