#!/bin/bash
# Round-5 session 29: config 5's one-batch-alone rate vs batches in flight / hardware queues
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "3 0" "8 16" "8 32" "3 16" "8 0"; do
  set -- $cfg
  STEPS=50 bash scripts/ab.sh "--warmup 5 --config cfg5 --inflight $1 --hw-queues $2" - 2>&1 | cut -c1-110 || exit 1
done
