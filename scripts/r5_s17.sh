#!/bin/bash
# Round-5 session 17: batches in flight x hardware queues (bench.py --hw-queues), 100 and 20 steps
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "6 16" "8 16" "8 32" "10 32" "12 32"; do
  set -- $cfg
  STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight $1 --hw-queues $2" - 2>&1 | cut -c1-110 || exit 1
  STEPS=20 bash scripts/ab.sh "--warmup 5 --inflight $1 --hw-queues $2" - - 2>&1 | cut -c1-110 || exit 1
done
