#!/bin/bash
# Batches in flight against the process's hardware queues (GPU_MAX_HW_QUEUES, HIP default 4):
# config 3 with 3-6 batches in flight at 4 and 8 queues
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
STEPS=60 bash scripts/ab.sh "" "-" "GPU_MAX_HW_QUEUES=8" || exit 1
STEPS=60 bash scripts/ab.sh "--inflight 4" "-" "GPU_MAX_HW_QUEUES=8" || exit 1
STEPS=60 bash scripts/ab.sh "--inflight 6" "GPU_MAX_HW_QUEUES=8" || exit 1
STEPS=60 bash scripts/ab.sh "--inflight 8" "GPU_MAX_HW_QUEUES=8" || exit 1
STEPS=20 bash scripts/ab.sh "" "-" "GPU_MAX_HW_QUEUES=8" || exit 1
STEPS=20 bash scripts/ab.sh "--inflight 6" "GPU_MAX_HW_QUEUES=8" || exit 1
# config 4, one batch alone: first-stage (fp32 pass) and tail caps
STEPS=30 bash scripts/ab.sh "--config cfg4 --inflight 1" "-" || exit 1
for c in 8,6 10,6 10,8 12,8 16,6; do
  STEPS=30 bash scripts/ab.sh "--config cfg4 --inflight 1 --stage-caps $c" "-" || exit 1
done
