#!/bin/bash
# Round-5 session 21: the cost of reading robots through an order list (wave order 64 = only the
# lanes of each wave permuted) vs the ordering's gain (host presort)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for wo in 0 64; do
  for ps in 0 512; do
    STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight 8 --hw-queues 16 --wave-order $wo --presort $ps" - 2>&1 | cut -c1-130 || exit 1
  done
done
STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight 1 --wave-order 64 --wave-order-alone" - 2>&1 | cut -c1-250 || exit 1
