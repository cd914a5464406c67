#!/bin/bash
# Round-5 session 35: the round-4 figures the new bench defaults moved down -- LTI alone (tail
# grid for long lists), config 5 alone (side stream under 16 hardware queues), config 2 in flight
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS=50 bash scripts/ab.sh "--warmup 5 --lti --inflight 1" - "RMPC_GROUP_GRID=1024" - "RMPC_GROUP_GRID=1024" 2>&1 | cut -c1-140 || exit 1
STEPS=50 bash scripts/ab.sh "--warmup 5 --lti" - 2>&1 | cut -c1-140 || exit 1
for v in "--alone-side 1" "--alone-side 0" "--alone-side 1 --hw-queues 0" "--inflight 3 --alone-side 1"; do
  STEPS=50 bash scripts/ab.sh "--warmup 5 --config cfg5 $v" - 2>&1 | cut -c1-140 || exit 1
done
for v in "" "--inflight 3 --hw-queues 0" "--inflight 8 --hw-queues 0" "--inflight 3" "--inflight 1"; do
  STEPS=100 bash scripts/ab.sh "--warmup 10 --config cfg2 $v" - 2>&1 | cut -c1-140 || exit 1
done
STEPS=100 bash scripts/ab.sh "--warmup 10" - 2>&1 | cut -c1-140 || exit 1
