#!/bin/bash
# Round-5 session 18: difficulty-ordered waves (bench.py --presort, host-side A/B) now that the
# in-flight pipeline keeps the SIMDs fed
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for S in 3 8; do
  for ps in 0 512 65536; do
    STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight $S --hw-queues 16 --presort $ps" - 2>&1 | cut -c1-150 || exit 1
  done
done
