#!/bin/bash
# Round-5 session 19: device wave order -- GPU suite, then in-flight count x queues with it
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_s19_suite.txt 2>&1 || { tail -30 gpurun_out/r5_s19_suite.txt; exit 1; }
tail -2 gpurun_out/r5_s19_suite.txt
for cfg in "3 4 512" "3 4 0" "8 16 512" "8 16 0" "6 16 512" "10 16 512" "8 16 1024" "8 16 256"; do
  set -- $cfg
  STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight $1 --hw-queues $2 --wave-order $3" - 2>&1 | cut -c1-120 || exit 1
  STEPS=20 bash scripts/ab.sh "--warmup 5 --inflight $1 --hw-queues $2 --wave-order $3" - 2>&1 | cut -c1-120 || exit 1
done
