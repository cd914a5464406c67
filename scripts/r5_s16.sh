#!/bin/bash
# Round-5 session 16: LDS slots without the gate -- driver A/B vs round 4; in-flight count x hardware queues at 20 steps
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
PAIRS=3 bash scripts/ab_driver.sh r5s16 $P/librmpc_h0.so - > gpurun_out/r5s16_ab.log 2>&1 || { cat gpurun_out/r5s16_ab.log; exit 1; }
cat gpurun_out/r5s16_ab.log
for cfg in "3 4" "4 8" "5 8" "6 8" "6 16" "8 16"; do
  set -- $cfg
  STEPS=20 bash scripts/ab.sh "--warmup 5 --inflight $1" "GPU_MAX_HW_QUEUES=$2" "GPU_MAX_HW_QUEUES=$2" 2>&1 | cut -c1-110 || exit 1
done
