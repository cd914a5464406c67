#!/bin/bash
# Round-5 session 15: one LDS slot per pipeline workgroup -- GPU suite, in-flight sweep, configs 4/5
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_s15_suite.txt 2>&1 || { tail -30 gpurun_out/r5_s15_suite.txt; exit 1; }
tail -2 gpurun_out/r5_s15_suite.txt
STEPS=100 bash scripts/ab.sh "--warmup 10" - "RMPC_GATE=0" 2>&1 | cut -c1-150 || exit 1
for S in 4 5 6; do
STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight $S" "GPU_MAX_HW_QUEUES=16" "GPU_MAX_HW_QUEUES=16 RMPC_GATE=0" 2>&1 | cut -c1-150 || exit 1
done
for c in cfg4 cfg5; do
STEPS=50 bash scripts/ab.sh "--warmup 5 --config $c" - "RMPC_LIB_PATH=$PWD/$P/librmpc_h0.so" 2>&1 | cut -c1-150 || exit 1
done
