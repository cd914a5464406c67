#!/bin/bash
# Round-5 session 32: x_pred / u_seq stored as staged row segments (RMPC_OUT_COAL) vs per-lane
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_s32_suite.txt 2>&1 || { tail -30 gpurun_out/r5_s32_suite.txt; exit 1; }
tail -1 gpurun_out/r5_s32_suite.txt
B="RMPC_LIB_PATH=$P/librmpc_nocoal.so"
STEPS=100 PROF=1 bash scripts/ab.sh "--warmup 10" - "$B" 2>&1 | cut -c1-220 || exit 1
STEPS=100 bash scripts/ab.sh "--warmup 10" - "$B" - "$B" 2>&1 | cut -c1-150 || exit 1
STEPS=20 bash scripts/ab.sh "--warmup 5" - "$B" - "$B" 2>&1 | cut -c1-150 || exit 1
STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight 1" - "$B" - "$B" 2>&1 | cut -c1-150 || exit 1
for c in cfg2 cfg5; do STEPS=50 bash scripts/ab.sh "--warmup 5 --config $c" - "$B" 2>&1 | cut -c1-150 || exit 1; done
