#!/bin/bash
# Round-5 session 33: control builds -- the current tree with and without the staged outputs,
# the current tree rebuilt by build_variant.sh, HEAD's fast kernel source
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
STEPS=20 bash scripts/ab.sh "--warmup 5 --inflight 1" - "RMPC_LIB_PATH=$P/librmpc_same.so" "RMPC_LIB_PATH=$P/librmpc_nocoal2.so" \
   "RMPC_LIB_PATH=$P/librmpc_head.so" "RMPC_LIB_PATH=$P/librmpc_nocoal.so" 2>&1 | sed -e "s#$P/##" | cut -c1-300 || exit 1
