#!/bin/bash
# Round-5 session 34: staged output rows (current tree) vs HEAD's fast kernel (librmpc_head.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
B="RMPC_LIB_PATH=$P/librmpc_head.so"
STEPS=20 PROF=1 bash scripts/ab.sh "--warmup 5" - "$B" 2>&1 | sed -e "s#$P/##" | cut -c1-250 || exit 1
STEPS=100 bash scripts/ab.sh "--warmup 10" - "$B" - "$B" 2>&1 | sed -e "s#$P/##" | cut -c1-160 || exit 1
STEPS=20 bash scripts/ab.sh "--warmup 5" - "$B" - "$B" 2>&1 | sed -e "s#$P/##" | cut -c1-160 || exit 1
STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight 1" - "$B" 2>&1 | sed -e "s#$P/##" | cut -c1-160 || exit 1
