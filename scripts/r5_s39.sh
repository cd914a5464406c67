#!/bin/bash
# Round-5 session 39: stage-1 setup with both reference arrays' loads issued up front (in-tree)
# vs each array's loads before its own LDS rounds (librmpc_spf0.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_s39_suite.txt 2>&1 || { tail -30 gpurun_out/r5_s39_suite.txt; exit 1; }
tail -1 gpurun_out/r5_s39_suite.txt
B="RMPC_LIB_PATH=$P/librmpc_spf0.so"
STEPS=20 PROF=1 bash scripts/ab.sh "--warmup 5" - "$B" 2>&1 | sed -e "s#$P/##" | grep -v "group\]" | cut -c1-200 || exit 1
STEPS=100 bash scripts/ab.sh "--warmup 10" - "$B" - "$B" 2>&1 | sed -e "s#$P/##" | cut -c1-130 || exit 1
STEPS=20 bash scripts/ab.sh "--warmup 5" - "$B" - "$B" 2>&1 | sed -e "s#$P/##" | cut -c1-130 || exit 1
STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight 1" - "$B" - "$B" 2>&1 | sed -e "s#$P/##" | cut -c1-130 || exit 1
STEPS=50 bash scripts/ab.sh "--warmup 5 --config cfg5" - "$B" 2>&1 | sed -e "s#$P/##" | cut -c1-130 || exit 1
