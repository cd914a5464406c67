#!/bin/bash
# Tile stores of unchanged gains skipped (build: bash scripts/build_variant.sh skip
# -DRMPC_TILE_SKIP=1) against the default always-store build: the GPU suite through the skip
# build first, then config 3 alone and in flight, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
K="RMPC_LIB_PATH=$L/librmpc_skip.so"
env $K timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tskip_suite.txt 2>&1 \
    || { tail -30 gpurun_out/tskip_suite.txt; exit 1; }
tail -1 gpurun_out/tskip_suite.txt
STEPS=50 timeout -k 10 400 bash scripts/ab.sh "--inflight 1" - "$K" - "$K" > gpurun_out/tskip_ab.txt 2>&1 || { cat gpurun_out/tskip_ab.txt; exit 1; }
STEPS=100 timeout -k 10 600 bash scripts/ab.sh "" - "$K" - "$K" - "$K" >> gpurun_out/tskip_ab.txt 2>&1 || { cat gpurun_out/tskip_ab.txt; exit 1; }
STEPS=20 timeout -k 10 600 bash scripts/ab.sh "" - "$K" - "$K" >> gpurun_out/tskip_ab.txt 2>&1 || { cat gpurun_out/tskip_ab.txt; exit 1; }
STEPS=50 timeout -k 10 600 bash scripts/ab.sh "--config cfg4 --inflight 1" - "$K" - "$K" >> gpurun_out/tskip_ab.txt 2>&1 || { cat gpurun_out/tskip_ab.txt; exit 1; }
STEPS=50 timeout -k 10 600 bash scripts/ab.sh "--config cfg4" - "$K" - "$K" >> gpurun_out/tskip_ab.txt 2>&1 || { cat gpurun_out/tskip_ab.txt; exit 1; }
sed 's/RMPC_LIB_PATH=[^ ]*skip.so/skip/' gpurun_out/tskip_ab.txt | cut -c1-200
