#!/bin/bash
# Round-5 session 43: the stage as a work queue on a capped grid (librmpc_wq.so, an
# RMPC_FAST_WQ=1 build, with RMPC_FAST_PERSIST=<workgroups>) vs the default one workgroup per wave
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
W="RMPC_LIB_PATH=$P/librmpc_wq.so"
timeout -k 10 300 env RMPC_DIAG=1 RMPC_FAST_PERSIST=256 RMPC_LIB_PATH=$P/librmpc_wq.so python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread -k "cfg3_tail or stage_caps or tail_grid or batches_in_flight" > gpurun_out/r5_s43_tests.txt 2>&1 || { tail -30 gpurun_out/r5_s43_tests.txt; exit 1; }
tail -1 gpurun_out/r5_s43_tests.txt
STEPS=100 bash scripts/ab.sh "--warmup 10" - "$W RMPC_FAST_PERSIST=1024" "$W RMPC_FAST_PERSIST=512" "$W RMPC_FAST_PERSIST=256" - "$W RMPC_FAST_PERSIST=512" 2>&1 | sed -e "s#$P/##" | cut -c1-150 || exit 1
STEPS=20 bash scripts/ab.sh "--warmup 5" - "$W RMPC_FAST_PERSIST=512" "$W RMPC_FAST_PERSIST=256" - "$W RMPC_FAST_PERSIST=512" "$W RMPC_FAST_PERSIST=256" 2>&1 | sed -e "s#$P/##" | cut -c1-150 || exit 1
STEPS=50 bash scripts/ab.sh "--warmup 5 --inflight 1" - "$W RMPC_FAST_PERSIST=1024" "$W RMPC_FAST_PERSIST=512" 2>&1 | sed -e "s#$P/##" | cut -c1-150 || exit 1
