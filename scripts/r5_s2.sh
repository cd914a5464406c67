#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
RMPC_DIAG=1 RMPC_LIB_PATH=$PWD/$P/librmpc_wlog.so timeout -k 10 240 python scripts/wave_timeline.py --steps 30 \
    --out gpurun_out/r5_wl2.npz > gpurun_out/r5_wl2.json 2> gpurun_out/r5_wl2.err || { tail -20 gpurun_out/r5_wl2.err; exit 1; }
cut -c1-300 gpurun_out/r5_wl2.json
