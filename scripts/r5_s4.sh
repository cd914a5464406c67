#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
for g in 1024 16384; do
RMPC_GROUP_GRID=$g RMPC_DIAG=1 RMPC_LIB_PATH=$PWD/$P/librmpc_wlog.so timeout -k 10 240 python scripts/wave_timeline.py --steps 30 \
    --out gpurun_out/r5_wl4_$g.npz > gpurun_out/r5_wl4_$g.json 2> gpurun_out/r5_wl4_$g.err || { tail -20 gpurun_out/r5_wl4_$g.err; exit 1; }
cut -c1-200 gpurun_out/r5_wl4_$g.json
done
