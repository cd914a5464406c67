#!/bin/bash
# Round-5 session 1: the driver-command A/B (round-3 library vs HEAD), a kernel trace of the
# in-flight run, and the per-wave timeline (wave-log build).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
bash scripts/ab_driver.sh r5ab $P/librmpc_r3.so - > gpurun_out/r5ab.log 2>&1 || { cat gpurun_out/r5ab.log; exit 1; }
cat gpurun_out/r5ab.log
RMPC_DIAG=1 RMPC_LIB_PATH=$PWD/$P/librmpc_wlog.so timeout -k 10 240 python scripts/wave_timeline.py --steps 30 \
    --out gpurun_out/r5_wl.npz > gpurun_out/r5_wl.json 2> gpurun_out/r5_wl.err || { tail -20 gpurun_out/r5_wl.err; exit 1; }
cut -c1-600 gpurun_out/r5_wl.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_tr -o run --output-format csv -- python3 bench.py \
    --steps 100 --warmup 10 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in > gpurun_out/r5_tr.json 2> gpurun_out/r5_tr.err || { tail gpurun_out/r5_tr.err; exit 1; }
echo done
