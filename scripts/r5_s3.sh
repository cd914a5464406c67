#!/bin/bash
# Round-5 session 3: the capped tail grid -- GPU suite, driver-command A/B against the round-4
# library, the wave timeline, and a grid-cap sweep.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_s3_suite.txt 2>&1 || { tail -30 gpurun_out/r5_s3_suite.txt; exit 1; }
tail -2 gpurun_out/r5_s3_suite.txt
PAIRS=3 bash scripts/ab_driver.sh r5s3 $P/librmpc_h0.so - > gpurun_out/r5s3_ab.log 2>&1 || { cat gpurun_out/r5s3_ab.log; exit 1; }
cat gpurun_out/r5s3_ab.log
PAIRS=1 ARGS="--steps 100 --warmup 10" bash scripts/ab_driver.sh r5s3l $P/librmpc_h0.so - > gpurun_out/r5s3_abl.log 2>&1 || { cat gpurun_out/r5s3_abl.log; exit 1; }
cat gpurun_out/r5s3_abl.log
RMPC_DIAG=1 RMPC_LIB_PATH=$PWD/$P/librmpc_wlog.so timeout -k 10 240 python scripts/wave_timeline.py --steps 30 \
    --out gpurun_out/r5_wl3.npz > gpurun_out/r5_wl3.json 2> gpurun_out/r5_wl3.err || { tail -20 gpurun_out/r5_wl3.err; exit 1; }
cut -c1-300 gpurun_out/r5_wl3.json
for g in 512 2048 4096; do
  RMPC_GROUP_GRID=$g STEPS=20 bash scripts/ab.sh "--warmup 5" - 2>&1 | sed "s/^/grid $g: /" || exit 1
done
STEPS=20 bash scripts/ab.sh "--warmup 5" - 2>&1 | sed "s/^/grid 1024: /" || exit 1
