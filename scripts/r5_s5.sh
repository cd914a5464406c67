#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
STEPS=20 RMPC_LIB_PATH=$PWD/$P/librmpc_wlog.so bash scripts/ab.sh "--warmup 5 --inflight 1" - || exit 1
RMPC_DIAG=1 RMPC_LIB_PATH=$PWD/$P/librmpc_wlog.so timeout -k 10 240 python scripts/wave_timeline.py --steps 10 \
    --out gpurun_out/r5_wl5.npz > gpurun_out/r5_wl5.json 2> gpurun_out/r5_wl5.err || { tail -20 gpurun_out/r5_wl5.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r5_wl5.json'):
    d=json.loads(l); print(d['label'], d['window_us'], d['solver'], d['fast']['dur_us_p10_50_90_max'], d['group']['dur_us_p10_50_90_max'])"
