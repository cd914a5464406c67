#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
for g in 1024 16384; do
RMPC_GROUP_GRID=$g RMPC_DIAG=1 RMPC_LIB_PATH=$PWD/$P/librmpc_wlog.so timeout -k 10 240 python scripts/wave_timeline.py --steps 30 \
    --out gpurun_out/r5_wl6_$g.npz > gpurun_out/r5_wl6_$g.json 2> gpurun_out/r5_wl6_$g.err || { tail -20 gpurun_out/r5_wl6_$g.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r5_wl6_$g.json'):
    d=json.loads(l); print($g, d['label'], round(d['window_us']/30,1), d['solver'], d['simd_busy_frac'], d['fast']['dur_us_p10_50_90_max'], d['group']['dur_us_p10_50_90_max'])"
done
