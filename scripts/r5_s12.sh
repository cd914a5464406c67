#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
for v in wlog wlogd; do
RMPC_DIAG=1 RMPC_LIB_PATH=$PWD/$P/librmpc_$v.so timeout -k 10 240 python scripts/wave_timeline.py --steps 30 --inflight 3 \
    --out gpurun_out/r5_wl12_$v.npz > gpurun_out/r5_wl12_$v.json 2> gpurun_out/r5_wl12_$v.err || { tail -20 gpurun_out/r5_wl12_$v.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r5_wl12_$v.json'):
    d=json.loads(l); f=lambda x: round(x/1024/30,1)
    print('$v', d['label'], 'step %.1f'%(d['window_us']/30), 'fast', f(d['fast']['simd_us']), 'group', f(d['group']['simd_us']), 'idle', f(d['gaps']['sum_simd_us']), d['fast']['dur_us_p10_50_90_max'], d['group']['dur_us_p10_50_90_max'])"
done
