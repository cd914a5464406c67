#!/bin/bash
# Round-5 session 30: wave timeline of the new default (8 in flight, 16 queues, zero-correction starts)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
GPU_MAX_HW_QUEUES=16 RMPC_DIAG=1 RMPC_LIB_PATH=$PWD/$P/librmpc_wlog.so timeout -k 10 240 python scripts/wave_timeline.py --steps 40 \
    --out gpurun_out/r5_wl30.npz > gpurun_out/r5_wl30.json 2> gpurun_out/r5_wl30.err || { tail -20 gpurun_out/r5_wl30.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r5_wl30.json'):
    d=json.loads(l); f=lambda x: round(x/1024/40,1)
    print(d['label'], 'step %.1f'%(d['window_us']/40), 'fast', f(d['fast']['simd_us']), 'group', f(d['group']['simd_us']), 'idle', f(d['gaps']['sum_simd_us']), d['fast']['dur_us_p10_50_90_max'], d['solver'])
    print({k: round(v/1024/40,2) for k,v in d['idle_simd_us_by_transition'].items()})"
