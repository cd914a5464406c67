#!/bin/bash
# Round-5 session 31: the tail grid sized from the last launch's list length
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_s31_suite.txt 2>&1 || { tail -30 gpurun_out/r5_s31_suite.txt; exit 1; }
tail -1 gpurun_out/r5_s31_suite.txt
STEPS=100 bash scripts/ab.sh "--warmup 10" - "RMPC_GROUP_GRID=1024" - "RMPC_GROUP_GRID=1024" 2>&1 | cut -c1-150 || exit 1
STEPS=20 bash scripts/ab.sh "--warmup 5" - "RMPC_GROUP_GRID=1024" - "RMPC_GROUP_GRID=1024" 2>&1 | cut -c1-150 || exit 1
for c in cfg4 cfg5; do STEPS=50 bash scripts/ab.sh "--warmup 5 --config $c" - "RMPC_GROUP_GRID=1024" 2>&1 | cut -c1-150 || exit 1; done
GPU_MAX_HW_QUEUES=16 RMPC_DIAG=1 RMPC_LIB_PATH=$PWD/$P/librmpc_wlog.so timeout -k 10 240 python scripts/wave_timeline.py --steps 40 \
    --out gpurun_out/r5_wl31.npz > gpurun_out/r5_wl31.json 2> gpurun_out/r5_wl31.err || { tail -20 gpurun_out/r5_wl31.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r5_wl31.json'):
    d=json.loads(l); f=lambda x: round(x/1024/40,1)
    print(d['label'], 'step %.1f'%(d['window_us']/40), 'fast', f(d['fast']['simd_us']), 'group', f(d['group']['simd_us']), 'idle', f(d['gaps']['sum_simd_us']), d['group']['waves'])
    print({k: round(v/1024/40,2) for k,v in d['idle_simd_us_by_transition'].items()})"
