#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
for S in 6; do
GPU_MAX_HW_QUEUES=16 RMPC_DIAG=1 RMPC_LIB_PATH=$PWD/$P/librmpc_wlog.so timeout -k 10 240 python scripts/wave_timeline.py --steps 30 --inflight $S \
    --out gpurun_out/r5_wl11_$S.npz > gpurun_out/r5_wl11_$S.json 2> gpurun_out/r5_wl11_$S.err || { tail -20 gpurun_out/r5_wl11_$S.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r5_wl11_$S.json'):
    d=json.loads(l); f=lambda x: round(x/1024/30,1)
    print(d['label'], 'step %.1f'%(d['window_us']/30), 'fast', f(d['fast']['simd_us']), 'group', f(d['group']['simd_us']), 'idle', f(d['gaps']['sum_simd_us']), d['fast']['dur_us_p10_50_90_max'], d['solver'])"
done
