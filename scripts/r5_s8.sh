#!/bin/bash
# Round-5 session 8: the stage admission gate -- GPU suite, driver A/B vs round 4, margin sweep,
# wave timeline.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_s8_suite.txt 2>&1 || { tail -30 gpurun_out/r5_s8_suite.txt; exit 1; }
tail -2 gpurun_out/r5_s8_suite.txt
PAIRS=3 bash scripts/ab_driver.sh r5s8 $P/librmpc_h0.so - > gpurun_out/r5s8_ab.log 2>&1 || { cat gpurun_out/r5s8_ab.log; exit 1; }
cat gpurun_out/r5s8_ab.log
STEPS=100 bash scripts/ab.sh "--warmup 10" "RMPC_GATE=0" - "RMPC_GATE_MARGIN=64" "RMPC_GATE_MARGIN=192" "RMPC_GATE_MARGIN=384" || exit 1
RMPC_DIAG=1 RMPC_LIB_PATH=$PWD/$P/librmpc_wlog.so timeout -k 10 240 python scripts/wave_timeline.py --steps 30 \
    --out gpurun_out/r5_wl8.npz > gpurun_out/r5_wl8.json 2> gpurun_out/r5_wl8.err || { tail -20 gpurun_out/r5_wl8.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r5_wl8.json'):
    d=json.loads(l); f=lambda x: round(x/1024/30,1)
    print(d['label'], 'step %.1f'%(d['window_us']/30), 'fast', f(d['fast']['simd_us']), 'group', f(d['group']['simd_us']), 'idle', f(d['gaps']['sum_simd_us']), d['solver'])"
