# wave timelines at the driver's 20 steps: the busy-SIMD profile (bubbles), 8 and 10 in flight
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
L=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc/librmpc_wlog.so
for S in 8 10; do
  GPU_MAX_HW_QUEUES=16 RMPC_DIAG=1 RMPC_LIB_PATH=$L timeout -k 10 200 python scripts/wave_timeline.py --steps 20 --inflight $S --out gpurun_out/r6tl20_$S.npz > gpurun_out/r6tl20_$S.json 2> gpurun_out/r6tl20_$S.err || { tail gpurun_out/r6tl20_$S.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/r6tl20_$S.json'):
    d=json.loads(l)
    if d['label']!='inflight': continue
    f=d['fast']; print('S=$S rate %.3e busy %.3f util %.3f'%(d['solves_per_s_from_span'], d['simd_busy_frac'], f['lane_utilisation']), list(d['idle_simd_us_by_transition'].items())[:5])
    print(' profile', ' '.join('%.2f'%v for v in d['busy_profile']))
"
done
