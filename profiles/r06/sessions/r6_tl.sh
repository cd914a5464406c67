# wave timelines + PMC of the in-flight pipeline, one pass vs multi-pass stage 1
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
L=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc/librmpc_wlog.so
for v in "0" "1" "1,3"; do
  GPU_MAX_HW_QUEUES=16 RMPC_DIAG=1 RMPC_FAST_SPLIT=$v RMPC_LIB_PATH=$L timeout -k 10 200 python scripts/wave_timeline.py --steps 30 --caps 9,3 --out gpurun_out/r6tl_$v.npz > gpurun_out/r6tl_$v.json 2> gpurun_out/r6tl_$v.err || { tail gpurun_out/r6tl_$v.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/r6tl_$v.json'):
    d=json.loads(l); f=d.get('fast',{}); g=d.get('group',{})
    print('$v', d['label'], 'rate %.3e'%d['solves_per_s_from_span'], 'busy %.3f'%d['simd_busy_frac'], 'fast simd_us %.0f util %.3f wave_its %s'%(f.get('simd_us',0), f.get('lane_utilisation',0), f.get('wave_iterations')), 'group simd_us %.0f'%g.get('simd_us',0), 'idle', list(d['idle_simd_us_by_transition'].items())[:4])
"
done
for v in "0" "1"; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    GPU_MAX_HW_QUEUES=16 RMPC_DIAG=1 RMPC_FAST_SPLIT=$v timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/r6pmc_${v}_p$i -o run -- python3 scripts/inflight_run.py --steps 16 > gpurun_out/r6pmc_${v}_p$i.log 2>&1 || { tail gpurun_out/r6pmc_${v}_p$i.log; exit 1; }
  done
  echo "== pmc split $v"; python scripts/pmc_summary.py gpurun_out/r6pmc_$v | grep -A30 "fast_kernel<20, 1, double, false, 3" | head -24
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py -x -v --timeout 300 --timeout-method thread -s > gpurun_out/r6_headline_tests.log 2>&1; echo "headline tests rc=$?"; grep -E "PASS|FAIL|Error|\[cfg" gpurun_out/r6_headline_tests.log | head -20
