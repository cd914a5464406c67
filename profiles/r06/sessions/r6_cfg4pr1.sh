# config 4: fp32 stage at one lane per robot (RMPC_F32_PR1) vs paired lanes: parity, in flight, alone
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
RMPC_DIAG=1 RMPC_F32_PR1=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_headline.py -x -v --timeout 300 --timeout-method thread -k "cfg4" -s > gpurun_out/r6_pr1_tests.txt 2>&1; rc=$?
grep -E "PASS|FAIL|cfg4" gpurun_out/r6_pr1_tests.txt | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in 0 1; do
    if [ $v = 1 ]; then E="RMPC_DIAG=1 RMPC_F32_PR1=1"; else E=""; fi
    env $E timeout -k 10 240 python bench.py --config cfg4 --steps 30 --no-cpu-baseline --no-pcie > gpurun_out/r6pr1_${v}_$r.json 2> gpurun_out/r6pr1_${v}_$r.err || { tail gpurun_out/r6pr1_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r6pr1_${v}_$r.json'));print('pr1=$v run $r value %.4e alone %.4e stage_ms %s'%(d['value'],d['value_one_batch_alone'],d['roofline'].get('stage_ms')))"
  done
done
