# the tail on a high-priority forked stream (RMPC_TAIL_HI) at the driver's command and at 100 steps
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2 3 4; do
  for v in 0 1; do
    if [ $v = 1 ]; then E="RMPC_DIAG=1 RMPC_TAIL_HI=1"; else E=""; fi
    env $E timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in > gpurun_out/r6thi_${v}_$r.json 2> gpurun_out/r6thi_${v}_$r.err || { tail gpurun_out/r6thi_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r6thi_${v}_$r.json'));print('tail_hi=$v run $r value %.4e alone %.4e'%(d['value'],d['value_one_batch_alone']))"
  done
done
for v in 0 1; do
  if [ $v = 1 ]; then E="RMPC_DIAG=1 RMPC_TAIL_HI=1"; else E=""; fi
  env $E timeout -k 10 240 python bench.py --steps 100 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in > gpurun_out/r6thih_${v}.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r6thih_${v}.json'));print('100 steps tail_hi=$v value %.4e'%d['value'])"
done
