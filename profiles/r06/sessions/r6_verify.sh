# verification of the committed tree: GPU suite, smoke, the driver's command twice, the default bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6v_gpu_suite.txt 2>&1 || { tail -30 gpurun_out/r6v_gpu_suite.txt; exit 1; }
tail -1 gpurun_out/r6v_gpu_suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6v_smoke.log 2>&1 || { cat gpurun_out/r6v_smoke.log; exit 1; }
tail -1 gpurun_out/r6v_smoke.log
for i in 1 2; do timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6v_driver$i.json 2> gpurun_out/r6v_driver$i.err || exit 1; done
timeout -k 10 600 python bench.py > gpurun_out/r6v_bench.json 2> gpurun_out/r6v_bench.err || exit 1
for f in gpurun_out/r6v_*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f','%.4e'%d['value'],'alone %.4e'%d['value_one_batch_alone'],'frac %.3f exec %.3f exec_in_flight %s'%(r['frac'],r.get('frac_executed') or 0,r.get('frac_executed_in_flight')))"; done
