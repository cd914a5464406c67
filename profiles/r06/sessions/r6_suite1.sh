# GPU suite on the multi-pass tree, then the driver's command twice and 100 steps
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_suite1.txt 2>&1; rc=$?
tail -3 gpurun_out/r6_suite1.txt; grep -E "FAIL|Error" gpurun_out/r6_suite1.txt | head; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in > gpurun_out/r6s1_drv$i.json 2> gpurun_out/r6s1_drv$i.err || exit 1; done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in > gpurun_out/r6s1_100.json 2> gpurun_out/r6s1_100.err || exit 1
for f in gpurun_out/r6s1_*.json; do python -c "import json;d=json.load(open('$f'));print('$f','%.4e'%d['value'],'alone %.4e'%d.get('value_one_batch_alone',0),d['ms_per_step'],d['config'].get('stage_passes'))"; done
