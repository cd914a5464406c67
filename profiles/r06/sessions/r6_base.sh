cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in > gpurun_out/r6b_drv$i.json 2> gpurun_out/r6b_drv$i.err || exit 1; done
timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in > gpurun_out/r6b_100.json 2> gpurun_out/r6b_100.err || exit 1
for f in gpurun_out/r6b_*.json; do python -c "import json;d=json.load(open('$f'));print('$f','%.4e'%d['value'],'alone %.4e'%d.get('value_one_batch_alone',0),d['ms_per_step'])"; done
