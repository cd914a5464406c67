#!/bin/bash
# Round-5 final bench lines with the (9, 3) in-flight caps: the default line, the driver's command
# four times, config 3's GPU stage-caps test
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/r5k_bench.json 2> gpurun_out/r5k_bench.err || { tail gpurun_out/r5k_bench.err; exit 1; }
for i in 1 2 3 4; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5k_bench_driver$i.json 2> gpurun_out/r5k_bench_driver$i.err || exit 1
done
for f in gpurun_out/r5k_bench*.json; do python -c "import json;d=json.load(open('$f'));c=d.get('closed_loop') or {};print('$f', '%.4e'%d['value'], 'alone %.4e'%d.get('value_one_batch_alone',0), d['config'].get('stage_caps'), d.get('max_abs_du_vs_cpu_port'), {k:round(v/1e6,1) for k,v in c.items() if isinstance(v,float)})"; done
