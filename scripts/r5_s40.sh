#!/bin/bash
# Round-5 session 40: the tail-grid test, the full GPU suite, bench lines on the final tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_s40_suite.txt 2>&1 || { tail -30 gpurun_out/r5_s40_suite.txt; exit 1; }
tail -1 gpurun_out/r5_s40_suite.txt
timeout -k 10 400 python bench.py > gpurun_out/r5i_bench.json 2> gpurun_out/r5i_bench.err || { tail gpurun_out/r5i_bench.err; exit 1; }
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5i_bench_driver$i.json 2> gpurun_out/r5i_bench_driver$i.err || exit 1
done
for f in gpurun_out/r5i_bench*.json; do python -c "import json;d=json.load(open('$f'));c=d.get('closed_loop') or {};print('$f', '%.4e'%d['value'], 'alone %.4e'%d.get('value_one_batch_alone',0), {k:round(v/1e6,1) for k,v in c.items() if isinstance(v,float)})"; done
