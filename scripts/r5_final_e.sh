#!/bin/bash
# Round-5 final verification of the committed tree: GPU suite, smoke, the default bench line and
# the driver's command
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5j_gpu_suite.txt 2>&1 || { tail -30 gpurun_out/r5j_gpu_suite.txt; exit 1; }
tail -1 gpurun_out/r5j_gpu_suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5j_smoke.log 2>&1 || { cat gpurun_out/r5j_smoke.log; exit 1; }
tail -1 gpurun_out/r5j_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r5j_bench.json 2> gpurun_out/r5j_bench.err || { tail gpurun_out/r5j_bench.err; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5j_bench_driver.json 2> gpurun_out/r5j_bench_driver.err || exit 1
for f in gpurun_out/r5j_bench*.json; do python -c "import json;d=json.load(open('$f'));print('$f', '%.4e'%d['value'], 'alone %.4e'%d.get('value_one_batch_alone',0))"; done
