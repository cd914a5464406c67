#!/bin/bash
# Round-5 final measurements, part C: GPU suite after the tail-grid change, the bench lines the
# new per-config defaults move (configs 2 and 5, LTI, config 3), rocprofv3 statistics and the
# PMC counter groups at the default in-flight count
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5g_gpu_suite.txt 2>&1 || { tail -30 gpurun_out/r5g_gpu_suite.txt; exit 1; }
tail -1 gpurun_out/r5g_gpu_suite.txt
timeout -k 10 600 python bench.py > gpurun_out/r5g_bench.json 2> gpurun_out/r5g_bench.err || { tail gpurun_out/r5g_bench.err; exit 1; }
for c in cfg2 cfg5; do
  timeout -k 10 400 python bench.py --config $c --no-pcie > gpurun_out/r5g_bench_$c.json 2> gpurun_out/r5g_bench_$c.err || { tail gpurun_out/r5g_bench_$c.err; exit 1; }
done
timeout -k 10 300 python bench.py --lti --no-cpu-baseline --no-pcie > gpurun_out/r5g_bench_lti.json 2> gpurun_out/r5g_bench_lti.err || exit 1
for f in gpurun_out/r5g_bench*.json; do python -c "import json;d=json.load(open('$f'));print('$f', '%.4e'%d['value'], 'alone %.4e'%d.get('value_one_batch_alone',0), d['config'].get('batches_in_flight'))"; done
bash scripts/measure_round.sh r5g profiles/r05 prof
