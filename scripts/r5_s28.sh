#!/bin/bash
# Round-5 session 28: cold-start setting -- GPU suite, then the default bench lines of configs 3/4/5
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_s28_suite.txt 2>&1 || { tail -30 gpurun_out/r5_s28_suite.txt; exit 1; }
tail -1 gpurun_out/r5_s28_suite.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5_s28_b20.json 2> gpurun_out/r5_s28_b20.err || { tail gpurun_out/r5_s28_b20.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5_s28_b20.json'));print('driver cmd', '%.4e'%d['value'], d['ms_per_step'], 'alone %.4e'%d['value_one_batch_alone'], 'cpu', d['cpu_baseline']['value'], 'cl', d.get('closed_loop',{}).get('cold_1_fleet'))"
for c in cfg3 cfg4 cfg5; do
  STEPS=100 bash scripts/ab.sh "--warmup 10 --config $c" - 2>&1 | cut -c1-150 || exit 1
done
