#!/bin/bash
# GPU suite (warm start with per-robot stamps, hybrid rollouts), config 5 and 3 bench lines with
# their closed-loop rates, smoke.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/suite_v9.txt 2>&1 || { tail -40 gpurun_out/suite_v9.txt; exit 1; }
tail -2 gpurun_out/suite_v9.txt; grep "warm start" gpurun_out/suite_v9.txt
for c in cfg5 cfg3; do
  timeout -k 10 600 python bench.py --config $c --no-pcie > gpurun_out/v9_bench_$c.json 2> gpurun_out/v9_bench_$c.err || { tail gpurun_out/v9_bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/v9_bench_$c.json'));c=d.get('closed_loop',{});print('$c', d['value'], {k: v for k, v in c.items() if k[:4] in ('cold', 'warm', 'max_')})"
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v9_smoke.log 2>&1 || { cat gpurun_out/v9_smoke.log; exit 1; }
echo smoke ok
