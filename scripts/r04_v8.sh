#!/bin/bash
# GPU suite, config 3 and 4 bench lines (with the closed-loop rates), smoke, cold-pipeline A/B
# against the previous tree's library.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/suite_v8.txt 2>&1 || { tail -40 gpurun_out/suite_v8.txt; exit 1; }
tail -2 gpurun_out/suite_v8.txt; grep "warm start" gpurun_out/suite_v8.txt
timeout -k 10 600 python bench.py > gpurun_out/v8_bench.json 2> gpurun_out/v8_bench.err || { tail gpurun_out/v8_bench.err; exit 1; }
timeout -k 10 600 python bench.py --config cfg4 --no-pcie > gpurun_out/v8_bench_cfg4.json 2> gpurun_out/v8_bench_cfg4.err || { tail gpurun_out/v8_bench_cfg4.err; exit 1; }
for f in gpurun_out/v8_bench.json gpurun_out/v8_bench_cfg4.json; do
  python -c "import json;d=json.load(open('$f'));c=d.get('closed_loop',{});print('$f', d['value'], d['value_one_batch_alone_default_caps'], {k: v for k, v in c.items() if k[:4] in ('cold', 'warm', 'max_')})"
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v8_smoke.log 2>&1 || { cat gpurun_out/v8_smoke.log; exit 1; }
echo smoke ok
H=RMPC_LIB_PATH=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc/librmpc_head.so
for r in 1 2; do
  STEPS=60 bash scripts/ab.sh "" - "$H" || exit 1
  STEPS=60 bash scripts/ab.sh "--inflight 1" - "$H" || exit 1
done
