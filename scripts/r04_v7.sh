#!/bin/bash
# Round-3 (session 2) check: GPU suite, the default bench line (with the closed-loop rates),
# smoke, and an A/B of the cold pipeline against the previous tree's library.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/suite_v7.txt 2>&1 || { tail -40 gpurun_out/suite_v7.txt; exit 1; }
tail -2 gpurun_out/suite_v7.txt; grep "warm start" gpurun_out/suite_v7.txt
timeout -k 10 600 python bench.py > gpurun_out/v7_bench.json 2> gpurun_out/v7_bench.err || { tail gpurun_out/v7_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/v7_bench.json'));print(d['value'], d['value_one_batch_alone_default_caps'], d.get('closed_loop'))"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v7_smoke.log 2>&1 || { cat gpurun_out/v7_smoke.log; exit 1; }
echo smoke ok
H=RMPC_LIB_PATH=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc/librmpc_head.so
for r in 1 2; do
  STEPS=60 bash scripts/ab.sh "" - "$H" || exit 1
  STEPS=60 bash scripts/ab.sh "--inflight 1" - "$H" || exit 1
done
