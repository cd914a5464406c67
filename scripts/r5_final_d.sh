#!/bin/bash
# Round-5 final measurements, part D (after the tail-hint change): GPU suite, smoke, every bench
# line, the driver's command twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5h_gpu_suite.txt 2>&1 || { tail -30 gpurun_out/r5h_gpu_suite.txt; exit 1; }
tail -1 gpurun_out/r5h_gpu_suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5h_smoke.log 2>&1 || { cat gpurun_out/r5h_smoke.log; exit 1; }
tail -1 gpurun_out/r5h_smoke.log
bash scripts/measure_round.sh r5h profiles/r05 bench
