#!/bin/bash
# Round-5 final measurements, part A: GPU suite, PMC traffic/flops passes, smoke
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5f_gpu_suite.txt 2>&1 || { tail -30 gpurun_out/r5f_gpu_suite.txt; exit 1; }
tail -1 gpurun_out/r5f_gpu_suite.txt
bash scripts/measure_round.sh r5f profiles/r05 pmc
