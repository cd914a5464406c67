#!/bin/bash
# Final check of the session: GPU suite, the round measurement (PMC passes without the closed
# loop, bench lines, rocprof stats, smoke), and the mpc_rate-5 closed loop with the warm caps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/suite_v11.txt 2>&1 || { tail -40 gpurun_out/suite_v11.txt; exit 1; }
tail -1 gpurun_out/suite_v11.txt
timeout -k 10 700 bash scripts/measure_round.sh v11 profiles/r03 > gpurun_out/v11_measure.log 2>&1 || { tail -20 gpurun_out/v11_measure.log; exit 1; }
tail -5 gpurun_out/v11_measure.log | cut -c1-250
timeout -k 10 250 bash scripts/r04_v10b.sh
