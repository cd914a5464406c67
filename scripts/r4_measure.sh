#!/bin/bash
# Round-4 measurement: GPU suite, then the round measurement (PMC per config, bench lines, rocprof, smoke)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r4m}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/suite_$tag.txt 2>&1 || { tail -40 gpurun_out/suite_$tag.txt; exit 1; }
tail -1 gpurun_out/suite_$tag.txt
timeout -k 10 850 bash scripts/measure_round.sh $tag profiles/r04 > gpurun_out/${tag}_measure.log 2>&1 || { tail -20 gpurun_out/${tag}_measure.log; exit 1; }
tail -8 gpurun_out/${tag}_measure.log | cut -c1-250
