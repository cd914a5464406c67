#!/bin/bash
# End-of-session check on the GPU box: GPU suite, the round measurement (scripts/measure_round.sh:
# PMC passes, every bench line, rocprof stats, smoke), and the closed loop at run_simulation.py's
# mpc_rate 5 with the warm start's caps.  Usage: bash scripts/check_session.sh <tag> [profiles dir]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-chk}; rdir=${2:-profiles/r06}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/suite_$tag.txt 2>&1 || { tail -40 gpurun_out/suite_$tag.txt; exit 1; }
tail -1 gpurun_out/suite_$tag.txt
timeout -k 10 900 bash scripts/measure_round.sh $tag $rdir > gpurun_out/${tag}_measure.log 2>&1 || { tail -20 gpurun_out/${tag}_measure.log; exit 1; }
tail -5 gpurun_out/${tag}_measure.log | cut -c1-250
CL_RATE=5 CL_CAPS="3,4;4,4" timeout -k 10 250 python scripts/closed_loop_warm.py 65536 100 1 3 \
    > gpurun_out/${tag}_clw5.out 2> gpurun_out/${tag}_clw5.err || { tail gpurun_out/${tag}_clw5.err; exit 1; }
cut -c1-200 gpurun_out/${tag}_clw5.out
