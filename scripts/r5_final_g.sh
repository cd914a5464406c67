#!/bin/bash
# Round-5 final rocprofv3 statistics and PMC counter groups of the final tree ((9, 3) in-flight
# caps, the setup's early loads)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/measure_round.sh r5l profiles/r05 prof
