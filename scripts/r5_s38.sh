#!/bin/bash
# Round-5 session 38: decaying-maximum tail hint (in-tree) vs last-length hint, 6 alternating
# pairs at the driver's exact command
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PAIRS=6 bash scripts/ab_driver.sh r5s38 - risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc/librmpc_hintlast.so
