#!/bin/bash
# Closed loop at the reference's mpc_rate 5 (warm sets shifted by 5 steps), config 3's QP.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
CL_RATE=5 CL_CAPS="3,4;4,4" timeout -k 10 300 python scripts/closed_loop_warm.py 65536 100 1 3 > gpurun_out/clw5.out 2> gpurun_out/clw5.err || { tail gpurun_out/clw5.err; exit 1; }
cut -c1-200 gpurun_out/clw5.out
