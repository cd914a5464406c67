#!/bin/bash
# Repeat of the in-flight A/B of scripts/r4_g32.sh: 16 against 32 lanes per robot in the N = 20
# tail, alternating, 100 steps each, config 3 and config 5 with three batches in flight.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
G="RMPC_LIB_PATH=$L/librmpc_g32.so"
STEPS=100 timeout -k 10 600 bash scripts/ab.sh "" - "$G" - "$G" - "$G" > gpurun_out/g32b_ab.txt 2>&1 || { cat gpurun_out/g32b_ab.txt; exit 1; }
STEPS=100 timeout -k 10 400 bash scripts/ab.sh "--config cfg5" - "$G" - "$G" >> gpurun_out/g32b_ab.txt 2>&1 || { cat gpurun_out/g32b_ab.txt; exit 1; }
sed 's/RMPC_LIB_PATH=[^ ]*g32.so/G32/' gpurun_out/g32b_ab.txt | cut -c1-200
