#!/bin/bash
# A/B: the N = 20 lane-group tail with 32 lanes per robot (two robots per wave) against 16
# (a local A/B build, not committed: group_lanes() returning 32 at N = 20 and the N = 20 tail
# instances built with G = 32, as bash scripts/build_variant.sh g32 -DRMPC_TAIL_G20=32; result in
# profiles/r04/ab_tail_32_lanes.txt).  Parity first (the full-size config-3 and tail-only tests
# through the variant library), then the bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
RMPC_LIB_PATH=$L/librmpc_g32.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -k "cfg3 or tail_only or stage_caps or in_flight or cfg5_full" \
    > gpurun_out/g32_tests.txt 2>&1 || { tail -30 gpurun_out/g32_tests.txt; exit 1; }
tail -1 gpurun_out/g32_tests.txt
STEPS=50 PROF=1 timeout -k 10 400 bash scripts/ab.sh "--inflight 1" - "RMPC_LIB_PATH=$L/librmpc_g32.so" - "RMPC_LIB_PATH=$L/librmpc_g32.so" \
    > gpurun_out/g32_ab.txt 2>&1 || { cat gpurun_out/g32_ab.txt; exit 1; }
STEPS=50 timeout -k 10 400 bash scripts/ab.sh "" - "RMPC_LIB_PATH=$L/librmpc_g32.so" >> gpurun_out/g32_ab.txt 2>&1 || { cat gpurun_out/g32_ab.txt; exit 1; }
STEPS=30 timeout -k 10 400 bash scripts/ab.sh "--config cfg5 --inflight 1" - "RMPC_LIB_PATH=$L/librmpc_g32.so" >> gpurun_out/g32_ab.txt 2>&1 || { cat gpurun_out/g32_ab.txt; exit 1; }
sed 's/RMPC_LIB_PATH=[^ ]*g32.so/G32/' gpurun_out/g32_ab.txt | cut -c1-260
