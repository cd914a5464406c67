# config 4: fp32 gain blocks held in registers (RMPC_GREG32 = 8 / 16 / 24 builds) -- parity, alone and in flight
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
RMPC_DIAG=1 RMPC_LIB_PATH=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc/librmpc_g32_16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -k "cfg4" -s > gpurun_out/r6_g32_tests.txt 2>&1; rc=$?
grep -E "PASS|FAIL|cfg4" gpurun_out/r6_g32_tests.txt | head; [ $rc -eq 0 ] || exit $rc
PAIRS=2 ARGS="--steps 30 --config cfg4" bash scripts/ab_driver.sh r6g32 - risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc/librmpc_g32_8.so risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc/librmpc_g32_16.so risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc/librmpc_g32_24.so
