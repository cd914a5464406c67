# the bench JSON contract test (tests/test_gpu_bench.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_benchtest.txt 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/r6_benchtest.txt | head -20; exit $rc
