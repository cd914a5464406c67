# stage passes inside the hybrid step and the device rollouts (bitwise one-pass)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -k "passes" > gpurun_out/r6_passes_more.txt 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/r6_passes_more.txt | head -20; exit $rc
