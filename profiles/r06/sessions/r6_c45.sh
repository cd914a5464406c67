# config 5 at its new default (10 on 32, no side streams) vs the old (8 on 16, side streams); config 4 at 10 on 32; the edge-case pass test
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_headline.py -x -v --timeout 300 --timeout-method thread -k "edge_cases or cfg5_headline" -s > gpurun_out/r6_c45_tests.txt 2>&1; rc=$?
grep -E "PASS|FAIL|Error|cfg5" gpurun_out/r6_c45_tests.txt | head; [ $rc -eq 0 ] || exit $rc
PAIRS=2 ARGS="--steps 30 --config cfg5" bash scripts/ab_args.sh r6c5b - "--inflight 8 --hw-queues 16 --inflight-side 1" || exit 1
PAIRS=2 ARGS="--steps 30 --config cfg4" bash scripts/ab_args.sh r6c4b - "--inflight 10 --hw-queues 32"
