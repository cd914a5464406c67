#!/bin/bash
# GPU parity tests only (one process), then smoke.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r01}
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/gpu_tests_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests_$tag.log
exit $rc
