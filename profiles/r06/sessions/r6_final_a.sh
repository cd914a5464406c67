# final measurements, part A: GPU suite, PMC passes (traffic, flops, in-flight flops), smoke
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6f_gpu_suite.txt 2>&1 || { tail -30 gpurun_out/r6f_gpu_suite.txt; exit 1; }
tail -1 gpurun_out/r6f_gpu_suite.txt
bash scripts/measure_round.sh r6f profiles/r06 pmc
