#!/bin/bash
# One GPU-box session: smoke -> parity tests -> bench -> rocprofv3 kernel stats.
# Stops at the first GPU step that faults/aborts/times out (exit >= 2 for pytest,
# != 0 for the others).  Everything goes to gpurun_out/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r01}
echo "== smoke" | tee gpurun_out/progress.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/progress.log
[ $rc -ne 0 ] && exit $rc
echo "== gpu tests" | tee -a gpurun_out/progress.log
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/progress.log
[ $rc -ge 2 ] && exit $rc
echo "== bench" | tee -a gpurun_out/progress.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/progress.log
[ $rc -ne 0 ] && exit $rc
echo "== rocprofv3 stats" | tee -a gpurun_out/progress.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench_$tag.json 2> gpurun_out/prof_$tag.err
rc=$?; echo "rocprof rc=$rc" | tee -a gpurun_out/progress.log
exit $rc
