export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4a_suite.txt 2>&1; rc=$?; tail -3 gpurun_out/r4a_suite.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err || exit 1
timeout -k 10 200 python bench.py --gpus 2 --rehearse-one-gpu --steps 20 --warmup 3 --no-closed-loop > gpurun_out/r4a_rehearse2.json 2> gpurun_out/r4a_rehearse2.err || exit 1
cut -c1-400 gpurun_out/r4a_bench.json gpurun_out/r4a_rehearse2.json
