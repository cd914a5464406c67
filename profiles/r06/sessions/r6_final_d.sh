# after the config-5 change: GPU suite, config 5's bench line at its new default, smoke
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6g_gpu_suite.txt 2>&1 || { tail -30 gpurun_out/r6g_gpu_suite.txt; exit 1; }
tail -1 gpurun_out/r6g_gpu_suite.txt
timeout -k 10 400 python bench.py --config cfg5 --no-pcie > gpurun_out/r6g_bench_cfg5.json 2> gpurun_out/r6g_bench_cfg5.err || { tail gpurun_out/r6g_bench_cfg5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r6g_bench_cfg5.json'));print('cfg5 %.4e alone %.4e'%(d['value'],d['value_one_batch_alone']), d['config'])"
