# continuing pass on a hint-sized looping grid vs the capacity grid (RMPC_PASS_GRID=0), then the pass tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_headline.py -x -v --timeout 300 --timeout-method thread -k "passes or headline" > gpurun_out/r6_pg_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/r6_pg_tests.txt; [ $rc -eq 0 ] || exit $rc
PAIRS=4 bash scripts/ab_args.sh r6pg - "--stage-passes 0" || exit 1
for r in 1 2 3 4; do
  RMPC_DIAG=1 RMPC_PASS_GRID=0 timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in > gpurun_out/r6pg_cap_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r6pg_cap_$r.json'));print('capacity grid run $r value %.4e'%d['value'])"
done
PAIRS=2 ARGS="--steps 100" bash scripts/ab_args.sh r6pgh - "--stage-passes 0"
