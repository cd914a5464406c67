#!/bin/bash
# One measurement session on the GPU box: PMC HBM passes -> traffic json (read by bench.py via
# profiles/<round>/pmc_traffic.json) -> default bench line -> other configs -> rocprofv3 stats.
# Stops at the first failing GPU step.  Usage: bash scripts/measure_round.sh <tag> <round-dir>
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-v}; rdir=${2:-profiles/r01}
set -o pipefail
step() { echo "== $*" | tee -a gpurun_out/progress_$tag.log; }
step pmc
bash scripts/pmc_hbm.sh ${tag}_hbm > gpurun_out/${tag}_pmc.log 2>&1 || exit $?
cp gpurun_out/${tag}_hbm_traffic.json $rdir/pmc_traffic.json
step bench cfg3
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit $?
for c in cfg2 cfg4 cfg5; do
  step bench $c
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${tag}_bench_$c.json 2> gpurun_out/${tag}_bench_$c.err || exit $?
done
step bench lti
timeout -k 10 300 python bench.py --lti --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${tag}_bench_lti.json 2> gpurun_out/${tag}_bench_lti.err || exit $?
step rocprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err || exit $?
step done
