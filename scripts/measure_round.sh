#!/bin/bash
# Measurement session of a round on the GPU box (stops at the first failing GPU step):
# PMC HBM passes -> pmc_traffic.json, PMC fp64-VALU passes -> pmc_flops.json (both read by
# bench.py from profiles/), bench lines for every BASELINE configuration, rocprofv3 kernel
# stats of config 3 (three in flight and one batch), config 4 (fp32 pass + fp64 refinement +
# tail) and config 5 (decide + LQR + MPC branch), smoke.
# Usage: bash scripts/measure_round.sh <tag> <profiles dir> [all|pmc|bench|prof]
#   (outputs under gpurun_out/<tag>_*; the PMC jsons are copied into the profiles dir, where
#   bench.py finds the newest; one phase per gpurun call keeps each call under its time limit)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
tag=${1:-m}; rdir=${2:-profiles/r06}; phase=${3:-all}
mkdir -p gpurun_out $rdir
step() { echo "== $(date +%T) $*"; }
prof() {   # prof <name> <bench args...>: rocprofv3 kernel trace + stats of a short bench run
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_$name -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in "$@" \
    > gpurun_out/${tag}_prof_${name}_bench.json 2> gpurun_out/${tag}_prof_$name.err || { tail gpurun_out/${tag}_prof_$name.err; exit 1; }
}
# PMC passes per configuration (entry kernel = the first kernel of each library call); the
# jsons land in the profiles dir as pmc_{traffic,flops}[_cfgN].json, where bench.py finds them
pmc() {   # pmc <suffix> <entry kernel> <bench args...>
  local sfx=$1 entry=$2; shift; shift
  step pmc hbm $sfx
  bash scripts/pmc_hbm.sh ${tag}_hbm$sfx "$entry" "$@" > gpurun_out/${tag}_pmc_hbm$sfx.log 2>&1 || { tail gpurun_out/${tag}_pmc_hbm$sfx.log; exit 1; }
  cp gpurun_out/${tag}_hbm${sfx}_traffic.json $rdir/pmc_traffic$sfx.json
  step pmc flops $sfx
  bash scripts/pmc_flops.sh ${tag}_fl$sfx "$entry" "$@" > gpurun_out/${tag}_pmc_flops$sfx.log 2>&1 || { tail gpurun_out/${tag}_pmc_flops$sfx.log; exit 1; }
  cp gpurun_out/${tag}_fl${sfx}_flops.json $rdir/pmc_flops$sfx.json
}
if [ $phase = all ] || [ $phase = pmc ]; then
pmc "" mpc_ltv_fast_kernel --inflight 1
pmc _cfg4 "mpc_ltv_fast_kernel<30, 1, float" --config cfg4 --inflight 1
pmc _cfg5 hybrid_decide_kernel --config cfg5 --inflight 1
# the headline's own executed flops: the op counters of the in-flight pipeline alone
# (scripts/inflight_run.py, the bench's in-flight settings; entry = a kernel run once per call)
step pmc flops in flight
GPU_MAX_HW_QUEUES=32 PROG="scripts/inflight_run.py --steps 20 --inflight 10" bash scripts/pmc_flops.sh ${tag}_fli "mpc_group_kernel<20" \
  > gpurun_out/${tag}_pmc_fli.log 2>&1 || { tail gpurun_out/${tag}_pmc_fli.log; exit 1; }
cp gpurun_out/${tag}_fli_flops.json $rdir/pmc_flops_inflight.json
GPU_MAX_HW_QUEUES=32 PROG="scripts/inflight_run.py --steps 20 --inflight 10" bash scripts/pmc_hbm.sh ${tag}_hbi "mpc_group_kernel<20" \
  > gpurun_out/${tag}_pmc_hbi.log 2>&1 || { tail gpurun_out/${tag}_pmc_hbi.log; exit 1; }
cp gpurun_out/${tag}_hbi_traffic.json $rdir/pmc_traffic_inflight.json
GPU_MAX_HW_QUEUES=16 PROG="scripts/inflight_run.py --steps 16 --config cfg4" bash scripts/pmc_flops.sh ${tag}_fli4 "mpc_ltv_fast_kernel<30, 1, float" \
  > gpurun_out/${tag}_pmc_fli4.log 2>&1 || { tail gpurun_out/${tag}_pmc_fli4.log; exit 1; }
cp gpurun_out/${tag}_fli4_flops.json $rdir/pmc_flops_inflight_cfg4.json
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { cat gpurun_out/${tag}_smoke.log; exit 1; }
fi
if [ $phase = all ] || [ $phase = bench ]; then
step bench cfg3
timeout -k 10 600 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail gpurun_out/${tag}_bench.err; exit 1; }
for c in cfg2 cfg4 cfg5; do
  step bench $c
  timeout -k 10 400 python bench.py --config $c --no-pcie > gpurun_out/${tag}_bench_$c.json 2> gpurun_out/${tag}_bench_$c.err || { tail gpurun_out/${tag}_bench_$c.err; exit 1; }
done
step bench lti
timeout -k 10 300 python bench.py --lti --no-cpu-baseline --no-pcie > gpurun_out/${tag}_bench_lti.json 2> gpurun_out/${tag}_bench_lti.err || exit 1
step bench the driver command, twice
for i in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_bench_driver$i.json 2> gpurun_out/${tag}_bench_driver$i.err || exit 1
done
step 8-rank rehearsal of config 4 on one GPU
timeout -k 10 400 python bench.py --gpus 8 --config cfg4 --rehearse-one-gpu --inflight 2 --hw-queues 4 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/${tag}_bench_rehearse8_cfg4.json 2> gpurun_out/${tag}_bench_rehearse8_cfg4.err || { tail gpurun_out/${tag}_bench_rehearse8_cfg4.err; exit 1; }
fi
if [ $phase = all ] || [ $phase = prof ]; then
step rocprof
prof cfg3_default
prof cfg3_inflight1 --inflight 1
prof cfg4_inflight1 --config cfg4 --inflight 1
prof cfg5_inflight1 --config cfg5 --inflight 1
step pmc groups at the default in-flight count
bash scripts/pmc.sh ${tag}_grp > gpurun_out/${tag}_pmc_groups.log 2>&1 || { tail gpurun_out/${tag}_pmc_groups.log; exit 1; }
fi
step done
for f in $(ls gpurun_out/${tag}_bench*.json 2>/dev/null); do python -c "import json,sys;d=json.load(open('$f'));r=d.get('roofline') or {};print('$f', '%.4e'%d['value'], d['unit'], 'alone %.4e'%d.get('value_one_batch_alone',0), 'ms %.4f'%d['ms_per_step'], 'frac', r.get('frac'), 'frac_exec', r.get('frac_executed'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"; done
