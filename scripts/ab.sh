#!/bin/bash
export RMPC_DIAG=1   # the library reads its A/B knobs in diagnostics mode only
# A/B of settings over one bench line (the only A/B driver): each variant is a set of
# environment assignments -- library knobs (RMPC_FAST_CAP=9, RMPC_GROUP_GRID=2048, ...) or an
# alternative library build (RMPC_LIB_PATH=$PWD/.../librmpc_<name>.so from build_variant.sh)
# -- or "-" for the defaults.  Prints one line per run: value, ms/step, per-stage device times,
# solver statistics and the parity against the C port on the timed batch.
# Usage: [STEPS=100] [PROF=1] bash scripts/ab.sh "<bench args>" "ENV=a ENV2=b" "-" ...
#   PROF=1 also prints the fast / tail kernels' per-phase cycle counters (RMPC_DENSE_PROF).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
args=$1; shift
steps=${STEPS:-30}
for v in "$@"; do
  [ "$v" = "-" ] && v=""
  tag=$(echo "$args $v" | tr -c 'a-zA-Z0-9' '_' | cut -c1-120)
  env $v timeout -k 10 240 python bench.py $args --steps $steps --warmup 3 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
      > gpurun_out/ab_$tag.json 2>gpurun_out/ab_$tag.err || { echo "[$args | $v] failed"; tail -5 gpurun_out/ab_$tag.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/ab_$tag.json'));r=d.get('roofline',{})
print('[$args | $v] value %.4e alone %.4e ms/step %.4f'%(d['value'],d.get('value_one_batch_alone',0),d['ms_per_step']),
      {k: round(x, 4) for k, x in (r.get('stage_ms') or {}).items()}, d.get('solver'), 'du', d.get('max_abs_du_vs_cpu_port'))"
  if [ -n "$PROF" ]; then
    env $v RMPC_DENSE_PROF=1 timeout -k 10 200 python bench.py $args --inflight 1 --steps 2 --warmup 1 --no-cpu-baseline --no-closed-loop --no-drop-in \
        --no-pcie > /dev/null 2> gpurun_out/ab_${tag}_prof.err || exit 1
    grep "\[group\]\|\[fast\]\|\[dense\]\|\[refine\]" gpurun_out/ab_${tag}_prof.err | tail -5
  fi
done
