#!/bin/bash
# Paired A/B of bench.py argument sets at one command line (default: the driver's exact
# command; the legs after the timed region are skipped, they do not touch `value`).  Variants
# are argument strings ("-" = none), run alternately for PAIRS rounds; one line per run.
# Usage: [PAIRS=4] [ARGS="--steps 20 --warmup 5"] bash scripts/ab_args.sh <tag> "<args>|-" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; shift
pairs=${PAIRS:-4}
args=${ARGS:---steps 20 --warmup 5}
for r in $(seq 1 $pairs); do
  j=0
  for v in "$@"; do
    j=$((j+1)); [ "$v" = "-" ] && v=""
    out=gpurun_out/${tag}_v${j}_$r.json
    timeout -k 10 240 python bench.py --gpus 1 $args $v --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
        > $out 2> ${out%.json}.err || { echo "[$v run $r] failed"; tail -5 ${out%.json}.err; exit 1; }
    python -c "
import json;d=json.load(open('$out'))
print('v$j %-32s run %d value %.4e ms/step %.4f alone %.4e' % ('$v'[:32], $r, d['value'], d['ms_per_step'], d.get('value_one_batch_alone', 0)))"
  done
done
