#!/bin/bash
# Paired A/B of library builds at the driver's exact bench command
# (python bench.py --gpus 1 --steps 20 --warmup 5; the extra legs after the timed region are
# skipped, they do not touch `value`).  Each variant is a library path (RMPC_LIB_PATH, "-" =
# the in-tree librmpc.so); the variants run alternately, PAIRS rounds.  One line per run.
# Usage: [PAIRS=4] [ARGS="--steps 20 --warmup 5"] bash scripts/ab_driver.sh <tag> <lib|-> <lib|-> ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; shift
pairs=${PAIRS:-4}
args=${ARGS:---steps 20 --warmup 5}
for r in $(seq 1 $pairs); do
  for v in "$@"; do
    if [ "$v" = "-" ]; then envs="RMPC_LIB_PATH="; name=head; else envs="RMPC_DIAG=1 RMPC_LIB_PATH=$PWD/$v"; name=$(basename $v .so); fi
    out=gpurun_out/${tag}_${name}_$r.json
    env $envs timeout -k 10 240 python bench.py --gpus 1 $args --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
        > $out 2> gpurun_out/${tag}_${name}_$r.err || { echo "[$name run $r] failed"; tail -5 gpurun_out/${tag}_${name}_$r.err; exit 1; }
    python -c "
import json;d=json.load(open('$out'))
print('%-14s run %d value %.4e ms/step %.4f alone %.4e' % ('$name', $r, d['value'], d['ms_per_step'], d.get('value_one_batch_alone', 0)))"
  done
done
