#!/bin/bash
# Round-5 session 42: 10 batches in flight on 32 queues vs the default 8 on 16, configs 4/5 and
# LTI, and config 3 at the driver's command
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {   # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
    > gpurun_out/r5s42.json 2> gpurun_out/r5s42.err || { tail gpurun_out/r5s42.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5s42.json'));print('%-26s %.4e alone %.4e ms/step %.4f'%('$tag', d['value'], d.get('value_one_batch_alone',0), d['ms_per_step']))"
}
for r in 1 2; do
  for c in cfg4 cfg5; do
    run "$c 8/16" --config $c --steps 50 --warmup 5
    run "$c 10/32" --config $c --steps 50 --warmup 5 --inflight 10 --hw-queues 32
  done
  run "lti 8/16" --lti --steps 50 --warmup 5
  run "lti 10/32" --lti --steps 50 --warmup 5 --inflight 10 --hw-queues 32
  run "cfg3 8/16 20st" --steps 20 --warmup 5
  run "cfg3 10/32 20st" --steps 20 --warmup 5 --inflight 10 --hw-queues 32
done
