#!/bin/bash
# Round-5 session 50: seven batches in flight against eight -- config 3 at 20 and 100 steps,
# configs 4 and 5 and LTI at 50 steps
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {   # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
    > gpurun_out/r5s50.json 2> gpurun_out/r5s50.err || { tail gpurun_out/r5s50.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5s50.json'));print('%-22s %.4e alone %.4e ms/step %.4f'%('$tag', d['value'], d.get('value_one_batch_alone',0), d['ms_per_step']))"
}
for r in 1 2 3; do
  run "8 20st" --steps 20 --warmup 5
  run "7 20st" --steps 20 --warmup 5 --inflight 7
done
for r in 1 2; do
  run "8 100st" --steps 100 --warmup 10
  run "7 100st" --steps 100 --warmup 10 --inflight 7
  for c in cfg4 cfg5; do
    run "$c 8" --config $c --steps 50 --warmup 5
    run "$c 7" --config $c --steps 50 --warmup 5 --inflight 7
  done
  run "lti 8" --lti --steps 50 --warmup 5
  run "lti 7" --lti --steps 50 --warmup 5 --inflight 7
done
