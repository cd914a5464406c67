#!/bin/bash
# Round-5 session 49: with the (9, 3) caps, the other in-flight settings at the driver's command:
# zero-correction first sets off, 6 / 7 / 9 batches in flight (three alternating rounds)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {   # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
    > gpurun_out/r5s49.json 2> gpurun_out/r5s49.err || { tail gpurun_out/r5s49.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5s49.json'));print('%-16s %.4e ms/step %.4f'%('$tag', d['value'], d['ms_per_step']))"
}
for r in 1 2 3; do
  run "default" --steps 20 --warmup 5
  run "cold-start 0" --steps 20 --warmup 5 --cold-start 0
  run "inflight 6" --steps 20 --warmup 5 --inflight 6
  run "inflight 7" --steps 20 --warmup 5 --inflight 7
  run "inflight 9" --steps 20 --warmup 5 --inflight 9
done
