#!/bin/bash
# Round-5 session 41: batches in flight at the driver's command -- 8 on 16 queues (default) vs
# 10 on 16 vs 10 on 32, alternating; then 100 steps
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {   # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
    > gpurun_out/r5s41.json 2> gpurun_out/r5s41.err || { tail gpurun_out/r5s41.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5s41.json'));print('%-22s %.4e ms/step %.4f'%('$tag', d['value'], d['ms_per_step']))"
}
for r in 1 2 3 4; do
  run "8/16 20st" --steps 20 --warmup 5
  run "10/16 20st" --steps 20 --warmup 5 --inflight 10
  run "10/32 20st" --steps 20 --warmup 5 --inflight 10 --hw-queues 32
done
for r in 1 2; do
  run "8/16 100st" --steps 100 --warmup 10
  run "10/16 100st" --steps 100 --warmup 10 --inflight 10
  run "10/32 100st" --steps 100 --warmup 10 --inflight 10 --hw-queues 32
done
