#!/bin/bash
# Round-5 session 45: alternating stream priorities across the in-flight slots (bench.py
# --stream-priority 1) vs equal priorities, config 3 at 20 and 100 steps
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
run() {   # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
    > gpurun_out/r5s45.json 2> gpurun_out/r5s45.err || { tail gpurun_out/r5s45.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5s45.json'));print('%-18s %.4e alone %.4e ms/step %.4f'%('$tag', d['value'], d.get('value_one_batch_alone',0), d['ms_per_step']))"
}
for r in 1 2 3 4; do
  run "equal 20st" --steps 20 --warmup 5
  run "alternate 20st" --steps 20 --warmup 5 --stream-priority 1
done
for r in 1 2; do
  run "equal 100st" --steps 100 --warmup 10
  run "alternate 100st" --steps 100 --warmup 10 --stream-priority 1
done
