#!/bin/bash
# Round-5 session 47: in-flight tail cap 3 vs 4 (stage caps 9,3 / 10,3 vs the default 9,4):
# config 3 at 20 and 100 steps, config 5 at 50 steps
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {   # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
    > gpurun_out/r5s47.json 2> gpurun_out/r5s47.err || { tail gpurun_out/r5s47.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5s47.json'));print('%-20s %.4e ms/step %.4f'%('$tag', d['value'], d['ms_per_step']))"
}
for r in 1 2 3; do
  for c in 9,4 9,3 10,3; do run "20st caps $c" --steps 20 --warmup 5 --stage-caps $c; done
done
for r in 1 2; do
  for c in 9,4 9,3 10,3; do run "100st caps $c" --steps 100 --warmup 10 --stage-caps $c; done
  for c in 9,4 9,3; do run "cfg5 caps $c" --config cfg5 --steps 50 --warmup 5 --stage-caps $c; done
done
