#!/bin/bash
# Round-5 session 46: in-flight stage caps with the zero-correction first sets, config 3 at the
# driver's command (9,4 = the bench default), three alternating rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {   # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
    > gpurun_out/r5s46.json 2> gpurun_out/r5s46.err || { tail gpurun_out/r5s46.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5s46.json'));print('%-14s %.4e ms/step %.4f'%('$tag', d['value'], d['ms_per_step']))"
}
for r in 1 2 3; do
  for c in 9,4 8,4 10,4 11,4 9,5 9,3; do run "caps $c" --steps 20 --warmup 5 --stage-caps $c; done
done
