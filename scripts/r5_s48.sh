#!/bin/bash
# Round-5 session 48: in-flight stage caps around (9, 3), config 3 at the
# driver's command ((9,3) = the bench default), three alternating rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {   # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
    > gpurun_out/r5s48.json 2> gpurun_out/r5s48.err || { tail gpurun_out/r5s48.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5s48.json'));print('%-14s %.4e ms/step %.4f'%('$tag', d['value'], d['ms_per_step']))"
}
for r in 1 2 3; do
  for c in 9,3 9,2 8,3 8,2 10,2; do run "caps $c" --steps 20 --warmup 5 --stage-caps $c; done
done
