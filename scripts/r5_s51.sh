#!/bin/bash
# Round-5 session 51: config 4's in-flight stage caps (default (14, 6)), 50 steps, two rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {   # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
    > gpurun_out/r5s51.json 2> gpurun_out/r5s51.err || { tail gpurun_out/r5s51.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5s51.json'));print('%-18s %.4e ms/step %.4f'%('$tag', d['value'], d['ms_per_step']))"
}
for r in 1 2; do
  for c in 14,6 14,5 14,4 13,5 15,5 16,6; do run "cfg4 caps $c" --config cfg4 --steps 50 --warmup 5 --stage-caps $c; done
done
