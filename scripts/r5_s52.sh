#!/bin/bash
# Round-5 session 52: LTI's in-flight caps (default (13, 4)) and config 5's (default (9, 4)),
# 50 steps, two rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {   # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
    > gpurun_out/r5s52.json 2> gpurun_out/r5s52.err || { tail gpurun_out/r5s52.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5s52.json'));print('%-18s %.4e ms/step %.4f'%('$tag', d['value'], d['ms_per_step']))"
}
for r in 1 2; do
  for c in 13,4 13,3 11,3 15,3; do run "lti caps $c" --lti --steps 50 --warmup 5 --stage-caps $c; done
  for c in 9,4 10,3 10,4; do run "cfg5 caps $c" --config cfg5 --steps 50 --warmup 5 --stage-caps $c; done
done
