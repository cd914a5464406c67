#!/bin/bash
# Round-5 session 44: config 4's one batch alone with the side stream on / off under the bench's
# 16 hardware queues
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do for v in 1 0; do
  timeout -k 10 300 python bench.py --config cfg4 --steps 30 --warmup 5 --alone-side $v --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
    > gpurun_out/r5s44.json 2> gpurun_out/r5s44.err || { tail gpurun_out/r5s44.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5s44.json'));print('cfg4 alone-side $v: value %.4e alone %.4e inflight-caps alone %.4e'%(d['value'], d['value_one_batch_alone'], d.get('value_one_batch_alone_inflight_caps',0)))"
done; done
