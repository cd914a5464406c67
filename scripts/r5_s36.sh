#!/bin/bash
# Round-5 session 36: the closed loops' three-fleet rate (round 4: 403M cold, this tree 374M):
# tail grid, generic-kernel grid and hardware-queue count, A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
export RMPC_DIAG=1
for v in "-" "RMPC_GROUP_GRID=16384" "RMPC_GENERIC_GRID=1024" "-" "RMPC_GROUP_GRID=1024"; do
  for q in 16 0; do
    [ "$v" = "-" ] && e="" || e="$v"
    env $e timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pcie --no-drop-in --hw-queues $q \
      > gpurun_out/r5s36.json 2> gpurun_out/r5s36.err || { tail gpurun_out/r5s36.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/r5s36.json'));c=d['closed_loop']
print('[$v | queues $q]', ' '.join('%s %.4e'%(k,c[k]) for k in ('cold_1_fleet','warm_1_fleet','cold_3_fleets','warm_3_fleets')))"
  done
done
