#!/bin/bash
# Round-5 session 37: tail-grid hint from a decaying maximum of the list lengths (default) vs the
# last length (librmpc_hintlast.so) vs a fixed 1024 grid: closed loops and config 3 in flight
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
export RMPC_DIAG=1
for rep in 1 2; do
for v in "-" "RMPC_LIB_PATH=$P/librmpc_hintlast.so" "RMPC_GROUP_GRID=1024"; do
  [ "$v" = "-" ] && e="" || e="$v"
  env $e timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pcie --no-drop-in \
    > gpurun_out/r5s37.json 2> gpurun_out/r5s37.err || { tail gpurun_out/r5s37.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/r5s37.json'));c=d['closed_loop']
print('[${v##*/}]', ' '.join('%s %.4e'%(k,c[k]) for k in ('cold_1_fleet','warm_1_fleet','cold_3_fleets','warm_3_fleets')))"
done
done
B="RMPC_LIB_PATH=$P/librmpc_hintlast.so"
STEPS=100 bash scripts/ab.sh "--warmup 10" - "$B" "RMPC_GROUP_GRID=1024" - "$B" "RMPC_GROUP_GRID=1024" 2>&1 | sed -e "s#$P/##" | cut -c1-130 || exit 1
STEPS=20 bash scripts/ab.sh "--warmup 5" - "$B" "RMPC_GROUP_GRID=1024" - "$B" "RMPC_GROUP_GRID=1024" 2>&1 | sed -e "s#$P/##" | cut -c1-130 || exit 1
for c in cfg4 cfg5; do STEPS=50 bash scripts/ab.sh "--warmup 5 --config $c" - "$B" 2>&1 | sed -e "s#$P/##" | cut -c1-130 || exit 1; done
