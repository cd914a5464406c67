#!/bin/bash
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (kernel counters only, no tracing domains).
# (PROG="scripts/inflight_run.py --steps 16": the in-flight pipeline alone instead of bench.py)
# Usage: [PROG=...] bash scripts/pmc_hbm.sh <tag> <entry kernel substring> [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-hbm}; entry=${2:-mpc_ltv_fast_kernel}; shift; shift
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${tag}_p$i -o run -- python3 ${PROG:-bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in} "$@" > gpurun_out/${tag}_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc ($grp)"
  [ $rc -ne 0 ] && exit $rc
done
python3 scripts/pmc_traffic.py gpurun_out/${tag} gpurun_out/${tag}_traffic.json "$entry"
