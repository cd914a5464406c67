#!/bin/bash
# Overlapped pipeline: per-wave timeline (RMPC_PIPE_DIAG) at config 3, one batch alone
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
for v in "RMPC_PIPE_NOWAIT=1" "RMPC_PIPE_SLEEP=1" "RMPC_PIPE_SLEEP=4" "RMPC_PIPE_SLEEP=8"; do
  echo "== $v"
  env RMPC_DIAG=1 RMPC_PIPE=1 RMPC_PIPE_DIAG=1 $v timeout -k 10 120 python bench.py --inflight 1 --steps 3 --warmup 1 \
    --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in > /dev/null 2> gpurun_out/r4_pipe_diag.err || { tail -5 gpurun_out/r4_pipe_diag.err; exit 1; }
  grep "\[pipe\]" gpurun_out/r4_pipe_diag.err | tail -2
done
