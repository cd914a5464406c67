#!/bin/bash
# One batch alone (config 3): the library's default stage caps (7, 4) against neighbours.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/alone_caps.txt
for c in "" "--stage-caps 6,4" "--stage-caps 8,4" "--stage-caps 7,3" "--stage-caps 7,5" "--stage-caps 7,6" ""; do
  STEPS=50 timeout -k 10 200 bash scripts/ab.sh "--inflight 1 $c" - >> gpurun_out/alone_caps.txt 2>&1 || { cat gpurun_out/alone_caps.txt; exit 1; }
done
cut -c1-220 gpurun_out/alone_caps.txt
