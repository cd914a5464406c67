#!/bin/bash
# Config 5 (hybrid step), one batch alone: the MPC branch's stage caps (library default (6, 4))
# against neighbours, alternating; then in flight (bench default (9, 4)) against (8, 4) / (10, 4).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/cfg5_caps.txt
for rep in 1 2; do
  for c in "" "--stage-caps 5,4" "--stage-caps 7,4" "--stage-caps 8,4" "--stage-caps 6,3" "--stage-caps 6,5"; do
    STEPS=50 timeout -k 10 200 bash scripts/ab.sh "--config cfg5 --inflight 1 $c" - >> gpurun_out/cfg5_caps.txt 2>&1 || { cat gpurun_out/cfg5_caps.txt; exit 1; }
  done
done
for c in "" "--stage-caps 8,4" "--stage-caps 10,4" ""; do
  STEPS=100 timeout -k 10 200 bash scripts/ab.sh "--config cfg5 $c" - >> gpurun_out/cfg5_caps.txt 2>&1 || { cat gpurun_out/cfg5_caps.txt; exit 1; }
done
cut -c1-120 gpurun_out/cfg5_caps.txt
