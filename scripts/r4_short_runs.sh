#!/bin/bash
# The driver times 20 steps: in-flight settings compared at 20 steps (and 100), alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/short_runs.txt
for rep in 1 2; do
  for v in "" "--stage-caps 7,4" "--stage-caps 8,4" "--inflight 2" "--inflight 4"; do
    STEPS=20 timeout -k 10 200 bash scripts/ab.sh "$v" - >> gpurun_out/short_runs.txt 2>&1 || { cat gpurun_out/short_runs.txt; exit 1; }
  done
done
cut -c1-110 gpurun_out/short_runs.txt
