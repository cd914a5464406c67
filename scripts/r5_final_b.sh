#!/bin/bash
# Round-5 final measurements, part B: bench lines of every configuration, the driver's command
# twice, the 8-rank rehearsal of config 4 on one GPU
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/measure_round.sh r5f profiles/r05 bench
