#!/bin/bash
# Batches in flight against the process's hardware queues (GPU_MAX_HW_QUEUES, HIP default 4):
# config 3 with 3-6 batches in flight at 4 and 8 queues
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
STEPS=60 bash scripts/ab.sh "" "-" "GPU_MAX_HW_QUEUES=8" || exit 1
STEPS=60 bash scripts/ab.sh "--inflight 4" "-" "GPU_MAX_HW_QUEUES=8" || exit 1
STEPS=60 bash scripts/ab.sh "--inflight 6" "GPU_MAX_HW_QUEUES=8" || exit 1
STEPS=60 bash scripts/ab.sh "--inflight 8" "GPU_MAX_HW_QUEUES=8" || exit 1
STEPS=20 bash scripts/ab.sh "" "-" "GPU_MAX_HW_QUEUES=8" || exit 1
STEPS=20 bash scripts/ab.sh "--inflight 6" "GPU_MAX_HW_QUEUES=8" || exit 1
# config 4, one batch alone: first-stage (fp32 pass) and tail caps
STEPS=30 bash scripts/ab.sh "--config cfg4 --inflight 1" "-" || exit 1
for c in 8,6 10,6 10,8 12,8 16,6; do
  STEPS=30 bash scripts/ab.sh "--config cfg4 --inflight 1 --stage-caps $c" "-" || exit 1
done
# clean rocprofv3 kernel statistics of one config-3 batch (no drop-in calls in the run)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4h_prof_cfg3_inflight1 -o run --output-format csv \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in --inflight 1 \
  > gpurun_out/r4h_prof_cfg3_inflight1_bench.json 2> gpurun_out/r4h_prof.err || exit 1
