#!/bin/bash
# Round-5 session 24: wave-order kernels' own durations (rocprofv3) and the in-flight A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_s24_prof -o run --output-format csv -- python3 bench.py \
    --inflight 1 --wave-order 512 --wave-order-alone --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
    > gpurun_out/r5_s24_prof.json 2> gpurun_out/r5_s24_prof.err || { tail gpurun_out/r5_s24_prof.err; exit 1; }
cut -d, -f1-4 gpurun_out/r5_s24_prof/run_kernel_stats.csv | head -8
for wo in 512 0; do
  STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight 8 --hw-queues 16 --wave-order $wo" - 2>&1 | cut -c1-120 || exit 1
done
