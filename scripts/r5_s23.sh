#!/bin/bash
# Round-5 session 23: wave order with the chunked key and lane-broadcast rank kernels
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wave_order" > gpurun_out/r5_s23_t.txt 2>&1 || { tail -30 gpurun_out/r5_s23_t.txt; exit 1; }
tail -1 gpurun_out/r5_s23_t.txt
for wo in 512 0 64; do
  STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight 8 --hw-queues 16 --wave-order $wo" - 2>&1 | cut -c1-120 || exit 1
done
STEPS=30 bash scripts/ab.sh "--warmup 5 --inflight 1 --wave-order 512 --wave-order-alone" - 2>&1 | cut -c1-250 || exit 1
STEPS=20 bash scripts/ab.sh "--warmup 5 --inflight 8 --hw-queues 16 --wave-order 512" - - 2>&1 | cut -c1-120 || exit 1
