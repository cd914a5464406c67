#!/bin/bash
# Round-5 session 20: device wave order with one-wave key / rank kernels
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wave_order" > gpurun_out/r5_s20_t.txt 2>&1 || { tail -30 gpurun_out/r5_s20_t.txt; exit 1; }
tail -1 gpurun_out/r5_s20_t.txt
for cfg in "8 16 512" "8 16 0" "3 4 512" "3 4 0" "8 16 1024"; do
  set -- $cfg
  STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight $1 --hw-queues $2 --wave-order $3" - 2>&1 | cut -c1-120 || exit 1
  STEPS=20 bash scripts/ab.sh "--warmup 5 --inflight $1 --hw-queues $2 --wave-order $3" - 2>&1 | cut -c1-120 || exit 1
done
