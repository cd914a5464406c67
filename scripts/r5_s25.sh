#!/bin/bash
# Round-5 session 25: leaner wave-order kernels: durations, parity, in-flight A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wave_order" > gpurun_out/r5_s25_t.txt 2>&1 || { tail -30 gpurun_out/r5_s25_t.txt; exit 1; }
tail -1 gpurun_out/r5_s25_t.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_s25_prof -o run --output-format csv -- python3 bench.py \
    --inflight 1 --wave-order 512 --wave-order-alone --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in \
    > gpurun_out/r5_s25_prof.json 2> gpurun_out/r5_s25_prof.err || { tail gpurun_out/r5_s25_prof.err; exit 1; }
python -c "
import csv
for r in csv.DictReader(open('gpurun_out/r5_s25_prof/run_kernel_stats.csv')):
    print(r['Name'][:50], r['Calls'], r['AverageNs'])" | head -6
for wo in 512 0 256; do
  STEPS=100 bash scripts/ab.sh "--warmup 10 --inflight 8 --hw-queues 16 --wave-order $wo" - 2>&1 | cut -c1-120 || exit 1
done
