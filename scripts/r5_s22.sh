#!/bin/bash
# Round-5 session 22: where the order list's cost goes (per-phase cycle counters, one batch)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PROF=1 STEPS=30 bash scripts/ab.sh "--warmup 5 --inflight 1 --wave-order 64 --wave-order-alone" - 2>&1 | cut -c1-400 || exit 1
PROF=1 STEPS=30 bash scripts/ab.sh "--warmup 5 --inflight 1 --wave-order 0" - 2>&1 | cut -c1-400 || exit 1
