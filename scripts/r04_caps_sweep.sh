#!/bin/bash
# Stage-cap re-sweep after round 3's fast-kernel changes (register/LDS-held gain blocks, the
# output pass): config 3 with three fleets in flight and one batch alone, two alternating rounds.
# Usage: bash scripts/r04_caps_sweep.sh   (outputs: gpurun_out/ab_*.json, one line per run on stdout)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do
  for c in 9,4 8,4 10,4 11,4 9,3 9,5 10,5; do
    STEPS=60 bash scripts/ab.sh "--stage-caps $c" - || exit 1
  done
  for c in 7,4 6,4 8,4 7,3 7,5; do
    STEPS=60 bash scripts/ab.sh "--inflight 1 --stage-caps $c" - || exit 1
  done
done
