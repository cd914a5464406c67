# config 4 in flight with the one-lane fp32 stage: passes and caps around (14, 6)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
PAIRS=2 ARGS="--steps 30 --config cfg4" bash scripts/ab_args.sh r6c4s - "--stage-passes 2" "--stage-passes 3" "--stage-caps 12,6" "--stage-caps 16,6" "--stage-caps 14,4"
