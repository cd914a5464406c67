cd "${GRAFT_REPO_ROOT:-/root/repo}"
PAIRS=5 bash scripts/ab_args.sh r6ab1 - "--stage-passes 1" "--stage-passes 1 --stage-caps 12,3" || exit 1
PAIRS=2 ARGS="--steps 100" bash scripts/ab_args.sh r6ab1h - "--stage-passes 1" "--stage-passes 1 --stage-caps 12,3"
