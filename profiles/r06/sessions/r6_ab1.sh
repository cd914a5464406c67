cd "${GRAFT_REPO_ROOT:-/root/repo}"
PAIRS=5 bash scripts/ab_args.sh r6ab1 - "--stage-passes 1" "--stage-passes 1 --stage-caps 12,3" || exit 1
PAIRS=2 ARGS="--steps 100" bash scripts/ab_args.sh r6ab1h - "--stage-passes 1" "--stage-passes 1 --stage-caps 12,3"
PAIRS=2 ARGS="--steps 30 --config cfg4" bash scripts/ab_args.sh r6ab1c4 - "--stage-passes 2" "--stage-passes 4" "--stage-passes 2,6"
PAIRS=2 ARGS="--steps 30 --lti" bash scripts/ab_args.sh r6ab1lti - "--stage-passes 1" "--stage-passes 2"
