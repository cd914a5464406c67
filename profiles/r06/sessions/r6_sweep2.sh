# config 3 around the new defaults (10 on 32 queues, passes (1)); config 5 and LTI in-flight options
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
PAIRS=3 bash scripts/ab_args.sh r6sw3 - "--inflight 12" "--inflight 16" "--stage-caps 10,3" "--stage-caps 8,3" || exit 1
PAIRS=2 ARGS="--steps 30 --config cfg5" bash scripts/ab_args.sh r6sw5 - "--stage-passes 1" "--inflight 10 --hw-queues 32" || exit 1
PAIRS=2 ARGS="--steps 30 --lti" bash scripts/ab_args.sh r6swl - "--inflight 10 --hw-queues 32"
