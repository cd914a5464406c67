# batches in flight x hardware queues at the driver's command and at 100 steps (config 3), and config 4 at 20 steps
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
PAIRS=4 bash scripts/ab_args.sh r6ifc - "--inflight 10" "--inflight 10 --hw-queues 32" "--inflight 5" || exit 1
PAIRS=2 ARGS="--steps 100" bash scripts/ab_args.sh r6ifch - "--inflight 10" "--inflight 10 --hw-queues 32" || exit 1
PAIRS=2 ARGS="--steps 20 --warmup 5 --config cfg4" bash scripts/ab_args.sh r6ifc4 - "--inflight 10" "--inflight 5"
