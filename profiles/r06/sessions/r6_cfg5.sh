# config 5 in flight: side streams and in-flight count
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
PAIRS=2 ARGS="--steps 30 --config cfg5" bash scripts/ab_args.sh r6c5 - "--inflight-side 0" "--inflight 10 --hw-queues 32 --inflight-side 0" "--inflight 6"
