# config 3 at the driver's command: tail caps and first sets around the final defaults
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
PAIRS=3 bash scripts/ab_args.sh r6sw4 - "--stage-caps 9,2" "--stage-caps 10,2" "--cold-start 0" "--stage-passes 1,3"
