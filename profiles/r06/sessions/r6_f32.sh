# config 3 through the fp32-request pipeline (fp32 active sets, fp64 refinement: fp64-exact outputs) vs fp64
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
PAIRS=2 bash scripts/ab_args.sh r6f32 - "--f32" || exit 1
PAIRS=1 ARGS="--steps 100" bash scripts/ab_args.sh r6f32h - "--f32"
