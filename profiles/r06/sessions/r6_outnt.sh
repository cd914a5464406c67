# stage 1's u_seq / x_pred stores non-temporal (RMPC_OUT_NT=1 build) vs the product library
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
L=risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc/librmpc_outnt.so
PAIRS=4 bash scripts/ab_driver.sh r6nt - $L || exit 1
PAIRS=2 ARGS="--steps 100" bash scripts/ab_driver.sh r6nth - $L
