# A/B of the multi-pass stage 1 (RMPC_FAST_SPLIT) at the bench defaults, 100 and 20 steps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
STEPS=100 bash scripts/ab.sh "" - "RMPC_FAST_SPLIT=1" "RMPC_FAST_SPLIT=2" "RMPC_FAST_SPLIT=1,3" "RMPC_FAST_SPLIT=3" "RMPC_FAST_SPLIT=1,4" || exit 1
STEPS=20 bash scripts/ab.sh "--warmup 5" - "RMPC_FAST_SPLIT=1" "RMPC_FAST_SPLIT=2" "RMPC_FAST_SPLIT=1,3" - "RMPC_FAST_SPLIT=1" "RMPC_FAST_SPLIT=2" "RMPC_FAST_SPLIT=1,3"
