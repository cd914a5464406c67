# final measurements, part C: rocprofv3 kernel statistics and the PMC counter groups in flight
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/measure_round.sh r6f profiles/r06 prof
