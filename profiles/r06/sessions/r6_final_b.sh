# final measurements, part B: every bench line, the driver's command twice, the 8-rank rehearsal
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/measure_round.sh r6f profiles/r06 bench
