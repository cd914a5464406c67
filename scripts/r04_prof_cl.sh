cd "${GRAFT_REPO_ROOT:-/root/repo}"; export RMPC_DIAG=1 RMPC_DENSE_PROF=1
timeout -k 10 200 python scripts/closed_loop_warm.py 65536 20 > gpurun_out/cl_prof.out 2> gpurun_out/cl_prof.err || { tail gpurun_out/cl_prof.err; exit 1; }
cat gpurun_out/cl_prof.out
grep -n "\[group\] in=\|waves by loop" gpurun_out/cl_prof.err | awk 'NR%20==0 || NR<3' | cut -c1-300
