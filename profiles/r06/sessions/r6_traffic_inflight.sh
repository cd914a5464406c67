# PMC HBM traffic per launch of the in-flight pipeline (config 3, the bench's settings), for roofline.traffic_in_flight
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=32 PROG="scripts/inflight_run.py --steps 20 --inflight 10" bash scripts/pmc_hbm.sh r6hbi "mpc_group_kernel<20" > gpurun_out/r6hbi.log 2>&1 || { tail gpurun_out/r6hbi.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r6hbi_traffic.json'));print('%.4g'%d['traffic_bytes_per_launch'], {k:(round(v['traffic_bytes']/1e6,1), v['dispatches_per_launch']) for k,v in d['kernels'].items()})"
