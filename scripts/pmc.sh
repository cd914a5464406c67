#!/bin/bash
# PMC counter passes for the MPC kernels (one pass per counter group; no tracing domains).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-pmc}
rocprofv3 -L > gpurun_out/${tag}_counters.txt 2>&1
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${tag}_p$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-closed-loop > gpurun_out/${tag}_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc ($grp)"
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
exit 0
