#!/bin/bash
# Executed VALU work of the library's kernels: fp64 + fp32 op counters (8 SQ counters), then the
# SQ cycle counters, each in its own --pmc pass (kernel counters only), then scripts/pmc_flops.py.
# (PROG="scripts/inflight_run.py --steps 16": the in-flight pipeline alone instead of bench.py)
# Usage: [PROG=...] bash scripts/pmc_flops.sh <tag> <entry kernel substring> [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-flops}; entry=${2:-mpc_ltv_fast_kernel}; shift; shift
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 \
  SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 \
  --output-format csv -d gpurun_out/${tag}_p1 -o run -- python3 ${PROG:-bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in} "$@" \
  > gpurun_out/${tag}_p1.log 2>&1
rc=$?; echo "pass 1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/${tag}_p2 -o run -- python3 ${PROG:-bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in} "$@" \
  > gpurun_out/${tag}_p2.log 2>&1
rc=$?; echo "pass 2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/pmc_flops.py gpurun_out/${tag} gpurun_out/${tag}_flops.json "$entry"
