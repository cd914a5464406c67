#!/bin/bash
# Instruction-cache vs memory contention in the fast kernel: PMC passes (one counter set each)
# over scripts/bw_probe.py at 32768 and 65536 robots, fast kernel only.
# Usage: bash scripts/pmc_icache.sh <tag>
export RMPC_DIAG=1
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-ic}
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES" \
           "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex mpc_ltv_fast --output-format csv \
    -d gpurun_out/${tag}_p$i -o run -- python3 scripts/bw_probe.py 32768 65536 > gpurun_out/${tag}_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 - "$tag" <<'EOF'
import csv, glob, sys, collections
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/{tag}_p*/**/*counter_collection.csv", recursive=True)):
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(float)
    for r in rows:
        agg[(int(r["Dispatch_Id"]), int(r["Grid_Size"]), r["Counter_Name"])] += float(r["Counter_Value"])
    print(f)
    for (d, g, c), v in sorted(agg.items()):
        print(f"  dispatch {d:3d} grid {g:6d} {c:24s} {v:.4e}")
EOF
