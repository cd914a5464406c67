#!/bin/bash
# Upper bound of what removing the stage-1 gain-tile traffic could save (round-3 review, item 4):
# two diagnostics builds that run every robot to the stage-1 cap and drop its outputs
# (RMPC_NOCERT), one of them without any tile traffic (RMPC_GAIN_NOMEM, wrong gains);
# their fast-kernel times (rocprofv3, one batch at a time) and in-flight rates compare the same
# sweeps with and without the tile.  Then the default bench line on the current tree.
# Build first: bash scripts/build_variant.sh nocert -DRMPC_NOCERT=1;
#              bash scripts/build_variant.sh nocert_nomem -DRMPC_NOCERT=1 -DRMPC_GAIN_NOMEM=1
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/gt; export TMPDIR=/tmp
L=$PWD/risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd/rmpc
B="--steps 30 --warmup 3 --no-cpu-baseline --no-pcie --no-closed-loop --no-drop-in"
for v in nocert nocert_nomem; do
  RMPC_DIAG=1 RMPC_LIB_PATH=$L/librmpc_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      -d gpurun_out/gt/$v -o run -- python3 bench.py --inflight 1 $B > gpurun_out/gt/$v.json 2> gpurun_out/gt/$v.err || exit 1
  RMPC_DIAG=1 RMPC_LIB_PATH=$L/librmpc_$v.so timeout -k 10 200 python3 bench.py $B > gpurun_out/gt/${v}_inflight.json \
      2> gpurun_out/gt/${v}_inflight.err || exit 1
done
# per-call stream-order event recorded only when a context changes streams (RMPC_LAZY_ORDER)
STEPS=50 timeout -k 10 500 bash scripts/ab.sh "--inflight 1" - "RMPC_LIB_PATH=$L/librmpc_lazy.so" - "RMPC_LIB_PATH=$L/librmpc_lazy.so" \
    > gpurun_out/gt/lazy_ab.txt 2>&1 || exit 1
STEPS=50 timeout -k 10 500 bash scripts/ab.sh "" - "RMPC_LIB_PATH=$L/librmpc_lazy.so" >> gpurun_out/gt/lazy_ab.txt 2>&1 || exit 1
cat gpurun_out/gt/lazy_ab.txt | cut -c1-200
timeout -k 10 400 python3 bench.py > gpurun_out/gt/default.json 2> gpurun_out/gt/default.err || exit 1
python3 - <<'EOF'
import csv, glob, json
for v in ["nocert", "nocert_nomem"]:
    f = glob.glob(f"gpurun_out/gt/{v}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "mpc_ltv_fast_kernel" in r["Name"]:
            print(v, r["Name"][:80], "calls", r["Calls"], "avg us %.1f" % (float(r["AverageNs"]) / 1e3))
    d = json.load(open(f"gpurun_out/gt/{v}_inflight.json"))
    print(v, "in flight %.4e" % d["value"], "ms/step %.4f" % d["ms_per_step"])
d = json.load(open("gpurun_out/gt/default.json"))
print("default", json.dumps({k: d.get(k) for k in ["value", "value_one_batch_alone", "ms_per_step"]}),
      json.dumps({k: d["roofline"].get(k) for k in ["kernel_avg_ms", "launch_ms_own_events", "frac"]}))
EOF
