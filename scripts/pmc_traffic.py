"""HBM traffic per MPC launch from rocprofv3 --pmc passes (separate FETCH_SIZE / WRITE_SIZE runs).

Usage: python scripts/pmc_traffic.py gpurun_out/<tag> profiles/r01/pmc_traffic.json

Corrections from the MI355X guide (HBM section): FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads, so it is doubled; WRITE_SIZE is exact
for 16-B-per-lane stores.  One "launch" = the three kernels of one rmpc_mpc_solve_batch_dev call.
"""
import csv
import glob
import json
import sys
from collections import defaultdict

tag, out = sys.argv[1], sys.argv[2]
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(tag + "_p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        key = ("fast" if "mpc_ltv_fast_kernel" in name else "dense" if "mpc_dense_kernel" in name
               else "group" if "mpc_group_kernel" in name
               else "generic" if "mpc_solve_kernel" in name else None)
        if key and r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {"note": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes; bytes = KiB*1024; "
               "FETCH doubled (gfx950 reports half of wide reads); per dispatch, averaged",
       "kernels": {}}
total = 0.0
for k, d in vals.items():
    fetch = 2 * 1024 * sum(d["FETCH_SIZE"]) / max(len(d["FETCH_SIZE"]), 1)
    write = 1024 * sum(d["WRITE_SIZE"]) / max(len(d["WRITE_SIZE"]), 1)
    res["kernels"][k] = {"fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write}
    total += fetch + write
res["traffic_bytes_per_launch"] = total
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
