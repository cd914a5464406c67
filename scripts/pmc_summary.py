"""Summarise rocprofv3 --pmc passes per kernel: python scripts/pmc_summary.py gpurun_out/<tag>"""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1]
tot = defaultdict(lambda: defaultdict(float))
calls = defaultdict(lambda: defaultdict(set))
for f in sorted(glob.glob(tag + "_p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k][r["Counter_Name"]].add(r["Dispatch_Id"])
for k, d in tot.items():
    if "rmpc" not in k and "mpc" not in k:
        continue
    print(k)
    for c, v in sorted(d.items()):
        n = len(calls[k][c])
        print(f"   {c:28s} per-dispatch {v / max(n, 1):16.4g}   (dispatches {n}, total {v:.4g})")
