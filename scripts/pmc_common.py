"""Per-launch sums of rocprofv3 --pmc counters over the kernels of one library call.

rocprofv3's counter_collection.csv has one row per (dispatch, counter).  A "launch" is one
library call (rmpc_mpc_solve_batch_dev, or one hybrid step): its kernels may run once (the fast
stage), twice (config 4's fp32 pass and fp64 refinement are two instances of one template; the
tail runs again for the refinement's hand-ons) or not at all.  So every counter is summed over
all dispatches of each kernel and divided by the number of launches, counted as the dispatches
of the call's entry kernel (the first kernel of every call: `entry`, a substring of its name).
"""
import csv
import glob
from collections import defaultdict

FAMILIES = (("mpc_ltv_fast_kernel", "fast"), ("mpc_group_kernel", "group"), ("mpc_solve_kernel", "generic"),
            ("lqr_control_kernel", "lqr"), ("hybrid_decide_kernel", "decide"))


def family(name):
    for sub, fam in FAMILIES:
        if sub in name:
            return fam
    return None


def per_launch(tag, entry):
    """{short kernel name: {counter: per-launch sum}}, launches, {short name: dispatches per launch}"""
    sums = defaultdict(lambda: defaultdict(float))
    cfiles = defaultdict(lambda: defaultdict(set))     # passes that collected each counter
    disp = defaultdict(set)
    for f in sorted(glob.glob(tag + "_p*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if family(name) is None:
                continue
            sums[name][r["Counter_Name"]] += float(r["Counter_Value"])
            cfiles[name][r["Counter_Name"]].add(f)
            disp[name].add((f, r["Dispatch_Id"]))
    ent = [n for n in disp if entry in n]
    if not ent:
        raise SystemExit(f"no dispatch of the entry kernel {entry!r}")
    # dispatches of the entry kernel per pass (every pass runs the same program)
    passes = len({f for n in ent for f, _ in disp[n]})
    launches = sum(len(disp[n]) for n in ent) / max(passes, 1)
    out, per = {}, {}
    for name, d in sums.items():
        short = family(name) + name[name.find("<"):name.find(">") + 1] if "<" in name else family(name)
        out[short] = {c: v / len(cfiles[name][c]) / launches for c, v in d.items()}
        per[short] = len(disp[name]) / (len({f for f, _ in disp[name]}) or 1) / launches
    return out, launches, per
