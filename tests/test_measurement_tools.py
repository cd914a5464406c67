"""The PMC post-processing behind bench.py's roofline.traffic / frac_executed (scripts/
pmc_common.py): counters collected in separate rocprofv3 passes, summed over every dispatch of
a library call's kernels and divided by the calls (the entry kernel's dispatches)."""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

from pmc_common import per_launch  # noqa: E402

FIELDS = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]


def _pass(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(FIELDS, r)))


def test_per_launch_sums_dispatches_and_normalises_by_entry_calls(tmp_path):
    """Two library calls per pass.  Each call: the fp32 pass and the fp64 refinement (two
    instances of the fast template), the tail twice (its second launch takes the refinement's
    hand-ons), the generic kernel once; a kernel outside the library is ignored.  FETCH_SIZE in
    pass 1, WRITE_SIZE in pass 2."""
    tag = str(tmp_path / "x")
    f32 = "void rmpc::mpc_ltv_fast_kernel<30, 1, float, false, 8, 2, true>(MpcFastArgs)"
    f64 = "void rmpc::mpc_ltv_fast_kernel<30, 1, double, false, 8, 2, true>(MpcFastArgs)"
    grp = "void rmpc::mpc_group_kernel<30, 1, 32, double, false, false>(rmpc::GroupArgs)"
    gen = "void rmpc::mpc_solve_kernel<double, true>(rmpc::MpcArgs<double>)"
    for p, counter in ((1, "FETCH_SIZE"), (2, "WRITE_SIZE")):
        rows, d = [], 0
        for call in range(2):
            for name, v in ((f32, 100.0), (f64, 40.0), (grp, 10.0), (grp, 2.0), (gen, 1.0), ("other_kernel", 999.0)):
                d += 1
                rows.append((d, name, counter, v * p))
        _pass(f"{tag}_p{p}/run/counter_collection.csv", rows)
    ks, launches, per = per_launch(tag, "mpc_ltv_fast_kernel<30, 1, float")
    assert launches == 2
    fast32 = ks["fast<30, 1, float, false, 8, 2, true>"]
    assert fast32 == {"FETCH_SIZE": 100.0, "WRITE_SIZE": 200.0}
    assert ks["group<30, 1, 32, double, false, false>"]["FETCH_SIZE"] == 12.0      # both tail launches
    assert per["group<30, 1, 32, double, false, false>"] == 2.0
    assert ks["generic<double, true>"]["WRITE_SIZE"] == 2.0
    assert not any("other" in k for k in ks)
