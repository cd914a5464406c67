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


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def test_bench_reads_the_newest_committed_pmc_profiles():
    """bench.py's roofline reads the newest profiles/r*/pmc_*.json of each workload: every file
    it names exists, holds the keys it reads, and is the newest round's."""
    bench = _bench()
    for name in ("pmc_traffic.json", "pmc_flops.json", "pmc_traffic_cfg4.json", "pmc_flops_cfg4.json",
                 "pmc_traffic_cfg5.json", "pmc_flops_cfg5.json", "pmc_traffic_inflight.json",
                 "pmc_flops_inflight.json", "pmc_traffic_inflight_cfg4.json", "pmc_flops_inflight_cfg4.json"):
        d, src = bench.latest_profile(name)
        assert d is not None, name
        rounds = sorted(p for p in os.listdir(os.path.join(ROOT, "profiles"))
                        if os.path.exists(os.path.join(ROOT, "profiles", p, name)))
        assert src == os.path.join("profiles", rounds[-1], name)
        key = "traffic_bytes_per_launch" if "traffic" in name else "fp64_flops_per_launch"
        assert d[key] > 0, (name, key)
    assert bench.latest_profile("no_such_profile.json") == (None, None)


def test_bench_roofline_fields_from_profiles():
    """pmc_into_roofline: traffic and executed flops per launch from the one-batch profiles,
    the in-flight ones scaled by the timed loop's launch rate; fractions against the FP64 and
    FP32 vector peaks."""
    bench = _bench()
    alg, k_avg, rate = 113e6, 344e-6, 6923.0
    roof = {}
    bench.pmc_into_roofline(roof, "", alg, k_avg, rate)
    tr, _ = bench.latest_profile("pmc_traffic.json")
    fl, _ = bench.latest_profile("pmc_flops.json")
    fi, _ = bench.latest_profile("pmc_flops_inflight.json")
    ti, _ = bench.latest_profile("pmc_traffic_inflight.json")
    assert roof["traffic"] == tr["traffic_bytes_per_launch"]
    assert abs(roof["traffic_vs_algorithmic"] - tr["traffic_bytes_per_launch"] / alg) < 1e-12
    e64, e32 = fl["fp64_flops_per_launch"], fl.get("fp32_flops_per_launch", 0.0)
    want = (e64 / bench.FP64_PEAK_TFLOPS + e32 / bench.FP32_PEAK_TFLOPS) / 1e12 / k_avg
    assert abs(roof["frac_executed"] - want) < 1e-12
    assert roof["traffic_in_flight"] == ti["traffic_bytes_per_launch"]
    e64, e32 = fi["fp64_flops_per_launch"], fi.get("fp32_flops_per_launch", 0.0)
    want = (e64 / bench.FP64_PEAK_TFLOPS + e32 / bench.FP32_PEAK_TFLOPS) * rate / 1e12
    assert abs(roof["frac_executed_in_flight"] - want) < 1e-12
    assert 0 < roof["frac_executed_in_flight"] < 1 and 0 < roof["frac_executed"] < 1
    # one batch alone (no launch rate): no in-flight fields
    alone = {}
    bench.pmc_into_roofline(alone, "_cfg4", alg, k_avg, None)
    assert "traffic" in alone and "traffic_in_flight" not in alone and "frac_executed_in_flight" not in alone
    # config 4 in flight: its own in-flight traffic (the one-lane stage), below the one-batch figure
    c4 = {}
    bench.pmc_into_roofline(c4, "_cfg4", alg, k_avg, rate)
    assert c4["traffic_in_flight"] < c4["traffic"]
