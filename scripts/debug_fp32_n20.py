"""fp32 lane-per-robot pass vs the fp64 C port: the robots whose u0 misses the 1e-4 bound, with
their iteration counts, status and lane position.  Cases: N=20 with the default obstacles
(2048 robots, the round-2 failing instance), N=30 with the union-8 obstacles (2048 robots,
paired lanes) and BASELINE config 4's full 32768-robot batch.  RMPC_NO_REFINE=1 is set so
the fp32 pass writes its own outputs (the library's default refines them in fp64).
Use with RMPC_LIB_PATH=<variant .so> (scripts/packed_fp32_probe.sh)."""
import os
import sys

import numpy as np

os.environ["RMPC_DIAG"] = "1"
os.environ["RMPC_NO_REFINE"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd"))
import rmpc as rm                                               # noqa: E402
from oracle import cpu, figure8, mpc as ompc                    # noqa: E402
from rmpc import workloads as W                                 # noqa: E402

for N, obs, B in [(20, ompc.default_obstacles(), 2048), (30, W.UNION8_OBS, 2048), (30, W.UNION8_OBS, 32768)]:
    rng = np.random.default_rng(2)
    t0 = (np.arange(B) / B) * (2 * np.pi / 0.5)
    xr, ur = figure8.offset_segments(2.0, 0.5, 0.02, t0, N + 1)
    x0 = xr[:, 0] + rng.normal(0, (0.05, 0.05, 0.1), (B, 3))
    p = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02, precision=1)
    out = rm.batch.mpc_solve_batch(p, x0, xr, ur, obs)
    cp = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
    ref = cpu.mpc_solve_batch(cp, x0, xr, ur, obs, threads=8)
    rel = np.abs(out["u0"] - ref["u0"]).max(axis=1) / np.maximum(1.0, np.abs(ref["u0"]).max(axis=1))
    bad = np.nonzero(rel > 1e-4)[0]
    print(os.environ.get("RMPC_LIB_PATH", "default"), f"N={N} B={B}", "bad", bad.size,
          "max rel %.2e" % rel.max(), flush=True)
    for b in bad[:12]:
        print("  robot", b, "rel %.2e" % rel[b], "iters", out["iters"][b], "ref iters", ref["iters"][b],
              "status", out["status"][b], "wave", b // 64, "lane", b % 64)
