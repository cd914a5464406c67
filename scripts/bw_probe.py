"""Is the fast stage slowed by its gain-tile traffic?  Solve strided subsets of the config-3
batch (the same difficulty mix at every size) and report, per size, the stage times and the
fast kernel's per-wave cycles per PDAS iteration (RMPC_DENSE_PROF=1).  If the per-iteration
cycles grow with the number of concurrently running waves, the waves contend for the memory
system (the 64 B/step/iteration gain rows spill out of L2).
Usage: RMPC_DIAG=1 python scripts/bw_probe.py [sizes...]"""
import json
import os
import subprocess
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd"))
import rmpc                                                     # noqa: E402
from rmpc import workloads as W                                 # noqa: E402

sizes = [int(s) for s in sys.argv[1:]] or [4096, 16384, 32768, 65536]
N, BT = 20, 65536
dev = torch.device("cuda:0")
p = rmpc._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
obs = torch.tensor(W.DEFAULT_OBS, dtype=torch.float64, device=dev)
for B in sizes:
    idx = np.arange(0, BT, BT // B)[:B]
    xr_h, ur_h = rmpc.batch.figure8_batch(W.t0_at(idx, BT), N + 1)
    x0 = torch.from_numpy(xr_h[:, 0] + W.noise_at(idx, 1)).to(dev)
    xr, ur = torch.from_numpy(xr_h).to(dev), torch.from_numpy(ur_h).to(dev)
    out = dict(u0=torch.empty(B, 2, dtype=torch.float64, device=dev),
               status=torch.empty(B, dtype=torch.int32, device=dev),
               iters=torch.empty(B, dtype=torch.int32, device=dev))
    sc = torch.full((B,), 10, dtype=torch.int32, device=dev)
    step = lambda: rmpc.batch.mpc_solve_batch_dev(p, x0, xr, ur, obs, out, step_count=sc)  # noqa: E731
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    rmpc.batch.set_stage_timing(True)
    st = []
    for _ in range(10):
        step()
        torch.cuda.synchronize()
        st.append(rmpc.batch.mpc_stage_times())
    rmpc.batch.set_stage_timing(False)
    st = np.mean(np.asarray(st), axis=0).tolist()
    its = out["iters"].cpu().numpy()
    rec = dict(B=B, waves=(B + 63) // 64, stage_ms=[round(v, 4) for v in st],
               iters_mean=float(its.mean()), iters_max=int(its.max()),
               beyond_cap=int((its > 7).sum()))
    print(json.dumps(rec), flush=True)
    os.environ["RMPC_DENSE_PROF"] = "1"
    step()
    torch.cuda.synchronize()
    del os.environ["RMPC_DENSE_PROF"]
