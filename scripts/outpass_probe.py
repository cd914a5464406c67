"""Output-pass cost probe (RMPC_DENSE_PROF=1 counters of the fast kernel): the config-3 batch
solved through the host API with and without u_seq / x_pred (want_seq), one batch at a time.
Usage: RMPC_DIAG=1 RMPC_DENSE_PROF=1 python scripts/outpass_probe.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd"))
import rmpc  # noqa: E402
from rmpc import workloads as W  # noqa: E402

B, N = 65536, 20
idx = np.arange(B)
xr, ur = rmpc.batch.figure8_batch(W.t0_at(idx, B), N + 1)
x0 = xr[:, 0] + W.noise_at(idx, 1)
p = rmpc._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
for seq in (True, False, True, False):
    print("want_seq", seq, flush=True)
    sys.stderr.flush()
    rmpc.batch.mpc_solve_batch(p, x0, xr, ur, W.DEFAULT_OBS, step_count=np.full(B, 10, np.int32), want_seq=seq)
    sys.stderr.flush()
