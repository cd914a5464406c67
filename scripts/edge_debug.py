"""Replay test_mpc_edge_cases step by step with flushed progress (debug helper)."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests'))
import conftest  # noqa: F401  (paths)
import rmpc as rm
from oracle import mpc as ompc
from test_gpu_parity import _workload

def say(*a):
    print(time.strftime('%X'), *a, flush=True)

obs = ompc.default_obstacles()
p = rm._native.mpc_params(6, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02, block_size=2)
say('empty')
out = rm.batch.mpc_solve_batch(p, np.zeros((0, 3)), np.zeros((0, 7, 3)), np.zeros((0, 7, 2)), obs)
say('empty ok')
x0, xr, ur = _workload(6, 6, 11, (0.1, 0.1, 0.2))
xr[0, :, 2] = np.linspace(3.05, 3.05 + 0.3, 7)
xr[0, :, 2] = (xr[0, :, 2] + np.pi) % (2 * np.pi) - np.pi
x0[1, 2] += 4 * np.pi
ur[2, :, 0] = 0.004
xr[3, 2, :2] = obs[0][:2]
xr[4, :, :2] = np.array(obs[1][:2]) + 0.25
for b in range(6):
    say('robot', b)
    out = rm.batch.mpc_solve_batch(p, x0[b:b + 1], xr[b:b + 1], ur[b:b + 1], obs)
    say('robot', b, 'status', out['status'], 'iters', out.get('iters'))
say('batch of 6')
sc = np.zeros(6, np.int32)
out = rm.batch.mpc_solve_batch(p, x0, xr, ur, obs, step_count=sc)
say('batch ok', out['status'])
x0n = x0.copy()
x0n[5, 0] = np.nan
say('nan batch')
out = rm.batch.mpc_solve_batch(p, x0n, xr, ur, obs)
say('nan ok', out['status'])
pl = rm._native.mpc_params(6, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02, ltv=False)
say('lti')
out = rm.batch.mpc_solve_batch(pl, x0[:3], xr[:3, :3], ur[:3, :2], obs)
say('lti ok', out['status'])
