"""Closed-loop simulations of run_simulation.py -- oracle restatement (test only).

lqr_closed_loop     run_simulation.py:34-96
mpc_closed_loop     run_simulation.py:139-280  (mpc_rate = 5, ZOH between solves)
hybrid_closed_loop  run_simulation.py:413-576  (risk, 10-step dwell, LQR/MPC branch)
"""
import numpy as np

from .figure8 import Figure8
from .lqr import LQRController
from .mpc import MPCController, default_obstacles
from .plant import simulate_step
from .risk import RiskMetrics


def lqr_closed_loop(duration=20.0, dt=0.02, Q=(15.0, 15.0, 8.0), steps=None, start=0, x0=None):
    g = Figure8(2.0, 0.5, dt)
    tab = g.generate(duration)
    c = LQRController(list(Q), [0.1, 0.1], dt, 2.0, 3.0)
    x = (g.reference_at_index(start)[0] if x0 is None else np.asarray(x0, float)).copy()
    st, ct = [x.copy()], []
    for k in range(len(tab) - 1 if steps is None else steps):
        xr, ur = g.reference_at_index(start + k)
        u, _ = c.compute_control_at_operating_point(x, xr, ur)
        x = simulate_step(x, u, dt, 2.0, 3.0)
        st.append(x.copy())
        ct.append(u)
    return np.array(st), np.array(ct)


def mpc_closed_loop(duration=20.0, dt=0.02, obstacles=None, steps=None, mpc_kwargs=None,
                    mpc_rate=5, start=0, x0=None):
    g = Figure8(2.0, 0.5, dt)
    tab = g.generate(duration)
    kw = dict(horizon=6, Q_diag=[15.0, 15.0, 50.0], R_diag=[0.1, 0.1],
              P_diag=[30.0, 30.0, 40.0], d_safe=0.3, slack_penalty=5000.0, dt=dt,
              v_max=2.0, omega_max=3.0, solver="OSQP", block_size=2)
    kw.update(mpc_kwargs or {})
    c = MPCController(**kw)
    obstacles = default_obstacles() if obstacles is None else obstacles
    x = (g.reference_at_index(start)[0] if x0 is None else np.asarray(x0, float)).copy()
    n = len(tab) - 1 if steps is None else steps
    st, ct = [x.copy()], []
    sol = None
    for k in range(n):
        xr, ur = g.segment(start + k, c.N + 1)
        if k % mpc_rate == 0:
            sol = c.solve_with_ltv(x, xr, ur, obstacles)
        u = sol.optimal_control
        x = simulate_step(x, u, dt, 2.0, 3.0)
        st.append(x.copy())
        ct.append(u)
    return np.array(st), np.array(ct)


def hybrid_closed_loop(duration=20.0, dt=0.02, obstacles=None, steps=None, mpc_kwargs=None,
                       lqr_Q=(15.0, 15.0, 8.0), start=0, x0=None, predictive=False, risk_kwargs=None):
    g = Figure8(2.0, 0.5, dt)
    tab = g.generate(duration)
    lq = LQRController(list(lqr_Q), [0.1, 0.1], dt, 2.0, 3.0)
    kw = dict(horizon=6, Q_diag=[15.0, 15.0, 50.0], R_diag=[0.1, 0.1],
              P_diag=[30.0, 30.0, 40.0], d_safe=0.3, slack_penalty=5000.0, dt=dt,
              v_max=2.0, omega_max=3.0, solver="OSQP")
    kw.update(mpc_kwargs or {})
    c = MPCController(**kw)
    rkw = dict(d_safe=0.3, d_trigger=1.0, alpha=0.6, beta=0.4, threshold_low=0.2,
               threshold_medium=0.5)
    rkw.update(risk_kwargs or {})
    rm = RiskMetrics(**rkw)
    obstacles = default_obstacles() if obstacles is None else obstacles
    x = (g.reference_at_index(start)[0] if x0 is None else np.asarray(x0, float)).copy()
    n = len(tab) - 1 if steps is None else steps
    prev, since = None, 0
    pred = None            # predictive: the last MPC solve's predicted_states (None after LQR)
    st, ct, used = [x.copy()], [], []
    for k in range(n):
        xr, ur = g.reference_at_index(start + k)
        a = rm.assess(x, obstacles, pred)
        if since >= 10:                                              # :533-537
            use_mpc = a["use_mpc"]
        else:
            use_mpc = (prev == "MPC") if prev else a["use_mpc"]
        cur = "MPC" if use_mpc else "LQR"
        if prev is not None and cur != prev:                         # :541-546
            since = 0
        else:
            since += 1
        prev = cur
        if use_mpc:
            xs, us = g.segment(start + k, c.N + 1)
            sol = c.solve_with_ltv(x, xs, us, obstacles)
            u = sol.optimal_control
            pred = sol.predicted_states if predictive else None
        else:
            u, _ = lq.compute_control_at_operating_point(x, xr, ur)
            pred = None
        used.append(use_mpc)
        x = simulate_step(x, u, dt, 2.0, 3.0)
        st.append(x.copy())
        ct.append(u)
    return np.array(st), np.array(ct), np.array(used)


