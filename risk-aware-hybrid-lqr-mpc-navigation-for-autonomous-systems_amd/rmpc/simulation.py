"""Batched closed-loop simulations -- the callers of the path (run_simulation.py), on the device.

  run_lqr_simulation      run_simulation.py:34-136
  run_mpc_simulation      run_simulation.py:139-334   (scenarios :191-221, mpc_rate 5, ZOH)
  run_hybrid_simulation   run_simulation.py:413-612   (risk, 10-step dwell, LQR/MPC branch)
  write_logs              SimulationLogger.export_to_csv / export_controls_to_csv column layout
                          (simulation_logger.py:135-235, 402-452)

Each function runs `robots` independent rollouts through one rmpc_rollout_batch call
(references, control and plant stay in HBM for the whole run) and returns the reference's
result dict.  With robots == 1 the arrays have the reference's shapes; otherwise they carry
a leading robot axis and the scalar metrics become per-robot arrays.  Robot r starts at
table row start_index[r] (default 0, as the reference) from the reference there, or x0[r].
"""
import time

import numpy as np

from . import _native as nat
from . import batch

SCENARIOS = {                                    # run_simulation.py:191-221 (x, y, radius)
    "default": [(1.0, 0.5, 0.2), (-0.5, -1.0, 0.25), (1.5, -0.3, 0.15)],
    "sparse": [(1.5, 0.8, 0.2)],
    "dense": [(1.0, 0.5, 0.2), (-0.5, -1.0, 0.25), (1.5, -0.3, 0.15), (-1.5, 0.5, 0.2),
              (0.0, 0.8, 0.15)],
    "corridor": [(1.0, 0.3, 0.15), (1.0, 0.7, 0.15), (-0.8, -0.7, 0.15), (-0.3, -1.2, 0.15)],
}

LQR_Q, LQR_R = [15.0, 15.0, 8.0], [0.1, 0.1]                 # run_simulation.py:54, :439
MPC_KW = dict(Q=[15.0, 15.0, 50.0], R=[0.1, 0.1], P=[30.0, 30.0, 40.0], d_safe=0.3, rho=5000.0,
              v_max=2.0, omega_max=3.0)                      # :164-176, :443-454


def _wrap(a):
    """The reference's while-loop wrap (mpc_controller.py:540-546): +-pi stay as they are."""
    a = np.array(a, dtype=np.float64, copy=True)
    while np.any(a > np.pi):
        a = np.where(a > np.pi, a - 2 * np.pi, a)
    while np.any(a < -np.pi):
        a = np.where(a < -np.pi, a + 2 * np.pi, a)
    return a


def _table(duration, dt, A=2.0, a=0.5):
    """generate(duration) rows [px, py, theta] (reference_generator.py:196-230) on the host,
    for errors and logs (the rollout evaluates the same points on the device)."""
    n = len(np.arange(0, duration, dt))
    t = np.arange(n) * dt
    px = A * np.sin(a * t)
    py = A * np.sin(a * t) * np.cos(a * t)
    dpx = a * A * np.cos(a * t)
    dpy = a * A * (np.cos(a * t) ** 2 - np.sin(a * t) ** 2)
    return np.stack([px, py, np.arctan2(dpy, dpx)], -1)


def _starts(robots, start_index):
    if start_index is None:
        return np.zeros(robots, np.int32)
    s = np.ascontiguousarray(start_index, np.int32).reshape(-1)
    if s.shape[0] != robots:
        raise ValueError("start_index must have one entry per robot")
    return s


def _refs_for(table, starts, steps):
    idx = np.minimum(starts[:, None] + np.arange(steps)[None, :], len(table) - 1)
    return table[idx]                                            # [R, steps, 3]


def _squeeze(d, robots):
    if robots != 1:
        return d
    return {k: (v[0] if isinstance(v, np.ndarray) and v.ndim >= 1 and v.shape[0] == 1 else v)
            for k, v in d.items()}


def run_lqr_simulation(duration=20.0, dt=0.02, robots=1, start_index=None, x0=None, device=0,
                       log_dir=None):
    """run_simulation.py:34-136 for `robots` robots (no plotting)."""
    table = _table(duration, dt)
    steps = len(table) - 1
    starts = _starts(robots, start_index)
    lp = nat.lqr_params(LQR_Q, LQR_R, dt, 2.0, 3.0)
    out = batch.rollout_batch("lqr", steps, lparams=lp, start_index=starts, x0=x0,
                              table_len=len(table), dt=dt, device=device)
    refs = _refs_for(table, starts, steps)
    err = out["states"][:, :-1] - refs                         # lqr_controller.py:209-210
    err[..., 2] = _wrap(err[..., 2])
    en = np.linalg.norm(err[..., :2], axis=-1)
    res = dict(states=out["states"], controls=out["controls"], errors=err,
               reference=np.broadcast_to(table, (robots,) + table.shape),
               mean_error=en.mean(axis=1), final_error=en[:, -1])
    if log_dir:
        write_logs(log_dir, "lqr_sim", out["states"], refs, err, out["controls"], ["LQR"] * steps)
    return _squeeze(res, robots)


def run_mpc_simulation(duration=20.0, dt=0.02, with_obstacles=True, scenario="default", robots=1,
                       start_index=None, x0=None, horizon=6, block_size=2, mpc_rate=5, device=0,
                       log_dir=None):
    """run_simulation.py:139-334 for `robots` robots: solve_with_ltv every mpc_rate steps,
    control held in between, the scenario's obstacles, collision count over the states."""
    table = _table(duration, dt)
    steps = len(table) - 1
    starts = _starts(robots, start_index)
    obs = SCENARIOS.get(scenario, SCENARIOS["default"]) if with_obstacles else []
    k = MPC_KW
    mp = nat.mpc_params(horizon, k["Q"], k["R"], k["P"], k["d_safe"], k["rho"], k["v_max"],
                        k["omega_max"], dt, block_size=block_size)
    t = time.perf_counter()
    out = batch.rollout_batch("mpc", steps, mparams=mp, start_index=starts, x0=x0, obstacles=obs,
                              table_len=len(table), mpc_rate=mpc_rate, dt=dt, device=device)
    wall = time.perf_counter() - t
    n_solves = robots * ((steps + mpc_rate - 1) // mpc_rate)
    refs = _refs_for(table, starts, steps)
    err = out["states"][:, :-1] - refs                           # :264-265
    err[..., 2] = _wrap(err[..., 2])
    en = np.linalg.norm(err[..., :2], axis=-1)
    hit_any = np.zeros(out["states"].shape[:2], bool)          # :292-298, one count per state
    for (ox, oy, r) in obs:                                      # Obstacle.is_collision (:44-46)
        hit_any |= np.hypot(out["states"][..., 0] - ox, out["states"][..., 1] - oy) < r + k["d_safe"]
    coll = hit_any.sum(axis=1)
    res = dict(states=out["states"], controls=out["controls"], errors=err,
               reference=np.broadcast_to(table, (robots,) + table.shape),
               mean_error=en.mean(axis=1), collision_count=coll,
               # amortised over the batch: wall time of the whole rollout / number of solves
               mean_solve_time=np.full(robots, 1e3 * wall / max(n_solves, 1)),
               mpc_status=out["mpc_status"])
    if log_dir:
        write_logs(log_dir, "mpc_sim", out["states"], refs, err, out["controls"], ["MPC"] * steps)
    return _squeeze(res, robots)


def run_hybrid_simulation(duration=20.0, dt=0.02, scenario="default", robots=1, start_index=None,
                          x0=None, horizon=6, block_size=1, device=0, log_dir=None,
                          use_predictive_risk=False):
    """run_simulation.py:413-612 for `robots` robots: risk-threshold switching with a 10-step
    dwell; risk_history is the combined risk of each step's state (:529).

    use_predictive_risk=True (not in the reference's loop, which passes no predicted states):
    a robot whose previous step ran MPC passes that solve's predicted_states to the risk
    assessment (RiskMetrics.compute_predictive_risk, risk_metrics.py:131-171).  risk_history
    then still reports the distance-only combined risk of each state."""
    table = _table(duration, dt)
    steps = len(table) - 1
    starts = _starts(robots, start_index)
    obs = SCENARIOS.get(scenario, SCENARIOS["default"])
    k = MPC_KW
    lp = nat.lqr_params(LQR_Q, LQR_R, dt, 2.0, 3.0)
    mp = nat.mpc_params(horizon, k["Q"], k["R"], k["P"], k["d_safe"], k["rho"], k["v_max"],
                        k["omega_max"], dt, block_size=block_size)
    rp = nat.risk_params(use_predicted=use_predictive_risk)
    out = batch.rollout_batch("hybrid", steps, lparams=lp, mparams=mp, rparams=rp,
                              start_index=starts, x0=x0, obstacles=obs, table_len=len(table),
                              dt=dt, device=device)
    refs = _refs_for(table, starts, steps)
    err = out["states"][:, :-1] - refs                           # :561 (not wrapped)
    en = np.linalg.norm(err[..., :2], axis=-1)
    risk, _, _ = batch.risk_batch(rp, out["states"][:, :-1].reshape(-1, 3), obs, device=device)
    used = out["used_mpc"]
    switches = (used[:, 1:] != used[:, :-1]).sum(axis=1)
    res = dict(states=out["states"], controls=out["controls"], errors=err,
               risk_history=risk[:, 2].reshape(robots, steps),
               controller_used=np.where(used, "MPC", "LQR"),
               lqr_steps=(~used).sum(axis=1), mpc_steps=used.sum(axis=1), switches=switches,
               mean_error=en.mean(axis=1), final_error=en[:, -1], mpc_status=out["mpc_status"])
    if log_dir:
        for r in range(robots):
            write_logs(log_dir, f"hybrid_sim_r{r}", out["states"][r:r + 1], refs[r:r + 1],
                       err[r:r + 1], out["controls"][r:r + 1],
                       ["MPC" if u else "LQR" for u in used[r]])
    return _squeeze(res, robots)


def write_logs(log_dir, tag, states, refs, errors, controls, controller, solve_time_ms=None,
               stamp=None):
    """states_<stamp>.csv / controls_<stamp>.csv with SimulationLogger's columns
    (simulation_logger.py:174-186, 221-227).  One pair per robot (suffix _r<i> when several)."""
    import csv
    import os
    os.makedirs(log_dir, exist_ok=True)
    stamp = stamp or time.strftime("%Y%m%d_%H%M%S")
    paths = []
    R = states.shape[0]
    for r in range(R):
        suf = f"{tag}_{stamp}" + (f"_r{r}" if R > 1 else "")
        sp = os.path.join(log_dir, f"states_{suf}.csv")
        with open(sp, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["timestep", "px", "py", "theta", "px_ref", "py_ref", "theta_ref",
                        "error_px", "error_py", "error_theta", "error_norm"])
            for k in range(errors.shape[1]):
                x, xr, e = states[r, k], refs[r, k], errors[r, k]
                w.writerow([k, float(x[0]), float(x[1]), float(x[2]), float(xr[0]), float(xr[1]),
                            float(xr[2]), float(e[0]), float(e[1]), float(e[2]),
                            float(np.linalg.norm(e))])
        cp = os.path.join(log_dir, f"controls_{suf}.csv")
        with open(cp, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["timestep", "v", "omega", "controller", "solve_time_ms"])
            for k in range(controls.shape[1]):
                st = "" if solve_time_ms is None else float(solve_time_ms)
                w.writerow([k, float(controls[r, k, 0]), float(controls[r, k, 1]), controller[k], st])
        paths.append((sp, cp))
    return paths
