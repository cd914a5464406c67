"""Generate the committed golden fixtures under tests/golden/ (build container only).

Run once here, where /root/reference exists:  python tests/golden/make_golden.py

Two kinds of fixture, both pure data (inputs + expected outputs):

1. Vectors produced by importing the reference's own modules in this container
   (lqr_controller.py, reference_generator.py, differential_drive.py,
   risk_metrics.py).  mpc_controller.py cannot be imported (cvxpy is absent,
   mpc_controller.py:25), so the package __init__ files are bypassed with bare
   namespace modules, as recorded in SURVEY.md 8(c).  No bytecode is written
   into the read-only reference tree.
2. Columns copied from the reference's committed run logs (logs/*.csv), which
   are the only pinned MPC outputs the reference offers.

The reference itself never travels to the GPU box; only these .npz files do.
"""
import csv
import importlib.util
import os
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference"
PKG = os.path.join(REF, "src", "hybrid_controller", "hybrid_controller")
OUT = os.path.dirname(os.path.abspath(__file__))


def _load_reference():
    for name, sub in (("hybrid_controller", ""), ("hybrid_controller.models", "models"),
                      ("hybrid_controller.controllers", "controllers"),
                      ("hybrid_controller.trajectory", "trajectory")):
        m = types.ModuleType(name)
        m.__path__ = [os.path.join(PKG, sub)] if sub else [PKG]
        sys.modules[name] = m
    mods = {}
    for name, rel in (("hybrid_controller.models.linearization", "models/linearization.py"),
                      ("hybrid_controller.models.differential_drive",
                       "models/differential_drive.py"),
                      ("hybrid_controller.controllers.lqr_controller",
                       "controllers/lqr_controller.py"),
                      ("hybrid_controller.controllers.risk_metrics",
                       "controllers/risk_metrics.py"),
                      ("hybrid_controller.trajectory.reference_generator",
                       "trajectory/reference_generator.py")):
        spec = importlib.util.spec_from_file_location(name, os.path.join(PKG, rel))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        mods[name.rsplit(".", 1)[1]] = mod
    return mods


def _csv(stamp, kind):
    with open(os.path.join(REF, "logs", f"{kind}_{stamp}.csv")) as f:
        return list(csv.DictReader(f))


def main():
    ref = _load_reference()
    rng = np.random.default_rng(1234)

    # ---------------------------------------------------------------- Figure-8
    G = ref["reference_generator"].ReferenceTrajectoryGenerator
    g = G(A=2.0, a=0.5, dt=0.02)
    table = g.generate(20.0)
    seg_starts = np.array([0, 1, 250, 500, 993, 995, 998, 999])
    segs_x = np.stack([g.get_trajectory_segment(int(s), 21)[0] for s in seg_starts])
    segs_u = np.stack([g.get_trajectory_segment(int(s), 21)[1] for s in seg_starts])
    t_pts = np.concatenate([[0.0, np.pi, 2 * np.pi, 6.2831853], rng.uniform(0, 40, 60)])
    at_time = np.array([np.concatenate(g.get_reference_at_time(float(t))) for t in t_pts])
    np.savez_compressed(os.path.join(OUT, "figure8.npz"), table=table, seg_starts=seg_starts,
                        segs_x=segs_x, segs_u=segs_u, t_pts=t_pts, at_time=at_time)

    # ---------------------------------------------------------------- plant
    R = ref["differential_drive"].DifferentialDriveRobot(v_max=2.0, omega_max=3.0)
    xs = np.column_stack([rng.uniform(-3, 3, 200), rng.uniform(-3, 3, 200),
                          rng.uniform(-3.3, 3.3, 200)])
    us = np.column_stack([rng.uniform(-3, 3, 200), rng.uniform(-5, 5, 200)])
    xs[:5, 2] = [np.pi, -np.pi, np.pi - 1e-12, 3.2, -3.2]
    euler = np.array([R.simulate_step(x.copy(), u.copy(), 0.02) for x, u in zip(xs, us)])
    rk4 = np.array([R.simulate_step(x.copy(), u.copy(), 0.02, method="rk4")
                    for x, u in zip(xs, us)])
    np.savez_compressed(os.path.join(OUT, "plant.npz"), x=xs, u=us, euler=euler, rk4=rk4,
                        dt=0.02, v_max=2.0, omega_max=3.0)

    # ---------------------------------------------------------------- LQR gains
    L = ref["lqr_controller"].LQRController
    vs = [0.0, 1e-7, 9.9e-7, 1e-3, 0.01, 0.1, 0.5, 0.6617, 1.0, 1.4142, 2.0, -0.5, -1.3]
    ths = list(np.linspace(-np.pi, np.pi, 9)) + list(rng.uniform(-np.pi, np.pi, 4))
    grid = np.array([(v, t) for v in vs for t in ths])
    out = {}
    for tag, Qd in (("sim", [15.0, 15.0, 8.0]), ("default", [10.0, 10.0, 1.0])):
        K = np.zeros((len(grid), 2, 3))
        P = np.zeros((len(grid), 3, 3))
        for i, (v, t) in enumerate(grid):
            c = L(Q_diag=Qd, R_diag=[0.1, 0.1], dt=0.02, v_max=2.0, omega_max=3.0)
            K[i] = c.compute_gain(float(v), float(t), force_recompute=True)
            P[i] = c.P
        out[f"K_{tag}"] = K
        out[f"P_{tag}"] = P
        out[f"Q_{tag}"] = np.array(Qd)
    # compute_control_at_operating_point on random perturbed states (sim weights)
    c = L(Q_diag=[15.0, 15.0, 8.0], R_diag=[0.1, 0.1], dt=0.02, v_max=2.0, omega_max=3.0)
    cx, cxr, cur, cu, ce = [], [], [], [], []
    for i in range(120):
        t0 = rng.uniform(0, 13)
        xr, ur = g.get_reference_at_time(t0)
        x = xr + rng.normal(0, [0.3, 0.3, 1.5])
        if i % 7 == 0:
            x[2] += 2 * np.pi * rng.choice([-2, -1, 1, 2])     # exercise the while-wrap
        if i % 11 == 0:
            x = xr + rng.normal(0, [3.0, 3.0, 0.1])           # saturate the actuators
        u, e = c.compute_control_at_operating_point(x.copy(), xr.copy(), ur.copy())
        cx.append(x), cxr.append(xr), cur.append(ur), cu.append(u), ce.append(e)
    np.savez_compressed(os.path.join(OUT, "lqr.npz"), grid=grid, R=np.array([0.1, 0.1]),
                        dt=0.02, ctl_x=np.array(cx), ctl_xref=np.array(cxr),
                        ctl_uref=np.array(cur), ctl_u=np.array(cu), ctl_e=np.array(ce), **out)

    # ---------------------------------------------------------------- LQR closed loop
    # run_simulation.py:34-96 replayed through the reference, plus the committed log
    c = L(Q_diag=[15.0, 15.0, 8.0], R_diag=[0.1, 0.1], dt=0.02, v_max=2.0, omega_max=3.0)
    x, _ = g.get_reference_at_index(0)
    x = x.copy()
    st, uu = [x.copy()], []
    for k in range(len(table) - 1):
        xr, ur = g.get_reference_at_index(k)
        u, _ = c.compute_control_at_operating_point(x, xr, ur)
        x = R.simulate_step(x, u, 0.02)
        st.append(x.copy())
        uu.append(u)
    lst = _csv("20260208_001916", "states")
    lct = _csv("20260208_001916", "controls")
    log_x = np.array([[float(r[k]) for k in ("px", "py", "theta")] for r in lst])
    log_u = np.array([[float(r["v"]), float(r["omega"])] for r in lct])
    np.savez_compressed(os.path.join(OUT, "lqr_closed_loop.npz"), states=np.array(st),
                        controls=np.array(uu), log_states=log_x, log_controls=log_u)

    # ---------------------------------------------------------------- risk
    Rk = ref["risk_metrics"].RiskMetrics(d_safe=0.3, d_trigger=1.0, alpha=0.6, beta=0.4,
                                        threshold_low=0.2, threshold_medium=0.5)
    obs = [{"x": 1.0, "y": 0.5, "radius": 0.2}, {"x": -0.5, "y": -1.0, "radius": 0.25},
           {"x": 1.5, "y": -0.3, "radius": 0.15}]
    rs = np.column_stack([rng.uniform(-2.5, 2.5, 300), rng.uniform(-1.5, 1.5, 300),
                          rng.uniform(-3, 3, 300)])
    rs[:3, :2] = [[1.0, 0.5 + 0.2 + 0.3], [1.0, 0.5 + 0.2 + 1.0], [1.0, 0.5]]  # boundaries
    pred = rs[:, None, :2] + rng.normal(0, 0.3, (300, 11, 2))
    pred = np.concatenate([pred, np.zeros((300, 11, 1))], -1)
    vals = []
    for s, p in zip(rs, pred):
        a0 = Rk.assess_risk(s, obs)
        a1 = Rk.assess_risk(s, obs, predicted_states=p)
        vals.append([a0.distance_risk, a0.combined_risk, a0.min_obstacle_distance,
                     a0.nearest_obstacle_id, float(a0.use_mpc),
                     a1.predictive_risk, a1.combined_risk, float(a1.use_mpc)])
    np.savez_compressed(os.path.join(OUT, "risk.npz"), states=rs, pred=pred,
                        obstacles=np.array([[o["x"], o["y"], o["radius"]] for o in obs]),
                        vals=np.array(vals))

    # ---------------------------------------------------------------- MPC logs
    # current config (run_simulation.py:164-176), mpc_rate = 5: solve at k % 5 == 0
    lst = _csv("20260208_014109", "states")
    lct = _csv("20260208_014109", "controls")
    ks = np.arange(0, len(lct), 5)
    np.savez_compressed(
        os.path.join(OUT, "mpc_log_014109.npz"), k=ks,
        x0=np.array([[float(lst[k][c]) for c in ("px", "py", "theta")] for k in ks]),
        u0=np.array([[float(lct[k]["v"]), float(lct[k]["omega"])] for k in ks]),
        solve_ms=np.array([float(lct[k]["solve_time_ms"]) for k in ks]),
        states=np.array([[float(r[c]) for c in ("px", "py", "theta")] for r in lst]),
        controls=np.array([[float(r["v"]), float(r["omega"])] for r in lct]))
    # v0.2 hybrid run: LQR rows + MPC rows (N=10, bs=1, rho=1000)
    lst = _csv("20260208_003249", "states")
    lct = _csv("20260208_003249", "controls")
    np.savez_compressed(
        os.path.join(OUT, "hybrid_log_003249.npz"),
        states=np.array([[float(r[c]) for c in ("px", "py", "theta")] for r in lst]),
        controls=np.array([[float(r["v"]), float(r["omega"])] for r in lct]),
        is_mpc=np.array([r["controller"] == "MPC" for r in lct]))
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
