"""Full-size GPU parity at BASELINE configs 3 and 5 against the INDEPENDENT exact-QP oracle.

The full-batch tests in test_gpu_parity.py compare every robot with the C restatement
(oracle/c), which runs the same active-set algorithm as the kernels.  Here the robots most
likely to expose a wrong certified active set -- every robot that leaves the lane-per-robot
stage for the lane-group tail (projected Newton, up to ~40 iterations), plus a random
sample -- are checked against oracle/qp.py (Mehrotra PDIP + polish on the QP CVXPY is
given, a different algorithm) through the committed fixtures of
tests/golden/make_hard_fixtures.py.  Inputs are regenerated from the same recipe.

Tolerances: |du| <= 1e-9 (fp64 kernels vs the exact QP); LQR branch vs SciPy's
DARE <= 1e-10 (SDA vs QZ Schur, gains ~1e-12).
"""
import os
import sys

import numpy as np
import pytest

from oracle import cpu, figure8, mpc as ompc

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from make_hard_fixtures import cfg3_inputs, cfg5_inputs  # noqa: E402

pytestmark = pytest.mark.gpu
N = 20


@pytest.fixture(scope="module")
def rm(gpu_lib):
    import rmpc
    return rmpc


def test_mpc_cfg3_tail_robots_match_exact_qp_oracle(rm, golden):
    """BASELINE config 3 (65536 robots): every robot the lane-per-robot stage hands to the
    lane-group tail, and 256 others, against the independent exact QP; the fixture's tail
    set must cover every robot the GPU solved in more than the stage's 7 PDAS iterations."""
    fx = golden("hard_cfg3.npz")
    x0, xr, ur = cfg3_inputs()
    p = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
    out = rm.batch.mpc_solve_batch(p, x0, xr, ur, ompc.default_obstacles())
    idx = fx["idx"]
    gpu_tail = np.where(out["iters"] > 7)[0]
    assert np.isin(gpu_tail, idx).all(), np.setdiff1d(gpu_tail, idx)[:10]
    assert len(gpu_tail) > 3000                       # ~5% of the batch: the tail is exercised
    ok = fx["ok"] & (out["status"][idx] == 0)
    assert ok.mean() >= 0.999
    d = np.abs(out["u_seq"][idx] - fx["u_seq"]).max(axis=(1, 2))
    assert np.all(d[ok] <= 1e-9), (d[ok].max(), idx[ok][np.argmax(d[ok])])
    assert np.array_equal(out["slack_used"][idx][ok].astype(bool), fx["slack_used"][ok])
    hardest = idx[np.argsort(fx["cport_iters"])[-20:]]          # the 20 longest solves
    assert np.all(out["status"][hardest] == 0)


def test_hybrid_cfg5_full_batch_matches_oracles(rm, golden):
    """BASELINE config 5 at its own configuration (bench.py --config cfg5): 65536 robots,
    N=20, one hybrid step from the initial switch state (run_simulation.py:513-559).
    - the switch decision of every robot equals oracle/risk.py's (risk_metrics.py:173-222);
    - every MPC-branch robot matches the C port (u0, 1e-9), and every MPC-branch robot that
      goes to the tail (cap 6 on the compacted device list), plus 256 others, matches the
      independent exact QP (1e-9);
    - every LQR-branch robot matches SciPy's DARE + gain + control (lqr_controller.py:191-215).
    The inputs are the bench's: the device Figure-8 kernel reproduces the fixture's numpy
    references to 1e-12."""
    fx = golden("hard_cfg5.npz")
    x0, xr, ur = cfg5_inputs()
    B = len(x0)
    from rmpc import workloads as W
    t0 = W.cfg5_t0(np.arange(B))
    xr_d, ur_d = rm.batch.figure8_batch(t0[::97], N + 1)          # bench.py's device references
    np.testing.assert_allclose(xr_d, xr[::97], atol=1e-12, rtol=0)
    np.testing.assert_allclose(ur_d, ur[::97], atol=1e-12, rtol=0)
    obs = ompc.default_obstacles()
    rp = rm._native.risk_params()
    lp = rm._native.lqr_params([15, 15, 8], [.1, .1], 0.02, 2.0, 3.0)
    mp = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
    state = rm.batch.new_hybrid_state(B)
    state["step_count"][:] = 10                                    # bench.py: past the ramp
    u, used, _ = rm.batch.hybrid_step_batch(rp, lp, mp, x0, xr, ur, obs, state)
    assert np.array_equal(used, fx["use_mpc"])
    assert 0.45 < used.mean() < 0.55
    im = np.where(used)[0]
    # MPC branch, every robot: the C port (same algorithm) at 1e-9
    cp = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
    ref = cpu.mpc_solve_batch(cp, x0[im], xr[im], ur[im], obs, step_count=np.full(len(im), 10, np.int32),
                              threads=8)
    okc = ref["status"] == 0
    assert okc.mean() >= 0.999
    dc = np.abs(u[im] - ref["u0"]).max(axis=1)
    assert np.all(dc[okc] <= 1e-9), dc[okc].max()
    assert np.all(state["step_count"][im][okc] == 11)
    # the tail robots (C-port iterations > 6) and a sample: the independent exact QP
    idx = fx["idx"]
    assert np.isin(im[ref["iters"] > 6], idx).all()
    assert (fx["cport_iters"] > 6).sum() > 3000
    ok = fx["ok"]
    d = np.abs(u[idx] - fx["u0"]).max(axis=1)
    assert np.all(d[ok] <= 1e-9), (d[ok].max(), idx[ok][np.argmax(d[ok])])
    # LQR branch, every robot: SciPy DARE
    il = fx["lqr_idx"]
    assert np.array_equal(il, np.where(~used)[0])
    np.testing.assert_allclose(u[il], fx["lqr_u"], atol=1e-10, rtol=0)
    assert np.all(state["cache"]["valid"][il] == 1)


def test_hybrid_cfg5_tail_robots_vs_device_mpc_iterations(rm, golden, monkeypatch):
    """The fixture's tail set is the one the device pipeline actually hands to the tail: the
    MPC-branch robots solved alone at the hybrid branch's fast cap (6) report more than 6
    iterations exactly for robots in the fixture."""
    fx = golden("hard_cfg5.npz")
    x0, xr, ur = cfg5_inputs()
    im = np.where(fx["use_mpc"])[0]
    monkeypatch.setenv("RMPC_DIAG", "1")   # knobs are read in diagnostics mode only
    monkeypatch.setenv("RMPC_FAST_CAP", "6")
    p = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
    out = rm.batch.mpc_solve_batch(p, x0[im], xr[im], ur[im], ompc.default_obstacles(),
                                   step_count=np.full(len(im), 10, np.int32))
    tail = im[out["iters"] > 6]
    assert np.isin(tail, fx["idx"]).all()
    sel = np.searchsorted(im, fx["idx"])
    d = np.abs(out["u0"][sel] - fx["u0"]).max(axis=1)
    assert np.all(d[fx["ok"]] <= 1e-9), d[fx["ok"]].max()


def _rel(a, b, axes):
    """Per-robot relative error max|a - b| / max(1, max|b|) (the north star's "relative
    control error"; the max(1, .) keeps near-zero controls from dividing by ~0)."""
    return np.abs(a - b).max(axis=axes) / np.maximum(1.0, np.abs(b).max(axis=axes))


@pytest.mark.parametrize("caps", [(0, 0), (14, 6)], ids=["default_caps", "inflight_caps"])
def test_mpc_cfg4_full_size_fp32_matches_fp64(rm, caps, capsys):
    """BASELINE config 4 at its own per-GPU size, exactly `bench.py --config cfg4`'s workload:
    32768 robots, N=30, the union-8 obstacles (run_simulation.py:191-221), fp32 arithmetic,
    device Figure-8 references at t0 = i/B * period, start noise seed 2, step_count 10; once
    with the library's default stage caps and once with the bench's in-flight caps (14, 6).
    Every output the reference returns -- u0, u_seq and x_pred (mpc_controller.py:497-505)
    -- against the fp64 C port, all robots: relative error <= 1e-4 (north star).  The 50
    robots with the largest u_seq error also go through the independent exact QP
    (oracle/qp.py, the QP CVXPY is given)."""
    from concurrent.futures import ThreadPoolExecutor
    from rmpc import workloads as W
    B, N = 32768, 30
    idx = np.arange(B)
    xr, ur = rm.batch.figure8_batch(W.t0_at(idx, B), N + 1)
    x0 = xr[:, 0] + W.noise_at(idx, W.CONFIGS["cfg4"]["seed"])
    obs = W.UNION8_OBS
    p = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02,
                              precision=1)
    rm.batch.set_stage_caps(*caps)
    try:
        out = rm.batch.mpc_solve_batch(p, x0, xr, ur, obs, step_count=np.full(B, 10, np.int32))
    finally:
        rm.batch.set_stage_caps(0, 0)
    cp = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
    ref = cpu.mpc_solve_batch(cp, x0, xr, ur, obs, step_count=np.full(B, 10, np.int32), threads=16)
    both = (out["status"] == 0) & (ref["status"] == 0)
    assert both.mean() >= 0.999, np.bincount(out["status"])
    e_u0 = _rel(out["u0"], ref["u0"], 1)[both]
    e_us = _rel(out["u_seq"], ref["u_seq"], (1, 2))[both]
    e_xp = _rel(out["x_pred"], ref["x_pred"], (1, 2))[both]
    with capsys.disabled():
        print(f"\n[cfg4 32768 caps {caps}] optimal {both.mean():.5f}; max rel u0 {e_u0.max():.2e} "
              f"u_seq {e_us.max():.2e} x_pred {e_xp.max():.2e}; iters mean {out['iters'].mean():.2f} "
              f"max {out['iters'].max()}")
    assert e_u0.max() <= 1e-4 and e_us.max() <= 1e-4 and e_xp.max() <= 1e-4
    # the worst robots against the independent exact QP
    worst = np.where(both)[0][np.argsort(e_us)[-50:]]

    def qp(b):
        oc = ompc.MPCController(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
        oc._step_count = 10
        return oc.solve_with_ltv(x0[b], xr[b], ur[b], obs)
    with ThreadPoolExecutor(8) as ex:
        sols = list(ex.map(qp, worst))
    assert all(s.status == "optimal" for s in sols)
    e_qp = np.array([_rel(out["u_seq"][b], s.control_sequence, (0, 1)) for b, s in zip(worst, sols)])
    e_qx = np.array([_rel(out["x_pred"][b], s.predicted_states, (0, 1)) for b, s in zip(worst, sols)])
    with capsys.disabled():
        print(f"[cfg4 worst 50 vs exact QP] max rel u_seq {e_qp.max():.2e} x_pred {e_qx.max():.2e}")
    assert e_qp.max() <= 1e-4 and e_qx.max() <= 1e-4


@pytest.mark.parametrize("cfg,rank", [("cfg4", 7), ("cfg3", 5)])
def test_mpc_eight_gpu_rank_shard_matches_cpu_port(rm, cfg, rank, capsys):
    """One rank's shard of the 8-GPU job, exactly as `bench.py --gpus 8` builds it on that
    rank: global batch 8 x the per-GPU size (config 4: 262144 robots over 8 GPUs, the
    BASELINE figure; config 3: 524288), robots rank, rank + 8, ... (round-robin), their
    Figure-8 offsets and start noise keyed on the global index.  The rank's 32768 / 65536
    robots against the fp64 C port: u0, u_seq, x_pred (fp64-exact: 1e-9 absolute)."""
    from rmpc import workloads as W
    c = W.CONFIGS[cfg]
    N, world = c["N"], 8
    B_per = 32768 if cfg == "cfg4" else c["B"]
    idx = W.shard_indices(B_per * world, world, rank)
    assert idx.size == B_per
    xr, ur = rm.batch.figure8_batch(W.t0_at(idx, B_per * world), N + 1)
    x0 = xr[:, 0] + W.noise_at(idx, c["seed"])
    p = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02,
                              precision=1 if cfg == "cfg4" else 0)
    out = rm.batch.mpc_solve_batch(p, x0, xr, ur, c["obs"], step_count=np.full(B_per, 10, np.int32))
    cp = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
    ref = cpu.mpc_solve_batch(cp, x0, xr, ur, c["obs"], step_count=np.full(B_per, 10, np.int32), threads=16)
    ok = (out["status"] == 0) & (ref["status"] == 0)
    assert ok.mean() >= 0.999
    d = {k: float(np.abs(out[k][ok] - ref[k][ok]).max()) for k in ("u0", "u_seq", "x_pred")}
    with capsys.disabled():
        print(f"\n[{cfg} rank {rank}/8, {B_per} robots] optimal {ok.mean():.5f} max |diff| {d}")
    assert max(d.values()) <= 1e-9, d


# ------------------------------------------------------------------ LQR API gaps (a11)
def test_lqr_get_lqr_gain_unguarded_and_dt_override(rm):
    """LQRController.get_lqr_gain (lqr_controller.py:217-242): no v_r guard, optional dt
    override, inv(R + B'PB) B'PA -- against SciPy's DARE at the same points.  Tolerance by
    conditioning (tests/lqr_checks.py): |dK| <= 1e-10 on the operating range, 1e-7 |K| down
    to |v_r| = 1e-3; below that (v_r = 5e-7 unguarded: ||P|| ~ 1e9) the two DARE solvers'
    gains differ by up to 5% (SciPy's QZ residual 1.4e-9 against the SDA's 1.3e-11), so the
    check there is the DARE residual, ours no worse than SciPy's.  v_r = 0 has no
    stabilising solution: SciPy raises, and so does the drop-in."""
    from lqr_checks import dare_residual
    from oracle import lqr as olqr
    Qd, Rd = [15.0, 15.0, 8.0], [0.1, 0.1]
    c = rm.LQRController(Qd, Rd, 0.02, 2.0, 3.0)
    o = olqr.LQRController(Qd, Rd, 0.02, 2.0, 3.0)
    for v, th in [(0.5, 0.3), (-1.2, 2.9), (2.0, -3.1), (1e-3, -1.0), (5e-7, 0.1)]:
        for dt in (None, 0.05, 0.02):
            K = c.get_lqr_gain(v, th, dt=dt)
            Ko = o.get_lqr_gain(v, th, dt=dt)
            d = dt or 0.02
            Kb, Pb, st = rm.batch.lqr_gain_batch(rm._native.lqr_params(Qd, Rd, d, 2.0, 3.0), [v], [th],
                                                 guard=False)
            assert st[0] == 0
            np.testing.assert_array_equal(K, Kb[0])
            if abs(v) >= 0.1:
                np.testing.assert_allclose(K, Ko, rtol=0, atol=1e-10)
            elif abs(v) >= 1e-3:
                np.testing.assert_allclose(K, Ko, rtol=0, atol=1e-7 * np.abs(Ko).max())
            from scipy.linalg import solve_discrete_are
            from oracle.plant import discrete_model_explicit
            A, B = discrete_model_explicit(v, th, d)
            Ps = solve_discrete_are(A, B, np.diag(Qd), np.diag(Rd))
            rs = dare_residual(Pb[0], v, th, np.diag(Qd), np.diag(Rd), dt=d, guard=False)
            rr = dare_residual(Ps, v, th, np.diag(Qd), np.diag(Rd), dt=d, guard=False)
            assert rs <= max(4 * rr, 1e-12), (v, th, dt, rs, rr)
    # v_r = 0, theta_r = 0: B = [[dt, 0], [0, 0], [0, dt]] exactly, the y mode is exactly
    # uncontrollable and unstable-marginal -- no stabilising solution: SciPy raises, and so
    # does the drop-in.  (At other headings sin/cos rounding leaves the mode controllable at
    # ~1e-17 and SciPy returns a gain with ||P|| ~ 1e10 or raises, depending on the angle: the
    # reference itself is rounding-dependent there, so no outcome is asserted.)
    with pytest.raises(np.linalg.LinAlgError):
        c.get_lqr_gain(0.0, 0.0)
    with pytest.raises(np.linalg.LinAlgError):
        o.get_lqr_gain(0.0, 0.0)
    assert c.K is None                                   # get_lqr_gain does not touch the cache


def test_lqr_set_weights_invalidates_cache(rm):
    """set_weights (lqr_controller.py:263-278) drops K and P; the next control uses the new
    weights (cache miss at the same operating point)."""
    from oracle import lqr as olqr
    c = rm.LQRController([15.0, 15.0, 8.0], [0.1, 0.1], 0.02, 2.0, 3.0)
    x, xr, ur = np.array([0.1, -0.05, 0.2]), np.array([0.0, 0.0, 0.15]), np.array([0.8, 0.3])
    u1, _ = c.compute_control_at_operating_point(x, xr, ur)
    assert c.gain_computed
    c.set_weights(Q_diag=[5.0, 40.0, 2.0], R_diag=[0.2, 0.05])
    assert not c.gain_computed and c.P is None
    u2, _ = c.compute_control_at_operating_point(x, xr, ur)
    o = olqr.LQRController([5.0, 40.0, 2.0], [0.2, 0.05], 0.02, 2.0, 3.0)
    uo, _ = o.compute_control_at_operating_point(x, xr, ur)
    np.testing.assert_allclose(u2, uo, atol=1e-10, rtol=0)
    assert np.abs(u2 - u1).max() > 1e-3
    Q, R = c.get_cost_matrices()
    assert np.allclose(np.diag(Q), [5.0, 40.0, 2.0]) and np.allclose(np.diag(R), [0.2, 0.05])


# ------------------------------------------------------------------ MPC drop-in gaps (a5, a2)
def test_mpc_fallback_solution_matches_in_library_law(rm):
    """MPCController._get_fallback_solution (mpc_controller.py:316-343) equals the fallback
    law the library applies to a robot whose data is not finite, and the oracle's."""
    c = rm.MPCController(6, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02, "OSQP", 2)
    o = ompc.MPCController(6, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02, "OSQP", 2)
    xr, ur = figure8.offset_segments(2.0, 0.5, 0.02, np.array([1.3]), 7)
    x0 = xr[0, 0] + np.array([0.4, -0.3, 2.5])
    fb = c._get_fallback_solution(x0, xr[0], ur[0], 1.25)
    so = o.fallback(x0, xr[0], ur[0])
    assert fb.status == "fallback" and fb.cost == float("inf") and fb.solve_time_ms == 1.25
    np.testing.assert_allclose(fb.optimal_control, so.optimal_control, atol=1e-15)
    np.testing.assert_array_equal(fb.control_sequence, np.tile(fb.optimal_control, (6, 1)))
    np.testing.assert_array_equal(fb.predicted_states, np.tile(x0, (7, 1)))
    # the device law: a NaN reference heading past row 0 makes the linearisation (and so the
    # QP data) non-finite -- CVXPY fails and the reference falls back (:521-522).  (A NaN
    # reference POSITION would not: its obstacle rows fail `dist > 0.01` and are skipped.)
    xr_bad = xr[0].copy()
    xr_bad[3, 2] = np.nan
    s = c.solve_with_ltv(x0, xr_bad, ur[0], ompc.default_obstacles())
    assert s.status == "fallback"
    np.testing.assert_allclose(s.optimal_control, fb.optimal_control, atol=1e-15)


def test_mpc_batches_in_flight_on_two_streams(rm):
    """Two solver contexts of one device (rmpc slots 0 and 1) with config-3 batches in flight
    on two streams at once (bench.py --inflight): every output of both equals a solve alone,
    bit for bit, for four overlapped launches (the contexts share no scratch)."""
    import torch
    x0h, xrh, urh = cfg3_inputs()
    dev = torch.device("cuda:0")
    x0, xr, ur = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x0h, xrh, urh))
    obs = torch.tensor(ompc.default_obstacles(), dtype=torch.float64, device=dev).reshape(-1, 3)
    B = x0.shape[0]
    p = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)

    def outs():
        return dict(u0=torch.empty(B, 2, dtype=torch.float64, device=dev),
                    u_seq=torch.empty(B, N, 2, dtype=torch.float64, device=dev),
                    x_pred=torch.empty(B, N + 1, 3, dtype=torch.float64, device=dev),
                    cost=torch.empty(B, dtype=torch.float64, device=dev),
                    status=torch.empty(B, dtype=torch.int32, device=dev),
                    iters=torch.empty(B, dtype=torch.int32, device=dev))
    alone = outs()
    rm.batch.mpc_solve_batch_dev(p, x0, xr, ur, obs, alone,
                                 step_count=torch.full((B,), 10, dtype=torch.int32, device=dev))
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    o = [outs() for _ in range(2)]
    sc = [torch.full((B,), 10, dtype=torch.int32, device=dev) for _ in range(2)]
    for k in range(4):
        i = k % 2
        with torch.cuda.stream(streams[i]):   # ordered before the slot's solve that reads it
            sc[i].fill_(10)
        rm.batch.mpc_solve_batch_dev(p, x0, xr, ur, obs, o[i], step_count=sc[i], stream=streams[i], slot=i)
    torch.cuda.synchronize()
    for i in range(2):
        for key in alone:
            assert torch.equal(o[i][key], alone[key]), (i, key)
    assert int((alone["status"] == 0).sum()) == B


def test_mpc_stage_caps_same_optimum(rm):
    """rmpc_ctx_set_stage_caps (9, 4), the in-flight bench setting, on its own context: every
    config-3 robot reaches the same optimum as with the library default (7, 4) (|du| <= 1e-9,
    all optimal), robots certify in the lane-per-robot stage after 8-9 PDAS solves, and caps
    outside [0, 64] are rejected."""
    import torch
    x0h, xrh, urh = cfg3_inputs()
    dev = torch.device("cuda:0")
    x0, xr, ur = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x0h, xrh, urh))
    obs = torch.tensor(ompc.default_obstacles(), dtype=torch.float64, device=dev).reshape(-1, 3)
    B = x0.shape[0]
    p = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
    res = []
    for slot, caps in ((0, (0, 0)), (2, (9, 4))):
        rm.batch.set_stage_caps(*caps, slot=slot)
        o = dict(u0=torch.empty(B, 2, dtype=torch.float64, device=dev),
                 u_seq=torch.empty(B, N, 2, dtype=torch.float64, device=dev),
                 status=torch.empty(B, dtype=torch.int32, device=dev),
                 iters=torch.empty(B, dtype=torch.int32, device=dev))
        rm.batch.mpc_solve_batch_dev(p, x0, xr, ur, obs, o,
                                     step_count=torch.full((B,), 10, dtype=torch.int32, device=dev), slot=slot)
        torch.cuda.synchronize()
        res.append({k: v.cpu().numpy() for k, v in o.items()})
    a, b = res
    assert np.all(a["status"] == 0) and np.all(b["status"] == 0)
    assert np.abs(a["u_seq"] - b["u_seq"]).max() <= 1e-9
    assert np.isin([8, 9], b["iters"]).all()
    with pytest.raises(rm.RmpcError):
        rm.batch.set_stage_caps(65, 4, slot=2)
    rm.batch.set_stage_caps(0, 0, slot=2)


def test_mpc_repeated_calls_reuse_zeroed_list_counters(rm):
    """A context keeps two list-counter sets; each call's lane-per-robot kernel zeroes the set
    the next call takes (no fill launch between pipelines).  Three calls in a row on one fresh
    context (so both sets are taken and handed back), with some
    robots handed down to the generic stage (a NaN reference heading: fallback law), give the
    same outputs bit for bit each time; a smaller batch after them on the same context
    matches a solve on another fresh context."""
    import torch
    x0h, xrh, urh = cfg3_inputs()
    dev = torch.device("cuda:0")
    Bs = 4096
    xrh = np.array(xrh[:Bs])
    bad = np.arange(7, Bs, 509)
    xrh[bad, 3, 2] = np.nan
    x0, xr, ur = (torch.from_numpy(np.ascontiguousarray(a[:Bs])).to(dev) for a in (x0h, xrh, urh))
    obs = torch.tensor(ompc.default_obstacles(), dtype=torch.float64, device=dev).reshape(-1, 3)
    p = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)

    def solve(slot, n):
        o = dict(u0=torch.empty(n, 2, dtype=torch.float64, device=dev),
                 u_seq=torch.empty(n, N, 2, dtype=torch.float64, device=dev),
                 status=torch.empty(n, dtype=torch.int32, device=dev),
                 iters=torch.empty(n, dtype=torch.int32, device=dev))
        rm.batch.mpc_solve_batch_dev(p, x0[:n], xr[:n], ur[:n], obs, o,
                                     step_count=torch.full((n,), 10, dtype=torch.int32, device=dev), slot=slot)
        torch.cuda.synchronize()
        return {k: v.cpu().numpy() for k, v in o.items()}

    runs = [solve(5, Bs) for _ in range(3)]
    st = runs[0]["status"]
    assert np.all(st[bad] == 2) and np.all(np.delete(st, bad) == 0)
    for r in runs[1:]:
        for k in r:
            np.testing.assert_array_equal(r[k], runs[0][k], err_msg=k)
    small = solve(5, 1000)          # a smaller batch on the same context
    fresh = solve(6, 1000)
    for k in small:
        np.testing.assert_array_equal(small[k], fresh[k], err_msg=k)
        np.testing.assert_array_equal(small[k], runs[0][k][:1000], err_msg=k)


def test_mpc_tail_grid_sizes_give_the_same_bits(rm):
    """The tail kernel's grid is sized from the list lengths its launch site saw before (a
    decaying maximum, rmpc_api.cpp tail_hint; a list longer than the 1024-round cap gets a
    workgroup per round, rmpc_mpc_group.hip) and its workgroups loop over rounds of robots, so
    the grid must not change any result.  Config 3's full batch after a 64-robot solve on the
    same fresh context (a 64-workgroup grid for ~900 rounds: ~14 rounds per workgroup) against
    the full batch on another fresh context (1024 workgroups); and LTI's full batch twice on a
    third context (the capped grid, then a workgroup per round): bit for bit."""
    import torch
    x0h, xrh, urh = cfg3_inputs()
    dev = torch.device("cuda:0")
    x0, xr, ur = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x0h, xrh, urh))
    obs = torch.tensor(ompc.default_obstacles(), dtype=torch.float64, device=dev).reshape(-1, 3)
    B = x0.shape[0]

    def solve(p, slot, n=B):
        o = dict(u0=torch.empty(n, 2, dtype=torch.float64, device=dev),
                 u_seq=torch.empty(n, N, 2, dtype=torch.float64, device=dev),
                 x_pred=torch.empty(n, N + 1, 3, dtype=torch.float64, device=dev),
                 status=torch.empty(n, dtype=torch.int32, device=dev),
                 iters=torch.empty(n, dtype=torch.int32, device=dev))
        rm.batch.mpc_solve_batch_dev(p, x0[:n], xr[:n], ur[:n], obs, o,
                                     step_count=torch.full((n,), 10, dtype=torch.int32, device=dev), slot=slot)
        torch.cuda.synchronize()
        return {k: v.cpu().numpy() for k, v in o.items()}

    ltv = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
    solve(ltv, 11, 64)
    small_grid = solve(ltv, 11)
    fresh = solve(ltv, 12)
    assert np.all(fresh["status"] == 0) and (fresh["iters"] > 7).sum() > 1000   # a long tail list
    for k in fresh:
        np.testing.assert_array_equal(small_grid[k], fresh[k], err_msg=k)
    lti = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02, ltv=False)
    first, second = solve(lti, 13), solve(lti, 13)
    assert np.all(first["status"] == 0)
    for k in first:
        np.testing.assert_array_equal(first[k], second[k], err_msg=k)


def test_tail_multi_round_loop_bounds_checked(rm, monkeypatch, capfd):
    """The lane-group tail loops its workgroups over rounds of robots on a grid sized from the
    list lengths its launch site saw (round 1's persistent form of this loop faulted; HISTORY.md
    section 10).  With the bounds-check instrumentation on (RMPC_GROUP_CHECK=2: every robot
    index, list count, retry slot and list entry checked, each wave's last site recorded in
    host-mapped memory), the multi-round shapes: config 3's full batch after a 64-robot solve
    on the same fresh context (a small grid, ~14 rounds per workgroup), and LTI's full batch
    twice (the whole batch through the tail: capped grid, then a workgroup per round).  No check
    fires, every wave reaches the kernel's exit (site 8), and every robot is optimal."""
    import re
    monkeypatch.setenv("RMPC_DIAG", "1")
    monkeypatch.setenv("RMPC_GROUP_CHECK", "2")
    x0, xr, ur = cfg3_inputs()
    obs = ompc.default_obstacles()
    ltv = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
    lti = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02, ltv=False)
    capfd.readouterr()
    outs = [rm.batch.mpc_solve_batch(ltv, x0[:64], xr[:64], ur[:64], obs, device=0, slot=14),
            rm.batch.mpc_solve_batch(ltv, x0, xr, ur, obs, device=0, slot=14),
            rm.batch.mpc_solve_batch(lti, x0, xr, ur, obs, device=0, slot=15),
            rm.batch.mpc_solve_batch(lti, x0, xr, ur, obs, device=0, slot=15)]
    err = capfd.readouterr().err
    checks = re.findall(r"\[group check\] grid (\d+): flags (-?\d+)", err)
    sites = re.findall(r"waves by last site 0\.\.9:((?: \d+)+)", err)
    assert len(checks) >= 4 and len(sites) == len(checks), err[-2000:]
    grids = [int(g) for g, _ in checks]
    assert all(int(f) == 0 for _, f in checks), checks
    for g, h in zip(grids, sites):
        hist = [int(v) for v in h.split()]
        assert hist[8] == g and sum(hist) == g, (g, hist)
    assert grids[1] < 128            # config 3's ~900 tail rounds on the 64-robot call's small grid
    for o in outs:
        assert np.all(o["status"] == 0)


@pytest.mark.parametrize("cold", [0, 1])
def test_stage_passes_give_the_one_pass_bits(rm, cold):
    """rmpc_ctx_set_stage_passes: the lane-per-robot stage in two or three passes, each later
    pass continuing only the uncertified robots from their records (active sets, iteration count
    and cycle history; a robot whose sets cycle goes straight to the tail) -- the same iterate
    path as one pass, so every output of config 3's full batch is bitwise the one-pass output,
    at the in-flight caps (9, 3), with empty and with zero-correction first sets; and config 4's
    fp32 request (paired lanes, fp64 refinement) at 8192 robots the same way."""
    import torch
    from rmpc import workloads as W
    dev = torch.device("cuda:0")

    def run(p, x0h, xrh, urh, obs_list, caps, passes, slot):
        x0, xr, ur = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x0h, xrh, urh))
        obs = torch.tensor(obs_list, dtype=torch.float64, device=dev).reshape(-1, 3)
        B, n = x0.shape[0], xrh.shape[1] - 1
        o = dict(u0=torch.empty(B, 2, dtype=torch.float64, device=dev),
                 u_seq=torch.empty(B, n, 2, dtype=torch.float64, device=dev),
                 x_pred=torch.empty(B, n + 1, 3, dtype=torch.float64, device=dev),
                 cost=torch.empty(B, dtype=torch.float64, device=dev),
                 status=torch.empty(B, dtype=torch.int32, device=dev),
                 slack_used=torch.empty(B, dtype=torch.uint8, device=dev),
                 iters=torch.empty(B, dtype=torch.int32, device=dev))
        rm.batch.configure(dict(caps=caps, cold_start=cold, passes=passes, side=True), slot=slot)
        rm.batch.mpc_solve_batch_dev(p, x0, xr, ur, obs, o, step_count=torch.full((B,), 10, dtype=torch.int32,
                                                                                 device=dev), slot=slot)
        torch.cuda.synchronize()
        return {k: v.cpu().numpy() for k, v in o.items()}

    x0, xr, ur = cfg3_inputs()
    p = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
    one = run(p, x0, xr, ur, ompc.default_obstacles(), (9, 3), (0, 0), 16)
    assert np.all(one["status"] == 0) and (one["iters"] > 9).sum() > 500
    for passes in ((1, 0), (1, 3), (2, 5)):
        got = run(p, x0, xr, ur, ompc.default_obstacles(), (9, 3), passes, 17)
        for k in one:
            np.testing.assert_array_equal(got[k], one[k], err_msg=f"{passes} {k}")
    B4, N4 = 8192, 30
    idx = np.arange(B4)
    xr4, ur4 = rm.batch.figure8_batch(W.t0_at(idx, B4), N4 + 1)
    x04 = xr4[:, 0] + W.noise_at(idx, W.CONFIGS["cfg4"]["seed"])
    p4 = rm._native.mpc_params(N4, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02, precision=1)
    one = run(p4, x04, xr4, ur4, W.UNION8_OBS, (14, 6), (0, 0), 16)
    assert np.all(one["status"] == 0)
    got = run(p4, x04, xr4, ur4, W.UNION8_OBS, (14, 6), (2, 6), 17)
    for k in one:
        np.testing.assert_array_equal(got[k], one[k], err_msg=f"cfg4 {k}")


def test_stage_passes_in_hybrid_step_and_rollouts(rm):
    """Stage-1 passes inside the other pipelines give the one-pass bits: the hybrid step's MPC
    branch (a device index list from the switch) at config 5's full size, and device closed
    loops -- an MPC rollout with the warm start across calls on (the first pass reads the warm
    sets, a continued robot its record), and a hybrid rollout."""
    import torch
    from rmpc import workloads as W
    x0h, xrh, urh = cfg5_inputs()
    B = len(x0h)
    dev = torch.device("cuda:0")
    x0, xr, ur = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x0h, xrh, urh))
    obs = torch.tensor(W.DEFAULT_OBS, dtype=torch.float64, device=dev)
    rp = rm._native.risk_params()
    lp = rm._native.lqr_params([15, 15, 8], [.1, .1], 0.02, 2.0, 3.0)
    mp = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
    res = []
    for slot, passes in ((19, (0, 0)), (20, (1, 0)), (21, (1, 3))):
        rm.batch.configure(dict(caps=(0, 0), cold_start=0, passes=passes, side=True), slot=slot)
        st = dict(prev_ctrl=torch.full((B,), -1, dtype=torch.int32, device=dev),
                  steps_since=torch.zeros(B, dtype=torch.int32, device=dev),
                  step_count=torch.full((B,), 10, dtype=torch.int32, device=dev),
                  cache=torch.zeros(B * rm._native.LQR_CACHE_DTYPE.itemsize, dtype=torch.uint8, device=dev))
        out = (torch.empty(B, 2, dtype=torch.float64, device=dev), torch.empty(B, dtype=torch.uint8, device=dev),
               torch.empty(B, dtype=torch.float64, device=dev))
        rm.batch.hybrid_step_batch_dev(rp, lp, mp, x0, xr, ur, obs, st, *out, slot=slot)
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in out] + [st["step_count"].cpu().numpy()])
    for r in res[1:]:
        for a, b in zip(r, res[0]):
            np.testing.assert_array_equal(a, b)
    start = (np.arange(2048) * 7) % 900
    for mode in ("mpc", "hybrid"):
        ro = []
        for slot, passes in ((19, (0, 0)), (20, (1, 0))):
            rm.batch.configure(dict(caps=(0, 0), cold_start=0, passes=passes, side=True), slot=slot)
            rm.batch.set_warm_start(True, slot=slot)
            kw = dict(lparams=lp, rparams=rp) if mode == "hybrid" else {}
            ro.append(rm.batch.rollout_batch(mode, 40, mparams=mp, start_index=start, obstacles=W.DEFAULT_OBS,
                                             mpc_rate=1, slot=slot, **kw))
            rm.batch.set_warm_start(False, slot=slot)
        assert ro[0]["mpc_status"][0] > 0 and ro[0]["mpc_status"][2] == 0
        for k in ("states", "controls", "used_mpc", "mpc_status"):
            np.testing.assert_array_equal(ro[1][k], ro[0][k], err_msg=f"{mode} {k}")


def test_stage_passes_edge_cases(rm):
    """Stage passes at the edges, bitwise against one pass: a partial wave (100 robots) with
    non-finite references (fallback law), LTI `solve()` (4096 robots), and an fp32 request at
    N = 20 (fp32 passes, fp64 refinement; 4096 robots)."""
    x0, xr, ur = cfg3_inputs()
    obs = ompc.default_obstacles()
    xb = np.array(xr[:100])
    xb[[3, 50, 97], 4, 2] = np.nan
    ltv = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
    lti = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02, ltv=False)
    f32 = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02, precision=1)
    cases = [("partial wave + NaN", ltv, x0[:100], xb, ur[:100], (1, 0)),
             ("LTI", lti, x0[:4096], xr[:4096], ur[:4096], (1, 3)),
             ("fp32 N=20", f32, x0[:4096], xr[:4096], ur[:4096], (2, 0))]
    for tag, p, a, b, c, passes in cases:
        outs = []
        for slot, ps in ((22, (0, 0)), (23, passes)):
            rm.batch.configure(dict(caps=(0, 0), cold_start=0, passes=ps, side=True), slot=slot)
            outs.append(rm.batch.mpc_solve_batch(p, a, b, c, obs, step_count=np.full(len(a), 10, np.int32),
                                                 slot=slot))
        for k in outs[0]:
            np.testing.assert_array_equal(outs[1][k], outs[0][k], err_msg=f"{tag} {k}")
        if tag.startswith("partial"):
            assert np.all(outs[0]["status"][[3, 50, 97]] == 2) and (outs[0]["status"] == 0).sum() == 97
        else:
            assert np.all(outs[0]["status"] == 0)
