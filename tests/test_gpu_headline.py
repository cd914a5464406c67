"""The headline's exact in-flight settings, pinned (review item: the bench's own settings had
no GPU test of their own).

bench.py times BASELINE configs 3, 4 and 5 with ten (config 3) or eight batches in flight, each
on its own context and stream, every context configured with rmpc.workloads.INFLIGHT[config]
(stage caps, zero-correction first sets, stage-1 passes, lanes per robot, side stream).  Here ten
slots on ten streams run
the full batch of each configuration with exactly those settings -- two rounds of launches for
the MPC configurations, so each slot's second launch overlaps the others' -- and:
  - the ten outputs are bitwise equal to a solve alone on an eleventh context with the same
    settings (the contexts share no scratch, and in-flight overlap changes no result);
  - config 3: every robot's u0, u_seq and x_pred (the outputs mpc_controller.py:497-505
    returns) against the C port at 1e-9, and every robot of hard_cfg3.npz (the tail robots
    plus a sample) against the independent exact QP at 1e-9;
  - config 4 (fp32 request): every robot against the fp64 C port, relative <= 1e-4 (north
    star), all optimal;
  - config 5 (hybrid step): the switch decision against oracle/risk.py's (the fixture), the MPC
    branch against the C port at 1e-9 and its fixture robots against the exact QP at 1e-9, the
    LQR branch against SciPy's DARE at 1e-10.
"""
import os
import sys

import numpy as np
import pytest

from oracle import cpu, mpc as ompc

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from make_hard_fixtures import cfg3_inputs, cfg5_inputs  # noqa: E402

pytestmark = pytest.mark.gpu
SLOTS = list(range(40, 50))     # ten in-flight contexts of their own (bench.py runs config 3 at 10; other tests use 0-18)
ALONE = 50


@pytest.fixture(scope="module")
def rm(gpu_lib):
    import rmpc
    return rmpc


def _mpc_inflight(rm, settings, p, x0h, xrh, urh, obs_list, step0, rounds=2):
    """Ten slots in flight (two rounds) and one solve alone, all configured with `settings`;
    returns (alone outputs, [slot outputs]) as numpy dicts."""
    import torch
    dev = torch.device("cuda:0")
    x0, xr, ur = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x0h, xrh, urh))
    obs = torch.tensor(obs_list, dtype=torch.float64, device=dev).reshape(-1, 3)
    B, N = x0.shape[0], urh.shape[1] if urh.shape[1] < xrh.shape[1] else xrh.shape[1] - 1

    def outs():
        return dict(u0=torch.empty(B, 2, dtype=torch.float64, device=dev),
                    u_seq=torch.empty(B, N, 2, dtype=torch.float64, device=dev),
                    x_pred=torch.empty(B, N + 1, 3, dtype=torch.float64, device=dev),
                    cost=torch.empty(B, dtype=torch.float64, device=dev),
                    status=torch.empty(B, dtype=torch.int32, device=dev),
                    slack_used=torch.empty(B, dtype=torch.uint8, device=dev),
                    iters=torch.empty(B, dtype=torch.int32, device=dev))
    for s in SLOTS + [ALONE]:
        rm.batch.configure(settings, slot=s)
    alone = outs()
    rm.batch.mpc_solve_batch_dev(p, x0, xr, ur, obs, alone,
                                 step_count=torch.full((B,), step0, dtype=torch.int32, device=dev), slot=ALONE)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in SLOTS]
    o = [outs() for _ in SLOTS]
    sc = [torch.full((B,), step0, dtype=torch.int32, device=dev) for _ in SLOTS]
    for _ in range(rounds):
        for i, s in enumerate(SLOTS):
            with torch.cuda.stream(streams[i]):    # ordered before the slot's solve that reads it
                sc[i].fill_(step0)
            rm.batch.mpc_solve_batch_dev(p, x0, xr, ur, obs, o[i], step_count=sc[i], stream=streams[i], slot=s)
    torch.cuda.synchronize()
    npy = lambda d: {k: v.cpu().numpy() for k, v in d.items()}     # noqa: E731
    return npy(alone), [npy(d) for d in o]


def _bitwise(alone, slots):
    for i, o in enumerate(slots):
        for k in alone:
            assert np.array_equal(o[k], alone[k], equal_nan=True), (SLOTS[i], k)


def _rel(a, b, axes):
    return np.abs(a - b).max(axis=axes) / np.maximum(1.0, np.abs(b).max(axis=axes))


def test_cfg3_headline_settings_inflight_match_cport_and_exact_qp(rm, golden, capsys):
    from rmpc import workloads as W
    st = W.inflight_settings("cfg3")
    x0, xr, ur = cfg3_inputs()
    obs = ompc.default_obstacles()
    B, N = len(x0), 20
    p = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
    alone, slots = _mpc_inflight(rm, st, p, x0, xr, ur, obs, 0)
    _bitwise(alone, slots)
    assert np.all(alone["status"] == 0)
    cp = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
    ref = cpu.mpc_solve_batch(cp, x0, xr, ur, obs, step_count=np.zeros(B, np.int32), threads=16)
    ok = ref["status"] == 0
    assert ok.mean() >= 0.999
    d = {k: float(np.abs(alone[k][ok] - ref[k][ok]).max()) for k in ("u0", "u_seq", "x_pred")}
    fx = golden("hard_cfg3.npz")
    idx, okq = fx["idx"], fx["ok"]
    dq = np.abs(alone["u_seq"][idx] - fx["u_seq"]).max(axis=(1, 2))[okq]
    with capsys.disabled():
        print(f"\n[cfg3 in flight {st}] vs C port {d}; {okq.sum()} fixture robots vs exact QP {dq.max():.2e}; "
              f"iters mean {alone['iters'].mean():.3f} max {alone['iters'].max()}")
    assert max(d.values()) <= 1e-9, d
    assert dq.max() <= 1e-9
    assert np.array_equal(alone["slack_used"][idx][okq].astype(bool), fx["slack_used"][okq])


def test_cfg4_headline_settings_inflight_match_fp64_cport(rm, capsys):
    from rmpc import workloads as W
    st = W.inflight_settings("cfg4")
    B, N = 32768, 30
    idx = np.arange(B)
    xr, ur = rm.batch.figure8_batch(W.t0_at(idx, B), N + 1)
    x0 = xr[:, 0] + W.noise_at(idx, W.CONFIGS["cfg4"]["seed"])
    obs = W.UNION8_OBS
    p = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02, precision=1)
    alone, slots = _mpc_inflight(rm, st, p, x0, xr, ur, obs, 10)
    _bitwise(alone, slots)
    cp = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
    ref = cpu.mpc_solve_batch(cp, x0, xr, ur, obs, step_count=np.full(B, 10, np.int32), threads=16)
    both = (alone["status"] == 0) & (ref["status"] == 0)
    assert both.mean() >= 0.999
    e = {k: float(_rel(alone[k], ref[k], (1,) if k == "u0" else (1, 2))[both].max()) for k in ("u0", "u_seq", "x_pred")}
    with capsys.disabled():
        print(f"\n[cfg4 in flight {st}] optimal {both.mean():.5f}; max rel vs fp64 C port {e}")
    assert max(e.values()) <= 1e-4, e


def test_cfg5_headline_settings_inflight_match_oracles(rm, golden, capsys):
    import torch
    from rmpc import workloads as W
    st = W.inflight_settings("cfg5")
    fx = golden("hard_cfg5.npz")
    x0h, xrh, urh = cfg5_inputs()
    B, N = len(x0h), 20
    dev = torch.device("cuda:0")
    x0, xr, ur = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x0h, xrh, urh))
    obs = torch.tensor(W.DEFAULT_OBS, dtype=torch.float64, device=dev)
    rp = rm._native.risk_params()
    lp = rm._native.lqr_params([15, 15, 8], [.1, .1], 0.02, 2.0, 3.0, use_cache=False)   # bench.py's
    mp = rm._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)

    def state():
        return dict(prev_ctrl=torch.full((B,), -1, dtype=torch.int32, device=dev),
                    steps_since=torch.zeros(B, dtype=torch.int32, device=dev),
                    step_count=torch.full((B,), 10, dtype=torch.int32, device=dev),
                    cache=torch.zeros(B * rm._native.LQR_CACHE_DTYPE.itemsize, dtype=torch.uint8, device=dev))

    def outs():
        return (torch.empty(B, 2, dtype=torch.float64, device=dev), torch.empty(B, dtype=torch.uint8, device=dev),
                torch.empty(B, dtype=torch.float64, device=dev))
    for s in SLOTS + [ALONE]:
        rm.batch.configure(st, slot=s)
    a_state, a_out = state(), outs()
    rm.batch.hybrid_step_batch_dev(rp, lp, mp, x0, xr, ur, obs, a_state, *a_out, slot=ALONE)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in SLOTS]
    states, o = [state() for _ in SLOTS], [outs() for _ in SLOTS]
    for i, s in enumerate(SLOTS):
        rm.batch.hybrid_step_batch_dev(rp, lp, mp, x0, xr, ur, obs, states[i], *o[i], stream=streams[i], slot=s)
    torch.cuda.synchronize()
    for i in range(len(SLOTS)):
        for t, ta in zip(o[i], a_out):
            assert torch.equal(t, ta), SLOTS[i]
        for k in a_state:
            assert torch.equal(states[i][k], a_state[k]), (SLOTS[i], k)
    u, used = a_out[0].cpu().numpy(), a_out[1].cpu().numpy().astype(bool)
    assert np.array_equal(used, fx["use_mpc"])
    im = np.where(used)[0]
    cp = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
    ref = cpu.mpc_solve_batch(cp, x0h[im], xrh[im], urh[im], W.DEFAULT_OBS, step_count=np.full(len(im), 10, np.int32),
                              threads=16)
    okc = ref["status"] == 0
    dc = np.abs(u[im] - ref["u0"]).max(axis=1)[okc]
    dq = np.abs(u[fx["idx"]] - fx["u0"]).max(axis=1)[fx["ok"]]
    dl = np.abs(u[fx["lqr_idx"]] - fx["lqr_u"]).max()
    with capsys.disabled():
        print(f"\n[cfg5 in flight {st}] MPC branch {len(im)} vs C port {dc.max():.2e}, {fx['ok'].sum()} vs exact QP "
              f"{dq.max():.2e}; LQR branch vs SciPy {dl:.2e}")
    assert okc.mean() >= 0.999 and dc.max() <= 1e-9
    assert dq.max() <= 1e-9
    assert dl <= 1e-10
