"""Batched entry points (numpy in / numpy out) over the librmpc.so C-ABI.

Each function computes on the HIP device through one C-ABI call; host arrays are staged
by the library.  ``*_dev`` variants take torch device tensors and a stream, and return
without synchronising (for benchmarks / on-device rollouts).
"""
import ctypes as C

import numpy as np

from . import _native as nat
from ._native import check, f64, ptr


def _obs(obstacles):
    if obstacles is None:
        return np.zeros((0, 3))
    o = np.asarray(obstacles, dtype=np.float64).reshape(-1, 3)
    if o.shape[0] > nat.MAX_OBSTACLES:
        raise ValueError(f"at most {nat.MAX_OBSTACLES} obstacles")
    return np.ascontiguousarray(o)


def mpc_solve_batch(params, x0, x_refs, u_refs, obstacles=None, step_count=None, device=0,
                    want_seq=True, slot=0, ctx=None):
    """MPCController.solve_with_ltv / solve for B robots (mpc_controller.py:150-522).

    x0 [B,3]; x_refs [B,R,3]; u_refs [B,U,2]; obstacles [n_obs,3]; step_count [B] int32
    (updated in place, LTV).  Returns dict u0, u_seq, x_pred, cost, status, slack_used, iters.
    ctx: a context of the caller's own (nat.own_context) instead of the shared (device, slot) one.
    """
    lib = nat.load()
    x0 = f64(x0)
    x_refs = f64(x_refs)
    u_refs = f64(u_refs)
    B = x0.shape[0]
    if x0.shape != (B, 3) or x_refs.ndim != 3 or x_refs.shape[0] != B or x_refs.shape[2] != 3 \
            or u_refs.ndim != 3 or u_refs.shape[0] != B or u_refs.shape[2] != 2:
        raise ValueError("shapes: x0 [B,3], x_refs [B,R,3], u_refs [B,U,2]")
    obs = _obs(obstacles)
    N = params.horizon
    out = dict(u0=np.empty((B, 2)), status=np.empty(B, np.int32), cost=np.empty(B),
               slack_used=np.empty(B, np.uint8), iters=np.empty(B, np.int32),
               u_seq=np.empty((B, N, 2)) if want_seq else None,
               x_pred=np.empty((B, N + 1, 3)) if want_seq else None)
    if step_count is not None:
        if not (isinstance(step_count, np.ndarray) and step_count.dtype == np.int32
                and step_count.shape == (B,) and step_count.flags.c_contiguous):
            raise ValueError("step_count must be a C-contiguous int32 array of shape [B]")
    if ctx is None:
        ctx = nat.context(device, slot)
    check(lib.rmpc_mpc_solve_batch(ctx, C.byref(params), B, ptr(x0), ptr(x_refs), x_refs.shape[1],
                                   ptr(u_refs), u_refs.shape[1], ptr(obs), obs.shape[0],
                                   ptr(step_count), ptr(out["u0"]), ptr(out["u_seq"]),
                                   ptr(out["x_pred"]), ptr(out["cost"]), ptr(out["status"]),
                                   ptr(out["slack_used"]), ptr(out["iters"])),
          "rmpc_mpc_solve_batch")
    return out


def mpc_solve_batch_dev(params, x0, x_refs, u_refs, obstacles, out, step_count=None, device=0,
                        stream=None, slot=0):
    """Device-pointer variant: all arguments torch tensors on `device` (float64/int32/uint8).

    out: dict with u0 [B,2] and status [B] (required); u_seq, x_pred, cost, slack_used,
    iters optional.  Asynchronous on `stream` (a torch.cuda.Stream or raw handle).  `slot`
    selects the device context (nat.context): batches in flight on different streams at once
    need one slot each.
    """
    lib = nat.load()
    B = x0.shape[0]
    s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    check(lib.rmpc_mpc_solve_batch_dev(
        nat.context(device, slot), C.byref(params), B, ptr(x0), ptr(x_refs), x_refs.shape[1],
        ptr(u_refs), u_refs.shape[1], ptr(obstacles), 0 if obstacles is None else obstacles.shape[0],
        ptr(step_count), ptr(out["u0"]), ptr(out.get("u_seq")), ptr(out.get("x_pred")),
        ptr(out.get("cost")), ptr(out["status"]), ptr(out.get("slack_used")), ptr(out.get("iters")),
        s), "rmpc_mpc_solve_batch_dev")


def lqr_control_batch(params, x, x_ref, u_ref, cache=None, device=0, want_K=False,
                      want_P=False):
    """LQRController.compute_control_at_operating_point for B robots (lqr_controller.py:191-215).

    cache: structured array of LQR_CACHE_DTYPE [B] (updated in place) or None.
    Returns (u [B,2], err [B,3], K [B,2,3] | None, P [B,3,3] | None, status [B]).
    """
    lib = nat.load()
    x, x_ref, u_ref = f64(x), f64(x_ref), f64(u_ref)
    B = x.shape[0]
    if x.shape != (B, 3) or x_ref.shape != (B, 3) or u_ref.shape != (B, 2):
        raise ValueError("shapes: x [B,3], x_ref [B,3], u_ref [B,2]")
    if cache is not None and (cache.dtype != nat.LQR_CACHE_DTYPE or cache.shape != (B,)):
        raise ValueError("cache must be np.zeros(B, LQR_CACHE_DTYPE)")
    u = np.empty((B, 2))
    e = np.empty((B, 3))
    K = np.empty((B, 2, 3)) if want_K else None
    P = np.full((B, 3, 3), np.nan) if want_P else None
    st = np.empty(B, np.int32)
    check(lib.rmpc_lqr_control_batch(nat.context(device), C.byref(params), B, ptr(x), ptr(x_ref),
                                     ptr(u_ref), ptr(cache), ptr(u), ptr(e), ptr(K), ptr(P),
                                     ptr(st)), "rmpc_lqr_control_batch")
    return u, e, K, P, st


def lqr_control_batch_dev(params, x, x_ref, u_ref, u_out, cache=None, err_out=None, K_out=None,
                          status=None, device=0, stream=None, slot=0):
    lib = nat.load()
    s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    check(lib.rmpc_lqr_control_batch_dev(nat.context(device, slot), C.byref(params), x.shape[0], ptr(x),
                                         ptr(x_ref), ptr(u_ref), ptr(cache), ptr(u_out),
                                         ptr(err_out), ptr(K_out), None, ptr(status), s),
          "rmpc_lqr_control_batch_dev")


def lqr_gain_batch(params, v_r, theta_r, guard=True, device=0):
    """compute_gain(force_recompute=True) (guard) / get_lqr_gain (no guard) for B points."""
    lib = nat.load()
    v_r = f64(v_r).reshape(-1)
    theta_r = f64(theta_r).reshape(-1)
    B = v_r.shape[0]
    K = np.empty((B, 2, 3))
    P = np.empty((B, 3, 3))
    st = np.empty(B, np.int32)
    check(lib.rmpc_lqr_gain_batch(nat.context(device), C.byref(params), B, ptr(v_r), ptr(theta_r),
                                  int(bool(guard)), ptr(K), ptr(P), ptr(st)), "rmpc_lqr_gain_batch")
    return K, P, st


def risk_batch(params, x, obstacles, pred=None, device=0):
    """RiskMetrics.assess_risk for B robots -> (out [B,5], use_mpc [B] bool, level [B])."""
    lib = nat.load()
    x = f64(x)
    B = x.shape[0]
    obs = _obs(obstacles)
    n_pred = 0
    if pred is not None:
        pred = f64(pred)
        if pred.ndim != 3 or pred.shape[0] != B or pred.shape[2] < 2:
            raise ValueError("pred must be [B, n, 3]")
        if pred.shape[2] == 2:
            pred = np.ascontiguousarray(np.concatenate([pred, np.zeros(pred.shape[:2] + (1,))], -1))
        n_pred = pred.shape[1]
    out = np.empty((B, 5))
    use = np.empty(B, np.uint8)
    lvl = np.empty(B, np.int32)
    check(lib.rmpc_risk_batch(nat.context(device), C.byref(params), B, ptr(x), ptr(pred), n_pred,
                              ptr(obs), obs.shape[0], ptr(out), ptr(use), ptr(lvl)),
          "rmpc_risk_batch")
    return out, use.astype(bool), lvl


def hybrid_step_batch(rparams, lparams, mparams, x, x_refs, u_refs, obstacles, state, device=0):
    """One run_hybrid_simulation switching step for B robots (run_simulation.py:525-559).

    state: dict of per-robot arrays prev_ctrl [B] i32 (-1 none), steps_since [B] i32,
    step_count [B] i32, cache [B] LQR_CACHE_DTYPE -- updated in place.
    Returns (u [B,2], used_mpc [B] bool, combined_risk [B]).
    """
    lib = nat.load()
    x, x_refs, u_refs = f64(x), f64(x_refs), f64(u_refs)
    B = x.shape[0]
    obs = _obs(obstacles)
    u = np.empty((B, 2))
    used = np.empty(B, np.uint8)
    risk = np.empty(B)
    check(lib.rmpc_hybrid_step_batch(nat.context(device), C.byref(rparams), C.byref(lparams),
                                     C.byref(mparams), B, ptr(x), ptr(x_refs), x_refs.shape[1],
                                     ptr(u_refs), u_refs.shape[1], ptr(obs), obs.shape[0],
                                     ptr(state["prev_ctrl"]), ptr(state["steps_since"]),
                                     ptr(state["step_count"]), ptr(state["cache"]), ptr(u),
                                     ptr(used), ptr(risk)), "rmpc_hybrid_step_batch")
    return u, used.astype(bool), risk


def hybrid_step_batch_dev(rparams, lparams, mparams, x, x_refs, u_refs, obstacles, state, u_out,
                          used_out, risk_out, device=0, stream=None, slot=0):
    """Device-tensor variant of hybrid_step_batch (torch tensors on cuda:device; state holds
    device tensors prev_ctrl, steps_since, step_count (int32) and cache (uint8 bytes of
    LQR_CACHE_DTYPE records)); asynchronous on `stream`."""
    lib = nat.load()
    s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    check(lib.rmpc_hybrid_step_batch_dev(nat.context(device, slot), C.byref(rparams), C.byref(lparams),
                                         C.byref(mparams), x.shape[0], ptr(x), ptr(x_refs),
                                         x_refs.shape[1], ptr(u_refs), u_refs.shape[1],
                                         ptr(obstacles), obstacles.shape[0],
                                         ptr(state["prev_ctrl"]), ptr(state["steps_since"]),
                                         ptr(state["step_count"]), ptr(state["cache"]),
                                         ptr(u_out), ptr(used_out), ptr(risk_out), s),
          "rmpc_hybrid_step_batch_dev")


def new_hybrid_state(B):
    return dict(prev_ctrl=np.full(B, -1, np.int32), steps_since=np.zeros(B, np.int32),
                step_count=np.zeros(B, np.int32), cache=np.zeros(B, nat.LQR_CACHE_DTYPE))


def plant_step_batch(x, u, dt, v_max, omega_max, method="euler", device=0):
    """DifferentialDriveRobot.simulate_step for B robots (differential_drive.py:138-172)."""
    lib = nat.load()
    x, u = f64(x), f64(u)
    B = x.shape[0]
    xn = np.empty((B, 3))
    m = {"euler": 0, "rk4": 1}[method]
    check(lib.rmpc_plant_step_batch(nat.context(device), B, ptr(x), ptr(u), dt, v_max, omega_max, m,
                                    ptr(xn)), "rmpc_plant_step_batch")
    return xn


def figure8_batch(t0, rows, A=2.0, a=0.5, dt=0.02, device=0):
    """Figure-8 reference segments at t0[b] + i*dt (reference_generator.py:86-172)."""
    lib = nat.load()
    t0 = f64(t0).reshape(-1)
    B = t0.shape[0]
    xr = np.empty((B, rows, 3))
    ur = np.empty((B, rows, 2))
    check(lib.rmpc_figure8_batch(nat.context(device), B, ptr(t0), int(rows), A, a, dt, ptr(xr),
                                 ptr(ur)), "rmpc_figure8_batch")
    return xr, ur


def set_stage_timing(on=True, device=0):
    """Diagnostics: record per-stage device time of each MPC launch on `device`."""
    lib = nat.load()
    check(lib.rmpc_ctx_set_timing(nat.context(device), int(bool(on))), "rmpc_ctx_set_timing")


def set_stage_caps(fast_cap=0, tail_cap=0, device=0, slot=0):
    """MPC pipeline stage caps of one context (rmpc_ctx_set_stage_caps; 0 = library default):
    PDAS solves in the lane-per-robot stage, then in the lane-group tail.  Same optimum either
    way; a longer first stage suits several batches in flight (HISTORY.md section 1)."""
    lib = nat.load()
    check(lib.rmpc_ctx_set_stage_caps(nat.context(device, slot), int(fast_cap), int(tail_cap)),
          "rmpc_ctx_set_stage_caps")


def set_stage_passes(first_cap=0, second_cap=0, device=0, slot=0):
    """Passes of the lane-per-robot stage on one context (rmpc_ctx_set_stage_passes): the first
    pass runs every robot for `first_cap` PDAS solves, the next ones continue only the
    uncertified robots in compacted waves.  Same optimum and iterate path; (0, 0) = one pass."""
    lib = nat.load()
    check(lib.rmpc_ctx_set_stage_passes(nat.context(device, slot), int(first_cap), int(second_cap)),
          "rmpc_ctx_set_stage_passes")


def set_lanes_per_robot(lanes=0, device=0, slot=0):
    """Lanes per robot in the lane-per-robot stage (rmpc_ctx_set_lanes_per_robot): 0 the
    library's choice (paired lanes for the fp32 N = 30, 8-obstacle stage), 1 one lane per robot,
    2 paired.  Same optimum."""
    lib = nat.load()
    check(lib.rmpc_ctx_set_lanes_per_robot(nat.context(device, slot), int(lanes)), "rmpc_ctx_set_lanes_per_robot")


def configure(settings, device=0, slot=0):
    """All performance settings of one context at once: `settings` a dict with caps (fast,
    tail), cold_start, passes (first, second), lanes (per robot) and side
    (rmpc.workloads.INFLIGHT / ALONE)."""
    set_stage_caps(*settings["caps"], device=device, slot=slot)
    set_cold_start(settings["cold_start"], device=device, slot=slot)
    set_stage_passes(*settings["passes"], device=device, slot=slot)
    set_lanes_per_robot(settings.get("lanes", 0), device=device, slot=slot)
    set_side_stream(settings["side"], device=device, slot=slot)


def set_side_stream(on=True, device=0, slot=0):
    """Side stream of one context (rmpc_ctx_set_side_stream): the refinement of fp32 requests
    and the hybrid step's LQR branch beside the main branch (on, the default) or in order."""
    lib = nat.load()
    check(lib.rmpc_ctx_set_side_stream(nat.context(device, slot), int(bool(on))), "rmpc_ctx_set_side_stream")


def set_cold_start(mode=0, device=0, slot=0):
    """First active sets of a cold solve on one context (rmpc_ctx_set_cold_start): 0 (default)
    empty, 1 the hinge rows the start error's free response violates.  Same optimum; mode 1
    pays with batches in flight and costs one batch alone."""
    lib = nat.load()
    check(lib.rmpc_ctx_set_cold_start(nat.context(device, slot), int(mode)), "rmpc_ctx_set_cold_start")


def set_warm_start(on=True, device=0, slot=0):
    """Warm start across calls on one context (rmpc_ctx_set_warm_start): each whole-batch MPC
    solve starts robot b's active-set iteration from robot b's previous certified sets, shifted
    by one step -- the counterpart of the reference's warm_start=True solves with
    get_warm_start's shift (mpc_controller.py:272-277, 470-475, 524-538).  Same optimum; fewer
    iterations in a closed loop.  Off by default."""
    lib = nat.load()
    check(lib.rmpc_ctx_set_warm_start(nat.context(device, slot), int(bool(on))), "rmpc_ctx_set_warm_start")


def mpc_stage_times(device=0):
    """Device ms of the last MPC launch: (lane-per-robot, wave-per-robot tail, generic)."""
    lib = nat.load()
    out = (C.c_double * 3)()
    check(lib.rmpc_mpc_stage_times(nat.context(device), out), "rmpc_mpc_stage_times")
    return tuple(out)


ROLLOUT_MODES = {"lqr": 0, "mpc": 1, "hybrid": 2}


def rollout_batch(mode, steps, lparams=None, mparams=None, rparams=None, start_index=None, x0=None,
                  obstacles=None, table_len=1000, mpc_rate=5, dt=0.02, A=2.0, a=0.5, v_max=2.0,
                  omega_max=3.0, plant="euler", B=None, device=0, slot=0):
    """Closed-loop rollouts of run_simulation.py --mode lqr|mpc|hybrid for B robots, entirely on
    the device (references, control, plant).  Robot b starts at table row start_index[b] from
    x0[b] (default: the reference there).  Returns dict states [B,steps+1,3], controls
    [B,steps,2], used_mpc [B,steps] (bool), mpc_status [4] (counts over all MPC solves)."""
    lib = nat.load()
    if start_index is not None:
        start_index = np.ascontiguousarray(start_index, np.int32).reshape(-1)
        B = start_index.shape[0]
    if x0 is not None:
        x0 = f64(x0).reshape(-1, 3)
        B = x0.shape[0]
    if B is None:
        raise ValueError("B, start_index or x0 is required")
    rp = nat.RolloutParams()
    rp.mode, rp.steps, rp.table_len = ROLLOUT_MODES[mode], int(steps), int(table_len)
    rp.mpc_rate, rp.plant_method = int(mpc_rate), {"euler": 0, "rk4": 1}[plant]
    rp.dt, rp.A, rp.a, rp.v_max, rp.omega_max = dt, A, a, v_max, omega_max
    obs = _obs(obstacles)
    states = np.empty((B, steps + 1, 3))
    controls = np.empty((B, steps, 2))
    used = np.zeros((B, steps), np.uint8)
    counts = np.zeros(4, np.int64)
    ref = lambda p: C.byref(p) if p is not None else None  # noqa: E731
    check(lib.rmpc_rollout_batch(nat.context(device, slot), C.byref(rp), ref(lparams), ref(mparams),
                                 ref(rparams), B, ptr(start_index), ptr(x0), ptr(obs), obs.shape[0],
                                 ptr(states), ptr(controls), ptr(used), ptr(counts)),
          "rmpc_rollout_batch")
    return dict(states=states, controls=controls, used_mpc=used.astype(bool), mpc_status=counts)
