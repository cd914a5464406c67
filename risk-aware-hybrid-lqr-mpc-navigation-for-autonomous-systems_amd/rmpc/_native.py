"""ctypes binding of librmpc.so (include/rmpc.h) -- the only way this package computes.

There is no CPU fallback: if the library is missing, or no HIP device is visible, every
entry point raises.  The library is built in-tree by ``__graft_entry__.build()``
(``make -C risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd``).
"""
import ctypes as C
import os
import weakref
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RMPC_LIB_PATH: load an alternative build of the library (A/B diagnostics only)
LIB_PATH = os.environ.get("RMPC_LIB_PATH") or os.path.join(_HERE, "librmpc.so")

RMPC_OK = 0
RMPC_OPTIMAL, RMPC_OPTIMAL_INACCURATE, RMPC_FALLBACK, RMPC_DARE_FALLBACK = 0, 1, 2, 3
RMPC_LTV, RMPC_LTI = 0, 1
RMPC_F64, RMPC_F32 = 0, 1
MAX_HORIZON = 64
MAX_OBSTACLES = 16


class RmpcError(RuntimeError):
    pass


class MpcParams(C.Structure):
    _fields_ = [("horizon", C.c_int32), ("block_size", C.c_int32), ("formulation", C.c_int32),
                ("soft", C.c_int32), ("precision", C.c_int32), ("max_iter", C.c_int32),
                ("ramp_up_steps", C.c_int32), ("_pad0", C.c_int32), ("Q", C.c_double * 3),
                ("R", C.c_double * 2), ("P", C.c_double * 3), ("d_safe", C.c_double),
                ("slack_penalty", C.c_double), ("v_max", C.c_double),
                ("omega_max", C.c_double), ("dt", C.c_double)]


class LqrParams(C.Structure):
    _fields_ = [("Q", C.c_double * 3), ("R", C.c_double * 2), ("dt", C.c_double),
                ("v_max", C.c_double), ("omega_max", C.c_double), ("max_iter", C.c_int32),
                ("use_cache", C.c_int32)]


class RiskParams(C.Structure):
    _fields_ = [("d_safe", C.c_double), ("d_trigger", C.c_double), ("alpha", C.c_double),
                ("beta", C.c_double), ("threshold_low", C.c_double),
                ("threshold_medium", C.c_double), ("threshold_high", C.c_double),
                ("min_dwell_steps", C.c_int32), ("use_predicted", C.c_int32)]


class RolloutParams(C.Structure):
    _fields_ = [("mode", C.c_int32), ("steps", C.c_int32), ("table_len", C.c_int32),
                ("mpc_rate", C.c_int32), ("plant_method", C.c_int32), ("_pad0", C.c_int32),
                ("dt", C.c_double), ("A", C.c_double), ("a", C.c_double), ("v_max", C.c_double),
                ("omega_max", C.c_double)]


class LqrCache(C.Structure):
    _fields_ = [("K", C.c_double * 6), ("last_v", C.c_double), ("last_theta", C.c_double),
                ("valid", C.c_int32), ("_pad0", C.c_int32)]


LQR_CACHE_DTYPE = np.dtype([("K", "<f8", (6,)), ("last_v", "<f8"), ("last_theta", "<f8"),
                            ("valid", "<i4"), ("_pad0", "<i4")])

_vp = C.c_void_p
_i64 = C.c_int64
_i32 = C.c_int32
_d = C.c_double

# name -> argtypes (all return int)
_PROTOS = {
    "rmpc_abi_version": [],
    "rmpc_ctx_create": [C.c_int, C.POINTER(_vp)],
    "rmpc_ctx_create_multi": [C.POINTER(C.c_int32), _i32, C.POINTER(_vp)],
    "rmpc_ctx_device_count": [_vp, C.POINTER(C.c_int32)],
    "rmpc_ctx_destroy": [_vp],
    "rmpc_ctx_synchronize": [_vp],
    "rmpc_device_count": [C.POINTER(C.c_int)],
    "rmpc_ctx_set_timing": [_vp, _i32],
    "rmpc_ctx_set_stage_caps": [_vp, _i32, _i32],
    "rmpc_ctx_set_stage_passes": [_vp, _i32, _i32],
    "rmpc_ctx_set_lanes_per_robot": [_vp, _i32],
    "rmpc_ctx_set_side_stream": [_vp, _i32],
    "rmpc_ctx_set_cold_start": [_vp, _i32],
    "rmpc_ctx_set_warm_start": [_vp, _i32],
    "rmpc_mpc_stage_times": [_vp, C.POINTER(C.c_double)],
    "rmpc_mpc_solve_batch": [_vp, C.POINTER(MpcParams), _i64, _vp, _vp, _i32, _vp, _i32, _vp, _i32,
                             _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "rmpc_mpc_solve_batch_dev": [_vp, C.POINTER(MpcParams), _i64, _vp, _vp, _i32, _vp, _i32, _vp,
                                 _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "rmpc_lqr_control_batch": [_vp, C.POINTER(LqrParams), _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                               _vp, _vp],
    "rmpc_lqr_control_batch_dev": [_vp, C.POINTER(LqrParams), _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp, _vp, _vp],
    "rmpc_lqr_gain_batch": [_vp, C.POINTER(LqrParams), _i64, _vp, _vp, _i32, _vp, _vp, _vp],
    "rmpc_risk_batch": [_vp, C.POINTER(RiskParams), _i64, _vp, _vp, _i32, _vp, _i32, _vp, _vp, _vp],
    "rmpc_hybrid_step_batch": [_vp, C.POINTER(RiskParams), C.POINTER(LqrParams),
                               C.POINTER(MpcParams), _i64, _vp, _vp, _i32, _vp, _i32, _vp, _i32,
                               _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "rmpc_hybrid_step_batch_dev": [_vp, C.POINTER(RiskParams), C.POINTER(LqrParams),
                                   C.POINTER(MpcParams), _i64, _vp, _vp, _i32, _vp, _i32, _vp,
                                   _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "rmpc_plant_step_batch": [_vp, _i64, _vp, _vp, _d, _d, _d, _i32, _vp],
    "rmpc_figure8_batch": [_vp, _i64, _vp, _i32, _d, _d, _d, _vp, _vp],
    "rmpc_rollout_batch": [_vp, C.POINTER(RolloutParams), C.POINTER(LqrParams), C.POINTER(MpcParams),
                           C.POINTER(RiskParams), _i64, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp],
    "rmpc_rollout_batch_dev": [_vp, C.POINTER(RolloutParams), C.POINTER(LqrParams),
                               C.POINTER(MpcParams), C.POINTER(RiskParams), _i64, _vp, _vp, _vp,
                               _i32, _vp, _vp, _vp, _vp, _vp],
}

_lib = None
_lock = threading.RLock()
_ctx = {}


def load():
    """Load librmpc.so and declare every exported prototype (no device needed)."""
    global _lib
    lib = _lib
    if lib is not None:              # (fast path: every batch call goes through here)
        return lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RmpcError(f"{LIB_PATH} not built: run __graft_entry__.build() "
                                "(make -C <package dir>); there is no CPU fallback")
            # One HIP runtime per process: PyTorch bundles its own libamdhip64.so.7 and its
            # libraries NEED it by a different file name, so if librmpc.so were loaded first
            # the process would end up with two runtimes (and torch's copy sees no device).
            # Importing torch first makes librmpc.so bind to the runtime already loaded.
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            lib = C.CDLL(LIB_PATH)
            for name, args in _PROTOS.items():
                if os.environ.get("RMPC_LIB_PATH") and not hasattr(lib, name):
                    continue        # an older A/B build (diagnostics) may lack newer entry points
                f = getattr(lib, name)
                f.argtypes = args
                f.restype = C.c_int
            lib.rmpc_last_error.argtypes = []
            lib.rmpc_last_error.restype = C.c_char_p
            _lib = lib
    return _lib


def exported_symbols():
    return list(_PROTOS) + ["rmpc_last_error"]


def check(rc, what="rmpc call"):
    if rc != RMPC_OK:
        msg = load().rmpc_last_error().decode(errors="replace")
        raise RmpcError(f"{what} failed ({rc}): {msg}")


def context(device=0, slot=0):
    """Per-process context for `device` (created on first use, lives until exit).

    `device` may be a sequence of device ids: a multi-device context
    (rmpc_ctx_create_multi) whose host-array batch calls split the robots over those devices
    -- 64-robot blocks dealt round-robin -- and gather every output back in input order.
    `slot` > 0 gives further independent contexts of the same device: each owns its own
    solver scratch, so solves on different streams can be in flight at once (one context per
    stream; a context's calls must not overlap each other)."""
    if type(device) is int and type(slot) is int:      # (fast path: an existing context)
        ctx = _ctx.get(device if not slot else (device, "slot", slot))
        if ctx is not None:
            return ctx
    lib = load()
    key = int(device) if np.ndim(device) == 0 else tuple(int(d) for d in device)
    if isinstance(key, tuple) and len(key) == 1:
        key = key[0]
    ck = key if not slot else (key, "slot", int(slot))
    with _lock:
        ctx = _ctx.get(ck)
        if ctx is None:
            h = _vp()
            if isinstance(key, tuple):
                ids = (C.c_int32 * len(key))(*key)
                check(lib.rmpc_ctx_create_multi(ids, len(key), C.byref(h)), "rmpc_ctx_create_multi")
            else:
                check(lib.rmpc_ctx_create(key, C.byref(h)), "rmpc_ctx_create")
            ctx = h
            _ctx[ck] = ctx
    return ctx


def own_context(device=0):
    """A context of its own for one caller (an MPCController instance: its warm-start sets
    belong to that controller).  Release it with release_context."""
    lib = load()
    h = _vp()
    key = int(device) if np.ndim(device) == 0 else tuple(int(d) for d in device)
    if isinstance(key, tuple) and len(key) == 1:
        key = key[0]
    if isinstance(key, tuple):                  # a device list: rmpc_ctx_create_multi, as context()
        ids = (C.c_int32 * len(key))(*key)
        check(lib.rmpc_ctx_create_multi(ids, len(key), C.byref(h)), "rmpc_ctx_create_multi")
    else:
        check(lib.rmpc_ctx_create(key, C.byref(h)), "rmpc_ctx_create")
    return h


def release_context(h):
    if h is not None and _lib is not None:
        _lib.rmpc_ctx_destroy(h)


def _release_quietly(h):
    """Finalizer form of release_context: at interpreter exit the library or the HIP runtime
    may already be torn down, and a destroy that fails there has nothing left to release."""
    try:
        release_context(h)
    except Exception:
        pass


class OwnedContext:
    """One caller's own context (own_context), destroyed exactly once: by release(), or by a
    weakref finalizer when the owner is collected (also at interpreter exit, before the
    library's own teardown).  Copies of the owning object must not share it (MPCController
    resets its owner on copy)."""

    def __init__(self, device=0):
        self.h = own_context(device)
        self._fin = weakref.finalize(self, _release_quietly, self.h)

    def release(self):
        self._fin()


def ptr(a):
    """Data pointer of a C-contiguous numpy array or torch tensor (None -> NULL)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if not a.flags.c_contiguous:
            raise ValueError("array must be C-contiguous")
        return a.ctypes.data
    return a.data_ptr()


def f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape)
    return a


def mpc_params(N, Q, R, P, d_safe, rho, v_max, omega_max, dt, block_size=1, ltv=True,
               soft=True, max_iter=64, ramp_up_steps=10, precision=RMPC_F64):
    p = MpcParams()
    p.horizon, p.block_size = int(N), int(block_size)
    p.formulation = RMPC_LTV if ltv else RMPC_LTI
    p.soft, p.precision, p.max_iter, p.ramp_up_steps = int(bool(soft)), precision, max_iter, ramp_up_steps
    p.Q[:] = [float(v) for v in Q]
    p.R[:] = [float(v) for v in R]
    p.P[:] = [float(v) for v in P]
    p.d_safe, p.slack_penalty = float(d_safe), float(rho)
    p.v_max, p.omega_max, p.dt = float(v_max), float(omega_max), float(dt)
    return p


def lqr_params(Q, R, dt, v_max, omega_max, max_iter=64, use_cache=True):
    p = LqrParams()
    p.Q[:] = [float(v) for v in Q]
    p.R[:] = [float(v) for v in R]
    p.dt, p.v_max, p.omega_max = float(dt), float(v_max), float(omega_max)
    p.max_iter, p.use_cache = max_iter, int(bool(use_cache))
    return p


def risk_params(d_safe=0.3, d_trigger=1.0, alpha=0.6, beta=0.4, threshold_low=0.2,
                threshold_medium=0.5, threshold_high=0.8, min_dwell_steps=10, use_predicted=False):
    """use_predicted: hybrid rollouts feed each robot's last MPC x_pred to the risk (off in
    the reference's loop, run_simulation.py:525-531)."""
    p = RiskParams()
    p.use_predicted = int(bool(use_predicted))
    p.d_safe, p.d_trigger, p.alpha, p.beta = d_safe, d_trigger, alpha, beta
    p.threshold_low, p.threshold_medium, p.threshold_high = (threshold_low, threshold_medium,
                                                             threshold_high)
    p.min_dwell_steps = min_dwell_steps
    return p
