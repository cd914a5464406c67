"""LQRController -- drop-in for hybrid_controller.controllers.lqr_controller (lqr_controller.py).

Same constructor, attributes (K, P, _last_v_r, _last_theta_r), cache rule, fallback gain
and clipping as lqr_controller.py:33-283.  The DARE + gain + control law run on the
MI355X (librmpc.so: SDA doubling instead of SciPy's QZ).  ``compute_control_batch``
serves B robots, each with its own gain cache.
"""
from typing import Optional, Tuple

import numpy as np

from . import _native as nat
from .batch import lqr_control_batch, lqr_gain_batch


class LQRController:
    def __init__(self, Q_diag: list = None, R_diag: list = None, dt: float = 0.02,
                 v_max: float = 1.0, omega_max: float = 1.5, device: int = 0):
        if Q_diag is None:
            Q_diag = [10.0, 10.0, 1.0]
        if R_diag is None:
            R_diag = [0.1, 0.1]
        self.Q = np.diag(Q_diag)
        self.R = np.diag(R_diag)
        self.dt = dt
        self.v_max = v_max
        self.omega_max = omega_max
        self.device = device
        self.K: Optional[np.ndarray] = None
        self.P: Optional[np.ndarray] = None
        self._last_v_r: float = 0.0
        self._last_theta_r: float = 0.0

    def _params(self, dt=None, use_cache=True):
        return nat.lqr_params(np.diag(self.Q), np.diag(self.R), self.dt if dt is None else dt,
                              self.v_max, self.omega_max, use_cache=use_cache)

    def _cache(self):
        c = np.zeros(1, nat.LQR_CACHE_DTYPE)
        if self.K is not None:
            c["K"][0] = np.asarray(self.K, dtype=np.float64).reshape(6)
            c["last_v"][0] = self._last_v_r
            c["last_theta"][0] = self._last_theta_r
            c["valid"][0] = 1
        return c

    def compute_gain(self, v_r: float, theta_r: float, force_recompute: bool = False) -> np.ndarray:
        """lqr_controller.py:92-147."""
        if not force_recompute and self.K is not None:
            if abs(v_r - self._last_v_r) < 1e-6 and abs(theta_r - self._last_theta_r) < 1e-6:
                return self.K
        K, P, st = lqr_gain_batch(self._params(), [v_r], [theta_r], guard=True, device=self.device)
        self.K = K[0]
        if st[0] == nat.RMPC_OPTIMAL:
            self.P = P[0]
        else:
            print("Warning: DARE solver failed, using fallback gain. Error: no stabilising solution")
        self._last_v_r = v_r
        self._last_theta_r = theta_r
        return self.K

    def compute_control(self, x: np.ndarray, x_ref: np.ndarray, u_ref: np.ndarray,
                        K: np.ndarray = None) -> np.ndarray:
        """lqr_controller.py:149-189 -- the law runs in the device kernel; an explicit K is
        passed through the kernel's gain-cache slot keyed to this operating point."""
        if K is None:
            if self.K is None:
                self.compute_gain(u_ref[0], x_ref[2])
            K = self.K
        c = np.zeros(1, nat.LQR_CACHE_DTYPE)
        c["K"][0] = np.asarray(K, dtype=np.float64).reshape(6)
        c["last_v"][0] = float(u_ref[0])
        c["last_theta"][0] = float(x_ref[2])
        c["valid"][0] = 1
        u, _, _, _, _ = lqr_control_batch(self._params(), np.asarray(x, np.float64)[None],
                                          np.asarray(x_ref, np.float64)[None],
                                          np.asarray(u_ref, np.float64)[None], cache=c,
                                          device=self.device)
        return u[0]

    def compute_control_at_operating_point(self, x: np.ndarray, x_ref: np.ndarray,
                                           u_ref: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """lqr_controller.py:191-215: gain (cached) + control in one kernel launch."""
        c = self._cache()
        u, e, K, P, st = lqr_control_batch(self._params(), np.asarray(x, np.float64)[None],
                                           np.asarray(x_ref, np.float64)[None],
                                           np.asarray(u_ref, np.float64)[None], cache=c,
                                           device=self.device, want_K=True, want_P=True)
        self.K = K[0]
        if not np.isnan(P[0]).any():
            self.P = P[0]
        if st[0] == nat.RMPC_DARE_FALLBACK:
            print("Warning: DARE solver failed, using fallback gain. Error: no stabilising solution")
        self._last_v_r = float(c["last_v"][0])
        self._last_theta_r = float(c["last_theta"][0])
        return u[0], e[0]

    def compute_control_batch(self, x, x_ref, u_ref, cache=None):
        """B robots; cache = np.zeros(B, LQR_CACHE_DTYPE) per-robot gain caches (in place)."""
        u, e, _, _, st = lqr_control_batch(self._params(), x, x_ref, u_ref, cache=cache,
                                           device=self.device)
        return u, e, st

    def get_lqr_gain(self, v_r: float, theta_r: float, dt: float = None) -> np.ndarray:
        """lqr_controller.py:217-242 (no v_r guard; raises like scipy when the DARE fails)."""
        use_dt = dt if (dt is not None and abs(dt - self.dt) > 1e-9) else None
        K, _, st = lqr_gain_batch(self._params(use_dt), [v_r], [theta_r], guard=False,
                                  device=self.device)
        if st[0] != nat.RMPC_OPTIMAL:
            raise np.linalg.LinAlgError("DARE has no stabilising solution at this operating point")
        return K[0]

    def _normalize_angle(self, angle: float) -> float:
        while angle > np.pi:
            angle -= 2 * np.pi
        while angle < -np.pi:
            angle += 2 * np.pi
        return angle

    def _clip_control(self, u: np.ndarray) -> np.ndarray:
        return np.array([np.clip(u[0], -self.v_max, self.v_max),
                         np.clip(u[1], -self.omega_max, self.omega_max)])

    def get_cost_matrices(self) -> Tuple[np.ndarray, np.ndarray]:
        return self.Q.copy(), self.R.copy()

    def set_weights(self, Q_diag: list = None, R_diag: list = None) -> None:
        if Q_diag is not None:
            self.Q = np.diag(Q_diag)
        if R_diag is not None:
            self.R = np.diag(R_diag)
        self.K = None
        self.P = None

    @property
    def gain_computed(self) -> bool:
        return self.K is not None
