"""LQR controller -- oracle restatement (test infrastructure only).

Follows lqr_controller.py:57-283.  The DARE is solved with
``scipy.linalg.solve_discrete_are``, the reference's own arithmetic dependency
(setup.py:23 ``scipy>=1.10.0``, no lock; this image has scipy 1.15.3), exactly as
lqr_controller.py:126 calls it.
"""
import numpy as np
from scipy.linalg import solve_discrete_are

from .plant import discrete_model_explicit, normalize_angle

FALLBACK_K = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, 1.0]])   # lqr_controller.py:137-140


def dare_gain(v_r, theta_r, Q, R, dt):
    """lqr_controller.py:116-141 without the cache.  Returns (K, P, ok)."""
    A, B = discrete_model_explicit(v_r, theta_r, dt)
    if abs(v_r) < 1e-6:                                     # :120-122
        A, B = discrete_model_explicit(0.01, theta_r, dt)
    try:
        P = solve_discrete_are(A, B, Q, R)                  # :126
        K = np.linalg.solve(R + B.T @ P @ B, B.T @ P @ A)   # :130-132
        return K, P, True
    except Exception:                                      # :134-141
        return FALLBACK_K.copy(), None, False


class LQRController:
    """lqr_controller.py:33-283 (same constructor defaults and cache rule)."""

    def __init__(self, Q_diag=None, R_diag=None, dt=0.02, v_max=1.0, omega_max=1.5):
        self.Q = np.diag(Q_diag if Q_diag is not None else [10.0, 10.0, 1.0])
        self.R = np.diag(R_diag if R_diag is not None else [0.1, 0.1])
        self.dt = dt
        self.v_max = v_max
        self.omega_max = omega_max
        self.K = None
        self.P = None
        self._last_v_r = 0.0
        self._last_theta_r = 0.0

    def compute_gain(self, v_r, theta_r, force_recompute=False):
        # cache rule lqr_controller.py:112-114
        if not force_recompute and self.K is not None:
            if abs(v_r - self._last_v_r) < 1e-6 and abs(theta_r - self._last_theta_r) < 1e-6:
                return self.K
        K, P, ok = dare_gain(v_r, theta_r, self.Q, self.R, self.dt)
        self.K = K
        if ok:
            self.P = P
        self._last_v_r = v_r
        self._last_theta_r = theta_r
        return self.K

    def _clip(self, u):
        return np.array([np.clip(u[0], -self.v_max, self.v_max),
                         np.clip(u[1], -self.omega_max, self.omega_max)])

    def compute_control(self, x, x_ref, u_ref, K=None):
        """lqr_controller.py:149-189."""
        if K is None:
            if self.K is None:
                self.compute_gain(u_ref[0], x_ref[2])
            K = self.K
        e = np.asarray(x, dtype=np.float64) - x_ref
        e[2] = normalize_angle(e[2])
        return self._clip(u_ref + (-K @ e))

    def compute_control_at_operating_point(self, x, x_ref, u_ref):
        """lqr_controller.py:191-215."""
        K = self.compute_gain(u_ref[0], x_ref[2])
        e = np.asarray(x, dtype=np.float64) - x_ref
        e[2] = normalize_angle(e[2])
        return self.compute_control(x, x_ref, u_ref, K), e

    def get_lqr_gain(self, v_r, theta_r, dt=None):
        """lqr_controller.py:217-242 (no v_r guard, inv instead of solve)."""
        A, B = discrete_model_explicit(v_r, theta_r, self.dt if dt is None else dt)
        P = solve_discrete_are(A, B, self.Q, self.R)
        return np.linalg.inv(self.R + B.T @ P @ B) @ (B.T @ P @ A)
