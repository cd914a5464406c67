"""Shared LQR gain parity check (CPU port and GPU kernel vs the reference's SciPy gains)."""
import numpy as np

from oracle.plant import discrete_model_explicit


def dare_residual(P, v, t, Q, R, dt=0.02, guard=True):
    if guard and abs(v) < 1e-6:
        v = 0.01
    A, B = discrete_model_explicit(v, t, dt)
    r = A.T @ P @ A - P - A.T @ P @ B @ np.linalg.solve(R + B.T @ P @ B, B.T @ P @ A) + Q
    return np.abs(r).max() / np.abs(P).max()


def assert_gains_match(grid, K, P, K_ref, P_ref, Q, R):
    """Tolerance follows the DARE's conditioning: on the operating range (|v_r| >= 0.1)
    |dK| <= 1e-10; at the near-uncontrollable guard points (|v_r| <= 0.01, ||P|| up to
    5e5) |dK| <= 1e-7 * max(1, |K|).  In both cases our DARE residual must not exceed
    SciPy's (QZ) residual by more than 4x (or 1e-13 relative, rounding level at
    ||P|| ~ 5e4): the SDA solution is as accurate as the reference's."""
    for i, (v, t) in enumerate(grid):
        tol = 1e-10 if abs(v) >= 0.1 else 1e-7 * max(1.0, np.abs(K_ref[i]).max())
        d = np.abs(K[i] - K_ref[i]).max()
        assert d <= tol, (v, t, d, tol)
        rs = dare_residual(P[i], v, t, Q, R)
        rr = dare_residual(P_ref[i], v, t, Q, R)
        floor = 1e-13 if abs(v) >= 0.1 else 1e-12    # ||P|| up to 5e5 below v_r = 0.01
        assert rs <= max(4 * rr, floor), (v, t, rs, rr)   # both at rounding level
