"""Unicycle plant + linearisation -- oracle restatement (test infrastructure only).

differential_drive.py: continuous_dynamics 111-136, simulate_step 138-172,
clip_control 199-213, normalize_angle 215-230.
linearization.py: get_discrete_model_explicit 190-225.
"""
import numpy as np


def normalize_angle(angle):
    """differential_drive.py:215-230 / mpc_controller.py:540-546 (while loops)."""
    while angle > np.pi:
        angle -= 2 * np.pi
    while angle < -np.pi:
        angle += 2 * np.pi
    return angle


def discrete_model_explicit(v_r, theta_r, dt):
    """linearization.py:190-225."""
    s = np.sin(theta_r)
    c = np.cos(theta_r)
    A = np.array([[1, 0, -v_r * s * dt],
                  [0, 1, v_r * c * dt],
                  [0, 0, 1]], dtype=np.float64)
    B = np.array([[c * dt, 0],
                  [s * dt, 0],
                  [0, dt]], dtype=np.float64)
    return A, B


def clip_control(u, v_max, omega_max):
    """differential_drive.py:199-213."""
    return np.array([np.clip(u[0], -v_max, v_max), np.clip(u[1], -omega_max, omega_max)])


def dynamics(x, u):
    """differential_drive.py:111-136."""
    return np.array([u[0] * np.cos(x[2]), u[0] * np.sin(x[2]), u[1]])


def simulate_step(x, u, dt, v_max, omega_max, method="euler"):
    """differential_drive.py:138-172."""
    u = clip_control(u, v_max, omega_max)
    x = np.asarray(x, dtype=np.float64)
    if method == "euler":
        nx = x + dt * dynamics(x, u)
    elif method == "rk4":
        k1 = dynamics(x, u)
        k2 = dynamics(x + 0.5 * dt * k1, u)
        k3 = dynamics(x + 0.5 * dt * k2, u)
        k4 = dynamics(x + dt * k3, u)
        nx = x + (dt / 6.0) * (k1 + 2 * k2 + 2 * k3 + k4)
    else:
        raise ValueError(method)
    nx[2] = normalize_angle(nx[2])
    return nx
