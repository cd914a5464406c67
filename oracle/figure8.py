"""Figure-8 reference trajectory -- oracle restatement (test infrastructure only).

Follows reference_generator.py:
  position 86-101, velocity 103-118, heading 120-133, linear_velocity 135-148,
  angular_velocity 150-172, generate 196-230, get_reference_at_index 277-297,
  get_trajectory_segment 299-326.
"""
import numpy as np


class Figure8:
    def __init__(self, A=2.0, a=0.5, dt=0.02):
        self.A = A
        self.a = a
        self.dt = dt
        self._traj = None

    # reference_generator.py:86-101
    def position(self, t):
        px = self.A * np.sin(self.a * t)
        py = self.A * np.sin(self.a * t) * np.cos(self.a * t)
        return px, py

    # reference_generator.py:103-118
    def velocity(self, t):
        dpx = self.a * self.A * np.cos(self.a * t)
        dpy = self.a * self.A * (np.cos(self.a * t) ** 2 - np.sin(self.a * t) ** 2)
        return dpx, dpy

    # reference_generator.py:120-133
    def heading(self, t):
        dpx, dpy = self.velocity(t)
        return np.arctan2(dpy, dpx)

    # reference_generator.py:135-148
    def linear_velocity(self, t):
        dpx, dpy = self.velocity(t)
        return np.sqrt(dpx ** 2 + dpy ** 2)

    # reference_generator.py:150-172 (while-loop wrap of the forward difference)
    def angular_velocity(self, t):
        th0 = self.heading(t)
        th1 = self.heading(t + self.dt)
        d = th1 - th0
        while d > np.pi:
            d -= 2 * np.pi
        while d < -np.pi:
            d += 2 * np.pi
        return d / self.dt

    def reference_at_time(self, t):
        px, py = self.position(t)
        return (np.array([px, py, self.heading(t)]),
                np.array([self.linear_velocity(t), self.angular_velocity(t)]))

    # reference_generator.py:196-230 ; table columns [t, px, py, theta, v, omega]
    def generate(self, duration):
        t = np.arange(0, duration, self.dt)
        tr = np.zeros((len(t), 6))
        tr[:, 0] = t
        for k, tk in enumerate(t):
            px, py = self.position(tk)
            tr[k, 1] = px
            tr[k, 2] = py
            tr[k, 3] = self.heading(tk)
            tr[k, 4] = self.linear_velocity(tk)
            tr[k, 5] = self.angular_velocity(tk)
        self._traj = tr
        return tr

    # reference_generator.py:277-297 (clamp to last row)
    def reference_at_index(self, k):
        k = min(k, len(self._traj) - 1)
        p = self._traj[k]
        return np.array([p[1], p[2], p[3]]), np.array([p[4], p[5]])

    # reference_generator.py:299-326 (end clamp)
    def segment(self, start, horizon):
        n = len(self._traj)
        idx = np.minimum(start + np.arange(horizon), n - 1)
        rows = self._traj[idx]
        return rows[:, 1:4].copy(), rows[:, 4:6].copy()


def offset_segments(A, a, dt, t0, rows):
    """Analytic Figure-8 segments for robots with time offsets t0 (shape [B]).

    Row i of robot b is the reference at time t0[b] + i*dt, evaluated exactly as
    reference_generator.py:86-172 (get_reference_at_time).  This is the
    synthetic workload of BASELINE configs 2-5.
    Returns x_refs [B, rows, 3], u_refs [B, rows, 2].
    """
    g = Figure8(A, a, dt)
    t = np.asarray(t0, dtype=np.float64)[:, None] + dt * np.arange(rows)[None, :]
    px = A * np.sin(a * t)
    py = A * np.sin(a * t) * np.cos(a * t)
    dpx = a * A * np.cos(a * t)
    dpy = a * A * (np.cos(a * t) ** 2 - np.sin(a * t) ** 2)
    th = np.arctan2(dpy, dpx)
    v = np.sqrt(dpx ** 2 + dpy ** 2)
    t1 = t + dt
    dpx1 = a * A * np.cos(a * t1)
    dpy1 = a * A * (np.cos(a * t1) ** 2 - np.sin(a * t1) ** 2)
    th1 = np.arctan2(dpy1, dpx1)
    d = th1 - th
    # vectorised form of the while-loop wrap (|d| < 3*pi here, so one pass each way
    # is exact; mirrored by a scalar loop in tests for the edge cases)
    d = np.where(d > np.pi, d - 2 * np.pi, d)
    d = np.where(d < -np.pi, d + 2 * np.pi, d)
    w = d / dt
    del g
    return np.stack([px, py, th], -1), np.stack([v, w], -1)
