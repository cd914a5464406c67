"""MPC controller -- oracle restatement (test infrastructure only).

Builds the reference's QPs literally -- the same decision variables, cost and
constraints CVXPY is given in mpc_controller.py -- and solves them exactly with
``oracle.qp.solve_qp`` (CVXPY/OSQP/ECOS are absent from this image):

* ``solve_with_ltv``  mpc_controller.py:345-522  (error-state LTV, move blocking,
  np.unwrap of the reference heading, x0 heading moved into the reference branch,
  cold-start omega ramp, step counter only on success)
* ``solve``           mpc_controller.py:150-314  (absolute-state LTI, padding)
* ``fallback``        mpc_controller.py:316-343
"""
import numpy as np

from .plant import discrete_model_explicit, normalize_angle
from .qp import solve_qp

KP_FALLBACK = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, 0.5]])   # mpc_controller.py:327-328


class OracleFailure(RuntimeError):
    """The exact QP oracle did not converge ("max_iter"): a failure of the checker, never a
    verdict on the QP -- so it is raised, not turned into the reference's fallback law (which
    the reference applies only when CVXPY reports the problem infeasible/unsolved,
    mpc_controller.py:521-522)."""


def _check_converged(res):
    if res.status == "max_iter":
        raise OracleFailure(f"oracle/qp.py: no convergence in {res.iters} iterations")


class Solution:
    def __init__(self, status, u0, u_seq, x_pred, cost, slack_used, iters=0, qp_status=""):
        self.status = status
        self.optimal_control = u0
        self.control_sequence = u_seq
        self.predicted_states = x_pred
        self.cost = cost
        self.slack_used = slack_used
        self.iterations = iters
        self.qp_status = qp_status


class MPCController:
    """Constructor defaults follow mpc_controller.py:89-148."""

    def __init__(self, horizon=10, Q_diag=None, R_diag=None, P_diag=None, d_safe=0.3,
                 slack_penalty=5000.0, v_max=1.0, omega_max=1.5, dt=0.02, solver="OSQP",
                 block_size=1):
        self.N = horizon
        self.dt = dt
        self.d_safe = d_safe
        self.slack_penalty = slack_penalty
        self.v_max = v_max
        self.omega_max = omega_max
        self.solver = solver
        self.block_size = block_size
        self.N_blocks = (horizon + block_size - 1) // block_size          # :121
        self.Q = np.diag(Q_diag if Q_diag is not None else [10.0, 10.0, 50.0])
        self.R = np.diag(R_diag if R_diag is not None else [0.1, 0.1])
        self.P = np.diag(P_diag if P_diag is not None else [20.0, 20.0, 40.0])
        self._step_count = 0
        self._ramp_up_steps = 10                                            # :144

    def reset(self):
        self._step_count = 0

    def _clip(self, u):
        return np.array([np.clip(u[0], -self.v_max, self.v_max),
                         np.clip(u[1], -self.omega_max, self.omega_max)])

    # ------------------------------------------------------------------ fallback
    def fallback(self, x0, x_refs, u_refs):
        """mpc_controller.py:316-343."""
        e = np.asarray(x0, dtype=np.float64) - x_refs[0]
        e[2] = normalize_angle(e[2])
        u = self._clip(u_refs[0] + (-KP_FALLBACK @ e))
        return Solution("fallback", u, np.tile(u, (self.N, 1)),
                        np.tile(np.asarray(x0, dtype=np.float64), (self.N + 1, 1)),
                        float("inf"), False)

    # ----------------------------------------------------------------- LTV QP
    def build_ltv(self, x0, x_refs, u_refs, obstacles, soft=True):
        """The QP of mpc_controller.py:366-468, variables w = [dx (N+1,3), du_b (Nb,2), s].

        Returns (H, c, const, E, f, G, h, layout) for 1/2 w'Hw + c'w + const.
        """
        N, nb, bs = self.N, self.N_blocks, self.block_size
        x0 = np.asarray(x0, dtype=np.float64)
        obstacles = list(obstacles or [])
        no = len(obstacles)
        use_slack = soft and no > 0                                         # :383-386
        ns = N * no if use_slack else 0
        ix = 0
        iu = 3 * (N + 1)
        isl = iu + 2 * nb
        n = isl + ns
        blk = [min(k // bs, nb - 1) for k in range(N)]                      # :374-380

        xr = x_refs.copy()
        xr[:, 2] = np.unwrap(x_refs[:, 2])                                  # :392-393
        th0 = xr[0, 2]
        x0a = x0.copy()
        x0a[2] = th0 + normalize_angle(x0[2] - th0)                         # :397-401

        H = np.zeros((n, n))
        c = np.zeros(n)
        const = 0.0
        for k in range(N):                                                  # :403-409
            H[ix + 3 * k: ix + 3 * k + 3, ix + 3 * k: ix + 3 * k + 3] += 2 * self.Q
            j = iu + 2 * blk[k]
            H[j:j + 2, j:j + 2] += 2 * self.R
            c[j:j + 2] += 2 * self.R @ u_refs[k]
            const += u_refs[k] @ self.R @ u_refs[k]
        H[ix + 3 * N: ix + 3 * N + 3, ix + 3 * N: ix + 3 * N + 3] += 2 * self.P  # :412
        for i in range(ns):                                                 # :414-415
            H[isl + i, isl + i] += 2 * self.slack_penalty

        Erows, frows = [], []
        for r in range(3):                                                  # :421
            e = np.zeros(n)
            e[ix + r] = 1.0
            Erows.append(e)
            frows.append(x0a[r] - xr[0, r])
        for k in range(N):                                                  # :424-428
            v_r = u_refs[k, 0] if abs(u_refs[k, 0]) > 0.01 else 0.1
            A, B = discrete_model_explicit(v_r, xr[k, 2], self.dt)
            for r in range(3):
                e = np.zeros(n)
                e[ix + 3 * (k + 1) + r] = 1.0
                e[ix + 3 * k: ix + 3 * k + 3] -= A[r]
                j = iu + 2 * blk[k]
                e[j:j + 2] -= B[r]
                Erows.append(e)
                frows.append(0.0)

        Grows, hrows = [], []
        for k in range(N):                                                  # :431-436
            j = iu + 2 * blk[k]
            for comp, lim in ((0, self.v_max), (1, self.omega_max)):
                e = np.zeros(n)
                e[j + comp] = 1.0
                Grows.append(e)
                hrows.append(-lim - u_refs[k, comp])
                e = np.zeros(n)
                e[j + comp] = -1.0
                Grows.append(e)
                hrows.append(-lim + u_refs[k, comp])
        si = 0
        for (ox, oy, rad) in obstacles:                                     # :439-468
            for k in range(N):
                px, py = xr[k, 0], xr[k, 1]
                ddx, ddy = px - ox, py - oy
                dist = np.sqrt(ddx ** 2 + ddy ** 2)
                if dist > 0.01:
                    nx, ny = ddx / dist, ddy / dist
                    safe = self.d_safe + rad
                    e = np.zeros(n)
                    e[ix + 3 * k] = nx
                    e[ix + 3 * k + 1] = ny
                    rhs = safe - (nx * (px - ox) + ny * (py - oy))
                    if use_slack:
                        e[isl + si] = 1.0
                        si += 1
                    Grows.append(e)
                    hrows.append(rhs)
        for i in range(ns):                                                 # nonneg slack
            e = np.zeros(n)
            e[isl + i] = 1.0
            Grows.append(e)
            hrows.append(0.0)
        layout = dict(ix=ix, iu=iu, isl=isl, ns=ns, blk=blk, xr=xr)
        return (H, c, const, np.array(Erows), np.array(frows),
                np.array(Grows).reshape(-1, n), np.array(hrows), layout)

    def solve_with_ltv(self, x0, x_refs, u_refs, obstacles=None, use_soft_constraints=True):
        """mpc_controller.py:345-522."""
        x_refs = np.asarray(x_refs, dtype=np.float64)
        u_refs = np.asarray(u_refs, dtype=np.float64)
        H, c, const, E, f, G, h, L = self.build_ltv(x0, x_refs, u_refs, obstacles,
                                                    use_soft_constraints)
        res = solve_qp(H, c, E, f, G, h)
        _check_converged(res)
        if res.status != "optimal":
            return self.fallback(x0, x_refs, u_refs)                        # :521-522
        w = res.w
        N = self.N
        dx = w[L["ix"]: L["ix"] + 3 * (N + 1)].reshape(N + 1, 3)
        dub = w[L["iu"]: L["iu"] + 2 * self.N_blocks].reshape(self.N_blocks, 2)
        du = dub[[min(k // self.block_size, self.N_blocks - 1) for k in range(N)]]  # :490-495
        s = w[L["isl"]: L["isl"] + L["ns"]]
        slack_used = bool(L["ns"] > 0 and np.any(s > 1e-6))                 # :485
        x_pred = x_refs[:N + 1] + dx                                        # :497
        u_pred = u_refs[:N] + du                                            # :498
        if self._step_count < self._ramp_up_steps:                          # :502-505
            lim = self.omega_max * ((self._step_count + 1) / self._ramp_up_steps)
            u_pred[0, 1] = np.clip(u_pred[0, 1], -lim, lim)
        self._step_count += 1                                               # :507
        cost = 0.5 * w @ H @ w + c @ w + const
        return Solution("optimal", u_pred[0].copy(), u_pred, x_pred, cost, slack_used,
                        res.iters, res.status)

    # ----------------------------------------------------------------- LTI QP
    def build_lti(self, x0, x_refs, u_refs, obstacles, soft=True):
        """The QP of mpc_controller.py:172-270, variables w = [x (N+1,3), u (N,2), s]."""
        N = self.N
        x0 = np.asarray(x0, dtype=np.float64)
        x_refs = np.asarray(x_refs, dtype=np.float64)
        u_refs = np.asarray(u_refs, dtype=np.float64)
        if x_refs.shape[0] < N + 1:                                         # :172-177
            pad = np.zeros((N + 1, 3))
            pad[:x_refs.shape[0]] = x_refs
            pad[x_refs.shape[0]:] = x_refs[-1]
            x_refs = pad
        if u_refs.shape[0] < N:                                             # :179-183
            pad = np.zeros((N, 2))
            pad[:u_refs.shape[0]] = u_refs
            pad[u_refs.shape[0]:] = u_refs[-1]
            u_refs = pad
        v_r = u_refs[0, 0] if abs(u_refs[0, 0]) > 0.01 else 0.1             # :186
        A, B = discrete_model_explicit(v_r, x_refs[0, 2], self.dt)          # :187-190
        obstacles = list(obstacles or [])
        no = len(obstacles)
        use_slack = soft and no > 0
        ns = N * no if use_slack else 0
        ix, iu = 0, 3 * (N + 1)
        isl = iu + 2 * N
        n = isl + ns
        H = np.zeros((n, n))
        c = np.zeros(n)
        const = 0.0
        for k in range(N):                                                  # :206-209
            sl = slice(ix + 3 * k, ix + 3 * k + 3)
            H[sl, sl] += 2 * self.Q
            c[sl] += -2 * self.Q @ x_refs[k]
            const += x_refs[k] @ self.Q @ x_refs[k]
            H[iu + 2 * k: iu + 2 * k + 2, iu + 2 * k: iu + 2 * k + 2] += 2 * self.R
        sl = slice(ix + 3 * N, ix + 3 * N + 3)                              # :212-213
        H[sl, sl] += 2 * self.P
        c[sl] += -2 * self.P @ x_refs[N]
        const += x_refs[N] @ self.P @ x_refs[N]
        for i in range(ns):
            H[isl + i, isl + i] += 2 * self.slack_penalty
        Erows, frows = [], []
        for r in range(3):                                                  # :223
            e = np.zeros(n)
            e[ix + r] = 1.0
            Erows.append(e)
            frows.append(x0[r])
        for k in range(N):                                                  # :226-227
            for r in range(3):
                e = np.zeros(n)
                e[ix + 3 * (k + 1) + r] = 1.0
                e[ix + 3 * k: ix + 3 * k + 3] -= A[r]
                e[iu + 2 * k: iu + 2 * k + 2] -= B[r]
                Erows.append(e)
                frows.append(0.0)
        Grows, hrows = [], []
        for k in range(N):                                                  # :230-234
            for comp, lim in ((0, self.v_max), (1, self.omega_max)):
                e = np.zeros(n)
                e[iu + 2 * k + comp] = 1.0
                Grows.append(e)
                hrows.append(-lim)
                e = np.zeros(n)
                e[iu + 2 * k + comp] = -1.0
                Grows.append(e)
                hrows.append(-lim)
        si = 0
        for (ox, oy, rad) in obstacles:                                     # :237-270
            for k in range(N):
                ddx, ddy = x_refs[k, 0] - ox, x_refs[k, 1] - oy
                dist = np.sqrt(ddx ** 2 + ddy ** 2)
                if dist > 0.01:
                    nx, ny = ddx / dist, ddy / dist
                    e = np.zeros(n)
                    e[ix + 3 * k] = nx
                    e[ix + 3 * k + 1] = ny
                    rhs = self.d_safe + rad + nx * ox + ny * oy
                    if use_slack:
                        e[isl + si] = 1.0
                        si += 1
                    Grows.append(e)
                    hrows.append(rhs)
        for i in range(ns):
            e = np.zeros(n)
            e[isl + i] = 1.0
            Grows.append(e)
            hrows.append(0.0)
        layout = dict(ix=ix, iu=iu, isl=isl, ns=ns, x_refs=x_refs, u_refs=u_refs)
        return (H, c, const, np.array(Erows), np.array(frows),
                np.array(Grows).reshape(-1, n), np.array(hrows), layout)

    def solve(self, x0, x_refs, u_refs, obstacles=None, use_soft_constraints=True):
        """mpc_controller.py:150-314 (no ramp, no step-count change)."""
        H, c, const, E, f, G, h, L = self.build_lti(x0, x_refs, u_refs, obstacles,
                                                    use_soft_constraints)
        res = solve_qp(H, c, E, f, G, h)
        _check_converged(res)
        if res.status != "optimal":
            return self.fallback(x0, L["x_refs"], L["u_refs"])
        w = res.w
        N = self.N
        x = w[:3 * (N + 1)].reshape(N + 1, 3)
        u = w[L["iu"]: L["iu"] + 2 * N].reshape(N, 2)
        s = w[L["isl"]: L["isl"] + L["ns"]]
        slack_used = bool(L["ns"] > 0 and np.any(s > 1e-6))
        cost = 0.5 * w @ H @ w + c @ w + const
        return Solution("optimal", u[0].copy(), u.copy(), x.copy(), cost, slack_used,
                        res.iters, res.status)


def default_obstacles():
    """run_simulation.py:215-219 (scenario 'default')."""
    return [(1.0, 0.5, 0.2), (-0.5, -1.0, 0.25), (1.5, -0.3, 0.15)]


def scenario_obstacles(name):
    """run_simulation.py:191-219."""
    if name == "sparse":
        return [(1.5, 0.8, 0.2)]
    if name == "dense":
        return [(1.0, 0.5, 0.2), (-0.5, -1.0, 0.25), (1.5, -0.3, 0.15),
                (-1.5, 0.5, 0.2), (0.0, 0.8, 0.15)]
    if name == "corridor":
        return [(1.0, 0.3, 0.15), (1.0, 0.7, 0.15), (-0.8, -0.7, 0.15), (-0.3, -1.2, 0.15)]
    return default_obstacles()


def union8_obstacles():
    """BASELINE config 4: default 3 + dense-only 2 + sparse 1 + corridor-only 2."""
    return default_obstacles() + [(-1.5, 0.5, 0.2), (0.0, 0.8, 0.15), (1.5, 0.8, 0.2),
                                  (-0.8, -0.7, 0.15), (-0.3, -1.2, 0.15)]

