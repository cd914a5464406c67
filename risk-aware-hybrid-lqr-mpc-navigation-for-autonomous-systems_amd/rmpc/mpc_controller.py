"""MPCController -- drop-in for hybrid_controller.controllers.mpc_controller (mpc_controller.py).

Same constructor, methods, dataclasses and error behaviour as the reference
(mpc_controller.py:33-571).  The QP is solved on the MI355X by librmpc.so
(rmpc_mpc_solve_batch) instead of building a CVXPY problem per call; ``solver`` is
accepted and recorded but the kernel always solves the QP exactly (active-set
certified), which is what OSQP's polish / ECOS return to their tolerances.

Additions for batched use: ``solve_batch`` / ``solve_with_ltv_batch`` run B robots in one
call, each robot with its own ``_step_count`` (ramp-up state).
"""
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from . import _native as nat
from .batch import mpc_solve_batch
from .linearization import Linearizer

_STATUS = {nat.RMPC_OPTIMAL: "optimal", nat.RMPC_OPTIMAL_INACCURATE: "optimal",
           nat.RMPC_FALLBACK: "fallback"}


@dataclass
class Obstacle:
    """Circular obstacle (mpc_controller.py:33-46)."""
    x: float
    y: float
    radius: float

    def distance_to(self, px: float, py: float) -> float:
        return np.sqrt((px - self.x) ** 2 + (py - self.y) ** 2)

    def is_collision(self, px: float, py: float, d_safe: float) -> bool:
        return self.distance_to(px, py) < self.radius + d_safe


@dataclass
class MPCSolution:
    """Result record (mpc_controller.py:49-59)."""
    status: str
    optimal_control: np.ndarray
    control_sequence: np.ndarray
    predicted_states: np.ndarray
    cost: float
    solve_time_ms: float
    slack_used: bool
    iterations: int


def _obstacle_array(obstacles) -> np.ndarray:
    if not obstacles:
        return np.zeros((0, 3))
    rows = []
    for o in obstacles:
        if isinstance(o, Obstacle):
            rows.append((o.x, o.y, o.radius))
        elif isinstance(o, dict):
            rows.append((o["x"], o["y"], o["radius"]))
        else:
            rows.append(tuple(o))
    return np.asarray(rows, dtype=np.float64)


class MPCController:
    """Model Predictive Controller with obstacle avoidance (mpc_controller.py:62-148)."""

    def __init__(self, horizon: int = 10, Q_diag: list = None, R_diag: list = None,
                 P_diag: list = None, d_safe: float = 0.3, slack_penalty: float = 5000.0,
                 v_max: float = 1.0, omega_max: float = 1.5, dt: float = 0.02,
                 solver: str = "OSQP", block_size: int = 1, device: int = 0, warm_start: bool = True):
        self.N = horizon
        self.dt = dt
        self.d_safe = d_safe
        self.slack_penalty = slack_penalty
        self.v_max = v_max
        self.omega_max = omega_max
        self.solver = solver
        self.block_size = block_size
        self.N_blocks = (horizon + block_size - 1) // block_size
        if Q_diag is None:
            Q_diag = [10.0, 10.0, 50.0]
        if R_diag is None:
            R_diag = [0.1, 0.1]
        if P_diag is None:
            P_diag = [20.0, 20.0, 40.0]
        self.Q = np.diag(Q_diag)
        self.R = np.diag(R_diag)
        self.P = np.diag(P_diag)
        self.linearizer = Linearizer(dt=dt)            # mpc_controller.py:136 (API surface)
        self.device = device
        # The reference solves with warm_start=True (mpc_controller.py:276-277, 474-475): here
        # each controller owns a library context whose warm-start sets are this robot's
        # previous certified active sets (rmpc_ctx_set_warm_start), shifted by one step.  Same
        # optimum, fewer PDAS iterations.  warm_start=False: the shared context, cold solves.
        self.warm_start = warm_start
        self._own: Optional[nat.OwnedContext] = None
        self._prev_solution: Optional[np.ndarray] = None
        self._prev_states: Optional[np.ndarray] = None
        self._step_count = 0
        self._ramp_up_steps = 10
        self.nx = 3
        self.nu = 2

    # -------------------------------------------------------------- params
    def _params(self, ltv: bool, soft: bool):
        return nat.mpc_params(self.N, np.diag(self.Q), np.diag(self.R), np.diag(self.P),
                              self.d_safe, self.slack_penalty, self.v_max, self.omega_max, self.dt,
                              block_size=self.block_size if ltv else 1, ltv=ltv, soft=soft,
                              ramp_up_steps=self._ramp_up_steps)

    def _context(self):
        if not self.warm_start:
            return None
        if self._own is None:
            self._own = nat.OwnedContext(self.device)     # released by its finalizer, once
            nat.check(nat.load().rmpc_ctx_set_warm_start(self._own.h, 1), "rmpc_ctx_set_warm_start")
        return self._own.h

    def __copy__(self):
        # a copy starts cold on a context of its own (never the original's handle)
        c = self.__class__.__new__(self.__class__)
        c.__dict__.update(self.__dict__)
        c._own = None
        return c

    def __deepcopy__(self, memo):
        import copy
        c = self.__class__.__new__(self.__class__)
        memo[id(self)] = c
        for k, v in self.__dict__.items():
            c.__dict__[k] = None if k == "_own" else copy.deepcopy(v, memo)
        return c

    # -------------------------------------------------------------- single robot
    def _one(self, x0, x_refs, u_refs, obstacles, soft, ltv):
        t = time.perf_counter()
        x_refs = np.asarray(x_refs, dtype=np.float64)
        u_refs = np.asarray(u_refs, dtype=np.float64)
        sc = np.array([self._step_count], np.int32)
        out = mpc_solve_batch(self._params(ltv, soft), np.asarray(x0, np.float64)[None],
                              x_refs[None], u_refs[None], _obstacle_array(obstacles),
                              step_count=sc if ltv else None, device=self.device, ctx=self._context())
        ms = (time.perf_counter() - t) * 1000.0
        st = int(out["status"][0])
        if st != nat.RMPC_FALLBACK:
            if ltv:
                self._step_count = int(sc[0])
            self._prev_solution = out["u_seq"][0]
            self._prev_states = out["x_pred"][0]
        return MPCSolution(status=_STATUS.get(st, "fallback"),
                           optimal_control=out["u0"][0].copy(),
                           control_sequence=out["u_seq"][0].copy(),
                           predicted_states=out["x_pred"][0].copy(),
                           cost=float(out["cost"][0]), solve_time_ms=ms,
                           slack_used=bool(out["slack_used"][0]),
                           iterations=int(out["iters"][0]))

    def solve(self, x0: np.ndarray, x_refs: np.ndarray, u_refs: np.ndarray,
              obstacles: List[Obstacle] = None, use_soft_constraints: bool = True) -> MPCSolution:
        """Absolute-state LTI MPC (mpc_controller.py:150-314)."""
        return self._one(x0, x_refs, u_refs, obstacles, use_soft_constraints, ltv=False)

    def solve_with_ltv(self, x0: np.ndarray, x_refs: np.ndarray, u_refs: np.ndarray,
                       obstacles: List[Obstacle] = None,
                       use_soft_constraints: bool = True) -> MPCSolution:
        """Error-state LTV MPC with move blocking and ramp-up (mpc_controller.py:345-522)."""
        return self._one(x0, x_refs, u_refs, obstacles, use_soft_constraints, ltv=True)

    # -------------------------------------------------------------- batched
    def solve_with_ltv_batch(self, x0, x_refs, u_refs, obstacles=None, step_count=None,
                             use_soft_constraints=True, want_seq=True) -> Dict[str, np.ndarray]:
        """B robots in one call; step_count [B] int32 (per-robot _step_count, updated)."""
        return mpc_solve_batch(self._params(True, use_soft_constraints), x0, x_refs, u_refs,
                               _obstacle_array(obstacles), step_count=step_count,
                               device=self.device, want_seq=want_seq)

    def solve_batch(self, x0, x_refs, u_refs, obstacles=None, use_soft_constraints=True,
                    want_seq=True) -> Dict[str, np.ndarray]:
        return mpc_solve_batch(self._params(False, use_soft_constraints), x0, x_refs, u_refs,
                               _obstacle_array(obstacles), device=self.device, want_seq=want_seq)

    def _get_fallback_solution(self, x0: np.ndarray, x_refs: np.ndarray, u_refs: np.ndarray,
                               solve_time: float) -> MPCSolution:
        """The fallback law (mpc_controller.py:316-343): proportional control on the wrapped
        tracking error, clipped.  The library applies the same law in-kernel to every robot
        whose QP fails (status RMPC_FALLBACK); this method serves callers that invoke it
        directly."""
        x0 = np.asarray(x0, dtype=np.float64)
        error = x0 - np.asarray(x_refs, dtype=np.float64)[0]
        error[2] = self._normalize_angle(error[2])
        K_p = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, 0.5]])
        u = self._clip_control(np.asarray(u_refs, dtype=np.float64)[0] - K_p @ error)
        return MPCSolution(status="fallback", optimal_control=u,
                           control_sequence=np.tile(u, (self.N, 1)),
                           predicted_states=np.tile(x0, (self.N + 1, 1)), cost=float("inf"),
                           solve_time_ms=solve_time, slack_used=False, iterations=0)

    # -------------------------------------------------------------- helpers (:524-571)
    def get_warm_start(self) -> Optional[np.ndarray]:
        if self._prev_solution is None:
            return None
        w = np.zeros_like(self._prev_solution)
        w[:-1] = self._prev_solution[1:]
        w[-1] = self._prev_solution[-1]
        return w

    def _normalize_angle(self, angle: float) -> float:
        while angle > np.pi:
            angle -= 2 * np.pi
        while angle < -np.pi:
            angle += 2 * np.pi
        return angle

    def reset(self):
        self._step_count = 0
        self._prev_solution = None
        self._prev_states = None
        if self._own is not None:           # cold sets again (reset: mpc_controller.py:548-552)
            nat.check(nat.load().rmpc_ctx_set_warm_start(self._own.h, 1), "rmpc_ctx_set_warm_start")

    def _clip_control(self, u: np.ndarray) -> np.ndarray:
        return np.array([np.clip(u[0], -self.v_max, self.v_max),
                         np.clip(u[1], -self.omega_max, self.omega_max)])

    def set_obstacles(self, obstacles: List[Dict[str, float]]) -> List[Obstacle]:
        return [Obstacle(x=o["x"], y=o["y"], radius=o["radius"]) for o in obstacles]
