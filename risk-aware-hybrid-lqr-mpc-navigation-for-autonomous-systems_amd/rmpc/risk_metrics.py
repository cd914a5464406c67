"""RiskMetrics -- drop-in for hybrid_controller.controllers.risk_metrics (risk_metrics.py).

Same constructor (alpha/beta renormalised, :79-82), RiskAssessment fields and
switching recommendation (:212).  Evaluated on the device by rmpc_risk_batch.
"""
from dataclasses import dataclass
from typing import Dict, List, Tuple

import numpy as np

from . import _native as nat
from .batch import risk_batch

_LEVELS = ("low", "medium", "high", "critical")


@dataclass
class RiskAssessment:
    distance_risk: float
    predictive_risk: float
    combined_risk: float
    min_obstacle_distance: float
    nearest_obstacle_id: int
    use_mpc: bool
    risk_level: str


def _obs(obstacles):
    if not obstacles:
        return np.zeros((0, 3))
    return np.array([[o["x"], o["y"], o["radius"]] if isinstance(o, dict) else list(o)
                     for o in obstacles], dtype=np.float64)


class RiskMetrics:
    def __init__(self, d_safe: float = 0.3, d_trigger: float = 1.0, alpha: float = 0.6,
                 beta: float = 0.4, threshold_low: float = 0.2, threshold_medium: float = 0.5,
                 threshold_high: float = 0.8, device: int = 0):
        self.d_safe = d_safe
        self.d_trigger = d_trigger
        self._alpha_raw, self._beta_raw = alpha, beta
        total = alpha + beta
        self.alpha = alpha / total
        self.beta = beta / total
        self.threshold_low = threshold_low
        self.threshold_medium = threshold_medium
        self.threshold_high = threshold_high
        self.device = device

    def params(self, min_dwell_steps=10):
        return nat.risk_params(self.d_safe, self.d_trigger, self._alpha_raw, self._beta_raw,
                               self.threshold_low, self.threshold_medium, self.threshold_high,
                               min_dwell_steps)

    def _eval(self, states, obstacles, pred=None):
        return risk_batch(self.params(), np.atleast_2d(np.asarray(states, np.float64)),
                          _obs(obstacles), pred=pred, device=self.device)

    def compute_distance_risk(self, state: np.ndarray, obstacles: List[Dict]) -> Tuple[float, float, int]:
        """risk_metrics.py:84-129."""
        if not obstacles:
            return 0.0, float("inf"), -1
        out, _, _ = self._eval(state, obstacles)
        return float(out[0, 0]), float(out[0, 3]), int(out[0, 4])

    def compute_predictive_risk(self, predicted_states: np.ndarray, obstacles: List[Dict]) -> float:
        """risk_metrics.py:131-171."""
        if not obstacles or predicted_states is None or len(predicted_states) == 0:
            return 0.0
        p = np.asarray(predicted_states, np.float64)
        out, _, _ = self._eval(p[0], obstacles, pred=p[None])
        return float(out[0, 1])

    def assess_risk(self, state: np.ndarray, obstacles: List[Dict],
                    predicted_states: np.ndarray = None) -> RiskAssessment:
        """risk_metrics.py:173-222."""
        pred = None
        if predicted_states is not None and len(predicted_states) > 0:
            pred = np.asarray(predicted_states, np.float64)[None]
        out, use, lvl = self._eval(state, obstacles, pred=pred)
        return RiskAssessment(distance_risk=float(out[0, 0]), predictive_risk=float(out[0, 1]),
                              combined_risk=float(out[0, 2]),
                              min_obstacle_distance=float(out[0, 3]),
                              nearest_obstacle_id=int(out[0, 4]), use_mpc=bool(use[0]),
                              risk_level=_LEVELS[int(lvl[0])])

    def assess_risk_batch(self, states, obstacles, predicted_states=None):
        """B robots -> (out [B,5], use_mpc [B], level [B])."""
        return self._eval(states, obstacles, pred=predicted_states)

    def get_risk_summary(self, assessment: RiskAssessment) -> str:
        return (f"Risk: {assessment.risk_level.upper()} "
                f"(combined={assessment.combined_risk:.2f}, "
                f"dist={assessment.distance_risk:.2f}, "
                f"pred={assessment.predictive_risk:.2f}, "
                f"min_d={assessment.min_obstacle_distance:.2f}m)")
