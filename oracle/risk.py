"""Risk metrics -- oracle restatement (test infrastructure only).

risk_metrics.py: __init__ 51-82 (alpha/beta renormalised), compute_distance_risk
84-129, compute_predictive_risk 131-171, assess_risk 173-222.
"""
import numpy as np


class RiskMetrics:
    def __init__(self, d_safe=0.3, d_trigger=1.0, alpha=0.6, beta=0.4,
                 threshold_low=0.2, threshold_medium=0.5, threshold_high=0.8):
        self.d_safe = d_safe
        self.d_trigger = d_trigger
        tot = alpha + beta
        self.alpha = alpha / tot
        self.beta = beta / tot
        self.threshold_low = threshold_low
        self.threshold_medium = threshold_medium
        self.threshold_high = threshold_high

    def distance_risk(self, state, obstacles):
        """risk_metrics.py:84-129; obstacles = iterable of (x, y, r)."""
        if len(obstacles) == 0:
            return 0.0, float("inf"), -1
        px, py = state[0], state[1]
        min_d, nid, mr = float("inf"), -1, 0.0
        for i, (ox, oy, r) in enumerate(obstacles):
            d = np.sqrt((px - ox) ** 2 + (py - oy) ** 2) - r
            if d < min_d:
                min_d, nid = d, i
            if d <= self.d_safe:
                risk = 1.0
            elif d >= self.d_trigger:
                risk = 0.0
            else:
                risk = 1.0 - (d - self.d_safe) / (self.d_trigger - self.d_safe)
            mr = max(mr, risk)
        return mr, min_d, nid

    def predictive_risk(self, pred, obstacles):
        """risk_metrics.py:131-171."""
        if len(obstacles) == 0 or pred is None or len(pred) == 0:
            return 0.0
        n = len(pred)
        sev = 0.0
        for k, s in enumerate(pred):
            for (ox, oy, r) in obstacles:
                d = np.sqrt((s[0] - ox) ** 2 + (s[1] - oy) ** 2) - r
                if d < self.d_safe:
                    w = 1.0 - (k / n) * 0.5
                    sev += w * (self.d_safe - d) / self.d_safe
        mv = n * len(obstacles)
        return min(1.0, sev / mv * 5) if mv > 0 else 0.0

    def assess(self, state, obstacles, pred=None):
        """risk_metrics.py:173-222 -> dict of the RiskAssessment fields."""
        dr, md, nid = self.distance_risk(state, obstacles)
        pr = self.predictive_risk(pred, obstacles) if pred is not None else 0.0
        c = self.alpha * dr + self.beta * pr
        if c < self.threshold_low:
            lvl = "low"
        elif c < self.threshold_medium:
            lvl = "medium"
        elif c < self.threshold_high:
            lvl = "high"
        else:
            lvl = "critical"
        return dict(distance_risk=dr, predictive_risk=pr, combined_risk=c,
                    min_obstacle_distance=md, nearest_obstacle_id=nid,
                    use_mpc=bool(c >= self.threshold_low), risk_level=lvl)
