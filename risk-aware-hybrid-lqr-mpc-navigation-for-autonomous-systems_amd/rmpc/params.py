"""params.yaml surface (src/hybrid_controller/config/params.yaml:6-51).

The reference ships params.yaml but never loads it; this loader
maps its sections onto the constructor arguments of the drop-in controllers and onto
the C-ABI parameter structs, so a deployment can configure the batched path from the
same file.
"""
import yaml

from . import _native as nat


def load_params(path):
    with open(path) as f:
        return yaml.safe_load(f)


def lqr_kwargs(cfg):
    """params.yaml lqr/robot/simulation -> LQRController(**kwargs)."""
    lq, rb, sim = cfg.get("lqr", {}), cfg.get("robot", {}), cfg.get("simulation", {})
    return dict(Q_diag=list(lq.get("Q_diag", [10.0, 10.0, 1.0])),
                R_diag=list(lq.get("R_diag", [0.1, 0.1])), dt=float(sim.get("dt", 0.02)),
                v_max=float(rb.get("max_linear_velocity", 1.0)),
                omega_max=float(rb.get("max_angular_velocity", 1.5)))


def mpc_kwargs(cfg):
    """params.yaml mpc/robot/simulation -> MPCController(**kwargs)."""
    mp, rb, sim = cfg.get("mpc", {}), cfg.get("robot", {}), cfg.get("simulation", {})
    return dict(horizon=int(mp.get("horizon", 10)), Q_diag=list(mp.get("Q_diag", [10.0, 10.0, 50.0])),
                R_diag=list(mp.get("R_diag", [0.1, 0.1])),
                P_diag=list(mp.get("P_diag", [20.0, 20.0, 40.0])),
                d_safe=float(mp.get("d_safe", 0.3)),
                slack_penalty=float(mp.get("slack_penalty", 5000.0)),
                v_max=float(rb.get("max_linear_velocity", 1.0)),
                omega_max=float(rb.get("max_angular_velocity", 1.5)),
                dt=float(sim.get("dt", 0.02)), solver=str(mp.get("solver", "OSQP")))


def mpc_struct(cfg, ltv=True, block_size=1):
    k = mpc_kwargs(cfg)
    return nat.mpc_params(k["horizon"], k["Q_diag"], k["R_diag"], k["P_diag"], k["d_safe"],
                          k["slack_penalty"], k["v_max"], k["omega_max"], k["dt"],
                          block_size=block_size, ltv=ltv)


def lqr_struct(cfg):
    k = lqr_kwargs(cfg)
    return nat.lqr_params(k["Q_diag"], k["R_diag"], k["dt"], k["v_max"], k["omega_max"])
