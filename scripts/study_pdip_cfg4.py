"""Round-4 model study (VERDICT r03 'next' item 3): would an interior-point tail shorten the
hardest robots at BASELINE config 4?  CPU only, oracle code (test infrastructure).

For config 4's workload (N = 30, the union-8 obstacles, 32768 robots, seed 2) the C port staged
like the device (fast cap 12, tail PDAS cap 6, then projected Newton) gives each robot's
iteration count; the device pipeline follows the same path (tests: config 3's histogram matches
robot by robot).  For the hardest robots, oracle/qp.py's dense Mehrotra PDIP is run for K
iterations and then its active-set polish (PDAS exchanges on the exact KKT system); the study
reports the smallest K after which the polish certifies the exact optimum in one exchange
round, i.e. what "PDIP then one PDAS solve" would need.
Usage: python scripts/study_pdip_cfg4.py [n_hardest]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd")]
from oracle import cpu, figure8, mpc as ompc, qp  # noqa: E402
from rmpc import workloads as W  # noqa: E402


def polish_rounds(H, c, E, f, G, h, z, t, max_rounds=10):
    """PDAS exchanges from the interior point's active set; returns rounds to certification."""
    act = z > t
    m, p = E.shape[0], G.shape[0]
    scale = 1.0 + max(np.abs(c).max(initial=0), np.abs(h).max(initial=0))
    for r in range(1, max_rounds + 1):
        C = np.vstack([E, G[act]])
        d = np.concatenate([f, h[act]])
        wp, lam = qp._kkt_solve(H, C, -c, d)
        lam = -lam
        slack = G @ wp - h
        viol = (~act) & (slack < -1e-10 * (1 + np.abs(h)))
        lz = np.zeros(p)
        lz[act] = lam[m:]
        neg = act & (lz < -1e-10 * scale)
        if not viol.any() and not neg.any():
            return r, wp
        act = (act | viol) & ~neg
    return None, None


def main():
    nh = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    cfg = W.CONFIGS["cfg4"]
    N, obs, B = cfg["N"], cfg["obs"], 32768
    idx = np.arange(B)
    xr, ur = figure8.offset_segments(2.0, 0.5, 0.02, W.t0_at(idx, B), N + 1)
    x0 = xr[:, 0] + W.noise_at(idx, cfg["seed"])
    cp = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
    cpu.set_pdas_caps(12, 6)
    r = cpu.mpc_solve_batch(cp, x0, xr, ur, obs, step_count=np.full(B, 10, np.int32), threads=8)
    cpu.set_pdas_caps(0, 0)
    its = r["iters"]
    hist = np.bincount(its)
    print("C port staged (12, 6) iterations: max", its.max(), "p99", np.percentile(its, 99),
          "robots >= 25:", int((its >= 25).sum()), "histogram tail:", hist[20:].tolist())
    hard = np.argsort(-its)[:nh]
    oc = ompc.MPCController(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02)
    rows = []
    for b in hard:
        H, c, const, E, f, G, h, L = oc.build_ltv(x0[b], xr[b], ur[b], obs)
        full = qp.solve_qp(H, c, E, f, G, h, tol=1e-11, polish=False, certify=False)
        kmin = None
        for K in range(4, full.iters + 1):
            res = qp.solve_qp(H, c, E, f, G, h, max_iter=K, tol=1e-30, polish=False, certify=False)
            t = G @ res.w - h
            rounds, wp = polish_rounds(H, c, E, f, G, h, res.z, t)
            if rounds == 1:
                kmin = K
                du = np.abs(wp[L["iu"]:L["iu"] + 2 * N] - r["u_seq"][b].ravel() + ur[b, :N].ravel()).max()
                break
        rows.append((int(b), int(its[b]), full.iters, kmin, du if kmin else None))
        print(f"robot {b}: device-path iterations {its[b]}, PDIP to 1e-11: {full.iters}, "
              f"PDIP + one PDAS polish: {kmin}", flush=True)
    k = np.array([q[3] if q[3] is not None else -1 for q in rows])
    print("hardest", nh, "robots: device-path iterations mean %.1f max %d; PDIP+polish mean %.1f max %d (failed %d)"
          % (np.mean([q[1] for q in rows]), max(q[1] for q in rows), k[k > 0].mean(), k.max(), int((k < 0).sum())))


if __name__ == "__main__":
    main()
