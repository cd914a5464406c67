"""Offline study of the hard MPC instances of BASELINE config 3 (CPU only, not product code).

Generates the cfg3 workload on the host, runs the C port (oracle/c) to find the robots that
need the most active-set iterations, and replays them with a small numpy PDAS on the
condensed problem (same set rules as the kernels), printing the active-set trajectory and
trying alternative strategies.  Usage: python scripts/study_hard.py [n_robots]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd")]
from oracle import cpu  # noqa: E402
from oracle.figure8 import offset_segments  # noqa: E402
from rmpc import workloads as W  # noqa: E402

Q = np.array([15., 15., 50.]); R = np.array([.1, .1]); P = np.array([30., 30., 40.])
RHO, DSAFE, VMAX, WMAX, DT = 5000.0, 0.3, 2.0, 3.0, 0.02


def condensed(x0, xr, ur, obs, N=20):
    th = np.unwrap(xr[:, 2])
    th0 = th[0]
    d = x0[2] - th0
    while d > np.pi:
        d -= 2 * np.pi
    while d < -np.pi:
        d += 2 * np.pi
    dx0 = np.array([x0[0] - xr[0, 0], x0[1] - xr[0, 1], d])
    n = 2 * N
    A = []; Bm = []
    for k in range(N):
        v = ur[k, 0] if abs(ur[k, 0]) > 0.01 else 0.1
        s, c = np.sin(th[k]), np.cos(th[k])
        A.append(np.array([[1, 0, -v * s * DT], [0, 1, v * c * DT], [0, 0, 1]]))
        Bm.append(np.array([[c * DT, 0], [s * DT, 0], [0, DT]]))
    G = np.zeros((N + 1, 3, n)); xf = np.zeros((N + 1, 3)); xf[0] = dx0
    for k in range(N):
        xf[k + 1] = A[k] @ xf[k]
        G[k + 1] = A[k] @ G[k]
        G[k + 1][:, 2 * k:2 * k + 2] += Bm[k]
    H = np.zeros((n, n)); g = np.zeros(n)
    for k in range(1, N + 1):
        W_ = Q if k < N else P
        H += 2 * G[k].T @ np.diag(W_) @ G[k]
        g += 2 * G[k].T @ (W_ * xf[k])
    for k in range(N):
        H[2 * k, 2 * k] += 2 * R[0]; H[2 * k + 1, 2 * k + 1] += 2 * R[1]
        g[2 * k] += 2 * R[0] * ur[k, 0]; g[2 * k + 1] += 2 * R[1] * ur[k, 1]
    rows = []     # (k, a (n,), c) with r = c - a.z
    for k in range(1, N):
        for (ox, oy, rad) in obs:
            ddx, ddy = xr[k, 0] - ox, xr[k, 1] - oy
            dist = np.hypot(ddx, ddy)
            if dist > 0.01:
                nx, ny = ddx / dist, ddy / dist
                hb = DSAFE + rad - (nx * ddx + ny * ddy)
                a = nx * G[k][0] + ny * G[k][1]
                rows.append((k, a, hb - nx * xf[k, 0] - ny * xf[k, 1]))
    lo = np.empty(n); hi = np.empty(n)
    for k in range(N):
        lo[2 * k] = -VMAX - ur[k, 0]; hi[2 * k] = VMAX - ur[k, 0]
        lo[2 * k + 1] = -WMAX - ur[k, 1]; hi[2 * k + 1] = WMAX - ur[k, 1]
    Am = np.array([r[1] for r in rows]).reshape(-1, n); cv = np.array([r[2] for r in rows])
    return H, g, Am, cv, lo, hi


def solve_sets(H, g, Am, cv, S, bf, lo, hi):
    n = H.shape[0]
    M = H + 2 * RHO * Am[S].T @ Am[S]
    q = g - 2 * RHO * Am[S].T @ cv[S]
    fixed = bf != 0
    zf = np.where(bf == 1, lo, hi)
    z = np.where(fixed, zf, 0.0)
    F = ~fixed
    if F.any():
        z[F] = np.linalg.solve(M[np.ix_(F, F)], -(q[F] + M[np.ix_(F, fixed)] @ z[fixed]))
    lam = M @ z + q
    return z, lam


def pdas(H, g, Am, cv, lo, hi, maxit=60, trace=False, S0=None, bf0=None):
    m = Am.shape[0]; n = H.shape[0]
    S = np.zeros(m, bool) if S0 is None else S0.copy()
    bf = np.zeros(n, int) if bf0 is None else bf0.copy()
    hist = []
    for it in range(1, maxit + 1):
        z, lam = solve_sets(H, g, Am, cv, S, bf, lo, hi)
        r = cv - Am @ z
        nS = np.where(S, r > -1e-14, r > 1e-14)
        nb = bf.copy()
        for i in range(n):
            if bf[i] == 0:
                nb[i] = 1 if z[i] < lo[i] - 1e-13 else (2 if z[i] > hi[i] + 1e-13 else 0)
            elif bf[i] == 1:
                nb[i] = 0 if lam[i] < 0 else 1
            else:
                nb[i] = 0 if lam[i] > 0 else 2
        if trace:
            dS = np.nonzero(nS != S)[0]; db = np.nonzero(nb != bf)[0]
            print(f"   it {it:2d}: |S|={S.sum():2d} |fix|={(bf != 0).sum():2d}  dS={list(dS)} dbox={list(db)}")
        if (nS == S).all() and (nb == bf).all():
            return it, z
        key = (nS.tobytes(), nb.tobytes())
        if key in hist:
            if trace:
                print("   cycle")
            return -it, z
        hist.append(key)
        S, bf = nS, nb
    return -maxit, z


def main():
    nrob = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    B = 65536
    lo, hi = 0, B
    t0 = W.t0_offsets(lo, hi, B)
    xr, ur = offset_segments(2.0, 0.5, 0.02, t0, 21)
    x0 = xr[:, 0] + W.noise_for(lo, hi, 1)
    obs = W.DEFAULT_OBS
    p = cpu.mpc_params(20, Q, R, P, DSAFE, RHO, VMAX, WMAX, DT)
    sel = np.arange(0, B, max(1, B // nrob))
    out = cpu.mpc_solve_batch(p, x0[sel], xr[sel], ur[sel], obs, step_count=np.full(len(sel), 10, np.int32),
                              threads=8)
    it = out["iters"]
    print("iterations: mean %.2f p99 %d max %d" % (it.mean(), np.percentile(it, 99), it.max()))
    hard = sel[np.argsort(-it)[:8]]
    for b in hard:
        Hm, g, Am, cv, blo, bhi = condensed(x0[b], xr[b], ur[b], obs)
        print(f"robot {b}: C-port iters {it[list(sel).index(b)]}, rows {Am.shape[0]}")
        k, z = pdas(Hm, g, Am, cv, blo, bhi, trace=True)
        print("   pdas ->", k)




def F_val(H, g, Am, cv, z):
    r = np.maximum(cv - Am @ z, 0.0)
    return 0.5 * z @ H @ z + g @ z + RHO * r @ r


def grad_val(H, g, Am, cv, z):
    r = np.maximum(cv - Am @ z, 0.0)
    return H @ z + g - 2 * RHO * Am.T @ r


def proj_newton(H, g, Am, cv, lo, hi, z, maxit=60, trace=False):
    """The kernels' phase 2: eps-active sets, Newton on the free set with the r>0 hinge piece,
    PDAS test of the candidate, Armijo along the projection arc."""
    F = F_val(H, g, Am, cv, z)
    for it in range(1, maxit + 1):
        gz = grad_val(H, g, Am, cv, z)
        eps = min(1e-6, np.max(np.abs(z - np.clip(z - gz, lo, hi))))
        S = (cv - Am @ z) > 0
        bf = np.where((z <= lo + eps) & (gz > 0), 1, np.where((z >= hi - eps) & (gz < 0), 2, 0))
        zc, lam = solve_sets(H, g, Am, cv, S, bf, lo, hi)
        # certification = PDAS test on the candidate
        r = cv - Am @ zc
        nS = np.where(S, r > -1e-14, r > 1e-14)
        ok = (nS == S).all()
        for i in range(len(z)):
            e = lam[i] if bf[i] else zc[i]
            if bf[i] == 0 and (e < lo[i] - 1e-13 or e > hi[i] + 1e-13):
                ok = False
            if bf[i] == 1 and e < 0:
                ok = False
            if bf[i] == 2 and e > 0:
                ok = False
        if ok:
            return it, zc
        a, acc = 1.0, False
        for _ in range(40):
            zt = np.clip(z + a * (zc - z), lo, hi)
            Ft = F_val(H, g, Am, cv, zt)
            if Ft <= F + 1e-4 * gz @ (zt - z):
                acc = True
                break
            a *= 0.5
        if trace:
            print(f"      pn it {it}: alpha {a:.3g} F {Ft:.12g} |fix| {(bf != 0).sum()} |S| {S.sum()}")
        if not acc:
            return -it, z
        z, F = zt, Ft
    return -maxit, z


def study_alternatives(nrob=65536):
    B = 65536
    t0 = W.t0_offsets(0, B, B)
    xr, ur = offset_segments(2.0, 0.5, 0.02, t0, 21)
    x0 = xr[:, 0] + W.noise_for(0, B, 1)
    p = cpu.mpc_params(20, Q, R, P, DSAFE, RHO, VMAX, WMAX, DT)
    out = cpu.mpc_solve_batch(p, x0, xr, ur, W.DEFAULT_OBS, step_count=np.full(B, 10, np.int32), threads=8)
    it = out["iters"]
    hard = np.argsort(-it)[:40]
    rows = []
    for b in hard:
        Hm, g, Am, cv, blo, bhi = condensed(x0[b], xr[b], ur[b], W.DEFAULT_OBS)
        k_pdas, _ = pdas(Hm, g, Am, cv, blo, bhi)
        # phase 2 from the projected unconstrained minimiser (no PDAS at all)
        z_unc = np.linalg.solve(Hm, -g)
        k_pn0, z1 = proj_newton(Hm, g, Am, cv, blo, bhi, np.clip(z_unc, blo, bhi))
        # PDAS for 4 iterations, then phase 2 from the projected iterate
        S = np.zeros(Am.shape[0], bool); bf = np.zeros(40, int)
        for _ in range(4):
            zc, lam = solve_sets(Hm, g, Am, cv, S, bf, blo, bhi)
            r = cv - Am @ zc
            S = np.where(S, r > -1e-14, r > 1e-14)
            nb = bf.copy()
            for i in range(40):
                if bf[i] == 0:
                    nb[i] = 1 if zc[i] < blo[i] - 1e-13 else (2 if zc[i] > bhi[i] + 1e-13 else 0)
                elif bf[i] == 1:
                    nb[i] = 0 if lam[i] < 0 else 1
                else:
                    nb[i] = 0 if lam[i] > 0 else 2
            bf = nb
        k_pn4, z2 = proj_newton(Hm, g, Am, cv, blo, bhi, np.clip(zc, blo, bhi))
        rows.append((b, it[b], k_pdas, k_pn0, k_pn4, np.abs(z1 - z2).max()))
    print(" robot  Cport  pdas  PN-from-unc  PDAS4+PN  |dz|")
    for r in rows:
        print("%6d %6d %5d %12d %9d  %.1e" % r)





def study_classify():
    B = 65536
    t0 = W.t0_offsets(0, B, B)
    xr, ur = offset_segments(2.0, 0.5, 0.02, t0, 21)
    x0 = xr[:, 0] + W.noise_for(0, B, 1)
    p = cpu.mpc_params(20, Q, R, P, DSAFE, RHO, VMAX, WMAX, DT)
    out = cpu.mpc_solve_batch(p, x0, xr, ur, W.DEFAULT_OBS, step_count=np.full(B, 10, np.int32), threads=8)
    it = out["iters"]
    cand = np.nonzero(it >= 5)[0]
    print("robots with >= 5 C-port iterations:", len(cand))
    res = []
    for b in cand:
        Hm, g, Am, cv, blo, bhi = condensed(x0[b], xr[b], ur[b], W.DEFAULT_OBS)
        S = np.zeros(Am.shape[0], bool); bf = np.zeros(40, int)
        nfix4 = None; k_conv = None; changes = []
        for k in range(1, 33):
            zc, lam = solve_sets(Hm, g, Am, cv, S, bf, blo, bhi)
            r = cv - Am @ zc
            nS = np.where(S, r > -1e-14, r > 1e-14)
            nb = bf.copy()
            for i in range(40):
                if bf[i] == 0:
                    nb[i] = 1 if zc[i] < blo[i] - 1e-13 else (2 if zc[i] > bhi[i] + 1e-13 else 0)
                elif bf[i] == 1:
                    nb[i] = 0 if lam[i] < 0 else 1
                else:
                    nb[i] = 0 if lam[i] > 0 else 2
            # box components released (fixed -> free) in this update: the cycling signature
            changes.append(int(((bf != 0) & (nb == 0)).sum()))
            if k == 4:
                nfix4 = int((bf != 0).sum())
            if (nS == S).all() and (nb == bf).all():
                k_conv = k
                break
            S, bf = nS, nb
        z_unc = np.linalg.solve(Hm, -g)
        k_pn, _ = proj_newton(Hm, g, Am, cv, blo, bhi, np.clip(z_unc, blo, bhi))
        rel_by4 = sum(changes[:4])
        res.append((it[b], k_conv or -1, nfix4 if nfix4 is not None else -1, rel_by4, k_pn))
    res = np.array(res)
    for lab, m in (("converge<=10", (res[:, 1] > 0) & (res[:, 1] <= 10)),
                   ("converge>10", res[:, 1] > 10), ("no conv 32", res[:, 1] < 0)):
        sub = res[m]
        if len(sub) == 0:
            continue
        print(f"{lab:14s} n={len(sub):5d}  fix@4 mean {sub[:,2].mean():5.1f} min {sub[:,2].min():3d}"
              f"  released-by-4 mean {sub[:,3].mean():4.1f}  PN-from-unc mean {np.abs(sub[:,4]).mean():4.1f}"
              f" max {np.abs(sub[:,4]).max()}")
    for th in (8, 12, 16, 20, 24):
        flag = res[:, 2] >= th
        print(f"fix@4 >= {th}: flags {flag.sum():5d}; of those converge<=10: "
              f"{((res[:,1] > 0) & (res[:,1] <= 10) & flag).sum()}, hard(>10 or none): "
              f"{(((res[:,1] > 10) | (res[:,1] < 0)) & flag).sum()} of {((res[:,1] > 10) | (res[:,1] < 0)).sum()}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "alt":
        study_alternatives()
    elif len(sys.argv) > 1 and sys.argv[1] == "classify":
        study_classify()
    else:
        main()
