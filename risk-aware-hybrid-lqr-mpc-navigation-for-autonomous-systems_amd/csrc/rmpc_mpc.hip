// rmpc_mpc.hip -- batched MPC QP solve on CDNA4 (gfx950).
//
// Replaces MPCController.solve_with_ltv (mpc_controller.py:345-522) and
// MPCController.solve (mpc_controller.py:150-314) for B independent robots.
//
// Mapping: one lane owns one robot.  The QP is the reference's, with the slacks
// eliminated analytically (min_{s>=0} rho s^2 s.t. s >= r  ==  rho max(0, r)^2), so
// each robot solves   min F(u)  s.t.  lo <= u <= hi   over its (blocked) inputs, F a
// strongly convex piecewise quadratic.  The solver is a primal-dual active set
// (semismooth Newton) method whose every iteration is ONE block Riccati recursion
// over the horizon (O(N) work, 3x3 / 2x2 algebra in registers, the LTV linearisation
// of linearization.py:190-225 fused in), followed by a projected Newton phase with
// Armijo backtracking for the rare instances where plain PDAS cycles.  A robot is
// certified OPTIMAL when its active sets reproduce themselves (exact KKT point).
//
// Per-robot state lives in a per-wave tiled workspace (64 lanes x record), so every
// load/store of a wave is a single coalesced 512-byte row.
#include "rmpc_device.h"
#include "rmpc_internal.h"
#include "rmpc_riccati.h"

#include <atomic>

namespace rmpc {

template <typename T>
struct MpcArgs {
    MpcDevParams prm;
    MpcLayout L;
    int64_t B;
    const double *x0, *x_refs, *u_refs, *obstacles;
    int ref_rows, uref_rows, n_obs;
    int32_t *step_count;
    double *u0, *u_seq, *x_pred, *cost;
    int32_t *status, *iters;
    uint8_t *slack_used;
    T *ws;
    const int32_t *index;   // optional robot index list (hybrid compaction); NULL = identity
    const int32_t *count;   // device-side length of `index`
    // the calling context's other list-counter set (RMPC_COUNT_WORDS words), zeroed by
    // workgroup 0 for the context's next call, which takes it (may be null)
    int32_t *zero_next;
    // leftover-list launches: the list length this launch saw, written to a host-mapped word
    // (the next launch's grid; may be null)
    int32_t *count_out;
};

// ------------------------------------------------------------------------------ setup
// LTV problem data (mpc_controller.py:366-468): np.unwrap of the reference heading,
// x0 heading moved into the reference branch, per-step linearisation, blocked box,
// linearised obstacle half-spaces (kept when dist > 0.01).
template <typename T>
__device__ void setup_ltv(const MpcArgs<T> &a, const WaveTile<T> &w, int64_t b, T x0adj[3]) {
    const MpcLayout &L = a.L;
    const MpcDevParams &p = a.prm;
    const int N = L.N;
    const double *xr = a.x_refs + ref_row0(a.prm.ref_off, b, a.ref_rows) * 3;
    const double *ur = a.u_refs + ref_row0(a.prm.ref_off, b, a.uref_rows) * 2;
    double corr = 0.0, prev = xr[2];
    double th0 = xr[2];
    for (int k = 0; k <= N; k++) {
        double th = xr[3 * k + 2];
        if (k > 0) {                                   // np.unwrap (numpy 2.x formula)
            double dd = th - prev;
            double ddmod = np_mod(dd + RMPC_PI, 2.0 * RMPC_PI) - RMPC_PI;
            if (ddmod == -RMPC_PI && dd > 0) ddmod = RMPC_PI;
            double ph = ddmod - dd;
            if (fabs(dd) < RMPC_PI) ph = 0.0;
            corr += ph;
        }
        prev = th;
        double thu = th + corr;
        if (k < N) {
            double v = ur[2 * k];
            double vr = fabs(v) > 0.01 ? v : 0.1;     // :425
            double s, c;
            sincos(thu, &s, &c);
            w(L.A0 + k) = (T)(-vr * s * p.dt);
            w(L.A1 + k) = (T)(vr * c * p.dt);
            w(L.B0 + k) = (T)(c * p.dt);
            w(L.B1 + k) = (T)(s * p.dt);
            w(L.US0 + k) = (T)ur[2 * k];
            w(L.US1 + k) = (T)ur[2 * k + 1];
            const double px = xr[3 * k], py = xr[3 * k + 1];
            for (int o = 0; o < L.no; o++) {          // :439-468
                const double ox = a.obstacles[3 * o], oy = a.obstacles[3 * o + 1];
                const double ddx = px - ox, ddy = py - oy;
                const double dist = sqrt(ddx * ddx + ddy * ddy);
                const int idx = k * L.no + o;
                if (dist > 0.01) {                     // soft (slack) or hard row alike
                    const double nx = ddx / dist, ny = ddy / dist;
                    const double safe = p.d_safe + a.obstacles[3 * o + 2];
                    w(L.HN0 + idx) = (T)nx;
                    w(L.HN1 + idx) = (T)ny;
                    w(L.HB + idx) = (T)(safe - (nx * (px - ox) + ny * (py - oy)));
                } else {                               // row absent: never active
                    w(L.HN0 + idx) = (T)0;
                    w(L.HN1 + idx) = (T)0;
                    w(L.HB + idx) = (T)-1e30;
                }
                w(L.HBO + idx) = w(L.HB + idx);
                w(L.HACT + idx) = (T)0;
            }
        }
        if (k == 0) th0 = thu;
    }
    for (int k = 0; k <= N; k++) {
        w(L.XS0 + k) = (T)0;
        w(L.XS1 + k) = (T)0;
        w(L.XS2 + k) = (T)0;
    }
    for (int j = 0; j < L.nb; j++) {                   // :431-436, intersected over the block
        double lo0 = -1e300, hi0 = 1e300, lo1 = -1e300, hi1 = 1e300;
        for (int k = j * L.bs; k < (j + 1) * L.bs && k < N; k++) {
            lo0 = fmax(lo0, -p.v_max - ur[2 * k]);
            hi0 = fmin(hi0, p.v_max - ur[2 * k]);
            lo1 = fmax(lo1, -p.omega_max - ur[2 * k + 1]);
            hi1 = fmin(hi1, p.omega_max - ur[2 * k + 1]);
        }
        w(L.LO0 + j) = (T)lo0;
        w(L.HI0 + j) = (T)hi0;
        w(L.LO1 + j) = (T)lo1;
        w(L.HI1 + j) = (T)hi1;
        w(L.BF0 + j) = (T)0;
        w(L.BF1 + j) = (T)0;
    }
    // x0 heading into the reference branch (:397-401); dx0 = x0_adj - x_ref_unwrapped[0]
    const double *x0 = a.x0 + 3 * b;
    double x0a = th0 + wrap_pi(x0[2] - th0);
    x0adj[0] = (T)(x0[0] - xr[0]);
    x0adj[1] = (T)(x0[1] - xr[1]);
    x0adj[2] = (T)(x0a - th0);
}

// LTI problem data (mpc_controller.py:172-270): padding, ONE linearisation at the first
// reference, absolute state with a tracking cost, |u| box.
template <typename T>
__device__ void setup_lti(const MpcArgs<T> &a, const WaveTile<T> &w, int64_t b, T x0v[3]) {
    const MpcLayout &L = a.L;
    const MpcDevParams &p = a.prm;
    const int N = L.N;
    const double *xr = a.x_refs + ref_row0(a.prm.ref_off, b, a.ref_rows) * 3;
    const double *ur = a.u_refs + ref_row0(a.prm.ref_off, b, a.uref_rows) * 2;
    double v = ur[0];
    double vr = fabs(v) > 0.01 ? v : 0.1;             // :186
    double s, c;
    sincos(xr[2], &s, &c);
    for (int k = 0; k <= N; k++) {
        const int kr = k < a.ref_rows ? k : a.ref_rows - 1;
        const double px = xr[3 * kr], py = xr[3 * kr + 1];
        w(L.XS0 + k) = (T)px;
        w(L.XS1 + k) = (T)py;
        w(L.XS2 + k) = (T)xr[3 * kr + 2];
        if (k < N) {
            w(L.A0 + k) = (T)(-vr * s * p.dt);
            w(L.A1 + k) = (T)(vr * c * p.dt);
            w(L.B0 + k) = (T)(c * p.dt);
            w(L.B1 + k) = (T)(s * p.dt);
            w(L.US0 + k) = (T)0;
            w(L.US1 + k) = (T)0;
            w(L.LO0 + k) = (T)-p.v_max;
            w(L.HI0 + k) = (T)p.v_max;
            w(L.LO1 + k) = (T)-p.omega_max;
            w(L.HI1 + k) = (T)p.omega_max;
            w(L.BF0 + k) = (T)0;
            w(L.BF1 + k) = (T)0;
            for (int o = 0; o < L.no; o++) {
                const double ox = a.obstacles[3 * o], oy = a.obstacles[3 * o + 1];
                const double ddx = px - ox, ddy = py - oy;
                const double dist = sqrt(ddx * ddx + ddy * ddy);
                const int idx = k * L.no + o;
                if (dist > 0.01) {
                    const double nx = ddx / dist, ny = ddy / dist;
                    w(L.HN0 + idx) = (T)nx;
                    w(L.HN1 + idx) = (T)ny;
                    w(L.HB + idx) = (T)(p.d_safe + a.obstacles[3 * o + 2] + nx * ox + ny * oy);
                } else {
                    w(L.HN0 + idx) = (T)0;
                    w(L.HN1 + idx) = (T)0;
                    w(L.HB + idx) = (T)-1e30;
                }
                w(L.HBO + idx) = w(L.HB + idx);
                w(L.HACT + idx) = (T)0;
            }
        }
    }
    const double *x0 = a.x0 + 3 * b;
    x0v[0] = (T)x0[0];
    x0v[1] = (T)x0[1];
    x0v[2] = (T)x0[2];
}

// ------------------------------------------------------------------------------ Riccati
// Backward block Riccati recursion for the current active sets, then the forward pass.
// mode 0 (PDAS): apply the set-update rule in place; mode 1: only test it.
// Returns 1 if the sets (would) change.  Writes U (per block) and X (per step).
template <typename T>
__device__ int riccati_pass(const MpcDevParams &p, const MpcLayout &L, const WaveTile<T> &w,
                            const T x0[3], int mode) {
    const int N = L.N, nb = L.nb, no = L.no, bs = L.bs;
    const T dt = (T)p.dt, rho = (T)p.rho;
    const T Q0 = (T)p.Q[0], Q1 = (T)p.Q[1], Q2 = (T)p.Q[2];
    const T R0 = (T)p.R[0], R1 = (T)p.R[1];
    // V(x) = x'Px + 2p'x, terminal
    RicV<T> V;
    V.P00 = (T)p.P[0]; V.P01 = 0; V.P02 = 0; V.P11 = (T)p.P[1]; V.P12 = 0; V.P22 = (T)p.P[2];
    V.p0 = -(T)p.P[0] * w(L.XS0 + N); V.p1 = -(T)p.P[1] * w(L.XS1 + N); V.p2 = -(T)p.P[2] * w(L.XS2 + N);
    for (int j = nb - 1; j >= 0; j--) {
        const int k0 = j * bs;
        const int k1 = min(k0 + bs, N);
        RicW<T> W = ric_open(V);
        for (int k = k1 - 1; k >= k0; k--) {
            T q00 = Q0, q01 = 0, q11 = Q1;
            T qv0 = -Q0 * w(L.XS0 + k), qv1 = -Q1 * w(L.XS1 + k), qv2 = -Q2 * w(L.XS2 + k);
            if (k > 0) {
                for (int o = 0; o < no; o++) {
                    const int idx = k * no + o;
                    if (w(L.HACT + idx) != (T)0) {
                        const T n0 = w(L.HN0 + idx), n1 = w(L.HN1 + idx), hb = w(L.HB + idx);
                        q00 += rho * n0 * n0;
                        q01 += rho * n0 * n1;
                        q11 += rho * n1 * n1;
                        qv0 -= rho * hb * n0;
                        qv1 -= rho * hb * n1;
                    }
                }
            }
            ric_step(W, w(L.A0 + k), w(L.A1 + k), w(L.B0 + k), w(L.B1 + k), dt, q00, q01, q11, Q2,
                     qv0, qv1, qv2, R0, R1, R0 * w(L.US0 + k), R1 * w(L.US1 + k));
        }
        const int bf0 = (int)w(L.BF0 + j), bf1 = (int)w(L.BF1 + j);
        const T uc0 = bf0 == 1 ? w(L.LO0 + j) : w(L.HI0 + j);
        const T uc1 = bf1 == 1 ? w(L.LO1 + j) : w(L.HI1 + j);
        T G[8];
        V = ric_block(W, bf0, bf1, uc0, uc1, G);
#pragma unroll
        for (int i = 0; i < 8; i++) w(L.K + i * nb + j) = G[i];
    }
    // ---- forward pass + set update
    const T eps_h = SetTol<T>::hinge, eps_b = SetTol<T>::box;
    int changed = 0;
    T x0s = x0[0], x1s = x0[1], x2s = x0[2];
    for (int j = 0; j < nb; j++) {
        const int bf0 = (int)w(L.BF0 + j), bf1 = (int)w(L.BF1 + j);
        const int G = L.K;
        const T r00 = w(G + 0 * nb + j), r01 = w(G + 1 * nb + j), r02 = w(G + 2 * nb + j);
        const T r10 = w(G + 3 * nb + j), r11 = w(G + 4 * nb + j), r12 = w(G + 5 * nb + j);
        const T c0 = w(G + 6 * nb + j), c1 = w(G + 7 * nb + j);
        const T e0 = r00 * x0s + r01 * x1s + r02 * x2s + c0;
        const T e1 = r10 * x0s + r11 * x1s + r12 * x2s + c1;
        const T lo0 = w(L.LO0 + j), hi0 = w(L.HI0 + j), lo1 = w(L.LO1 + j), hi1 = w(L.HI1 + j);
        const T u0v = bf0 == 0 ? e0 : (bf0 == 1 ? lo0 : hi0);
        const T u1v = bf1 == 0 ? e1 : (bf1 == 1 ? lo1 : hi1);
        // box set update (lambda = e when fixed)
        const int ns0 = box_rule(bf0, e0, lo0, hi0, eps_b), ns1 = box_rule(bf1, e1, lo1, hi1, eps_b);
        if (ns0 != bf0 || ns1 != bf1) {
            changed = 1;
            if (mode == 0) { w(L.BF0 + j) = (T)ns0; w(L.BF1 + j) = (T)ns1; }
        }
        w(L.U0 + j) = u0v;
        w(L.U1 + j) = u1v;
        const int k0 = j * bs, k1 = min(k0 + bs, N);
        for (int k = k0; k < k1; k++) {
            w(L.X0 + k) = x0s;
            w(L.X1 + k) = x1s;
            w(L.X2 + k) = x2s;
            if (k > 0) {
                for (int o = 0; o < no; o++) {
                    const int idx = k * no + o;
                    const T r = w(L.HB + idx) - w(L.HN0 + idx) * x0s - w(L.HN1 + idx) * x1s;
                    const int act = w(L.HACT + idx) != (T)0;
                    const int na = act ? (r > -eps_h) : (r > eps_h);
                    if (na != act) {
                        changed = 1;
                        if (mode == 0) w(L.HACT + idx) = (T)na;
                    }
                }
            }
            const T n0 = x0s + w(L.A0 + k) * x2s + w(L.B0 + k) * u0v;
            const T n1 = x1s + w(L.A1 + k) * x2s + w(L.B1 + k) * u0v;
            const T n2 = x2s + dt * u1v;
            x0s = n0; x1s = n1; x2s = n2;
        }
    }
    w(L.X0 + N) = x0s;
    w(L.X1 + N) = x1s;
    w(L.X2 + N) = x2s;
    return changed;
}

// F at u(alpha) = clamp(Z + alpha (U - Z)) (or at Z when alpha < 0); writes X and, with
// `commit`, the evaluated point into Z.  gd accumulates g . (u(alpha) - Z).
template <typename T>
__device__ T simulate_F(const MpcDevParams &p, const MpcLayout &L, const WaveTile<T> &w,
                        const T x0[3], T alpha, T *gd, int commit) {
    const int N = L.N, no = L.no, bs = L.bs;
    const T dt = (T)p.dt, rho = (T)p.rho;
    T x0s = x0[0], x1s = x0[1], x2s = x0[2];
    T F = 0, gdd = 0;
    T u0v = 0, u1v = 0;
    for (int k = 0; k < N; k++) {
        const int j = k / bs;
        if (k == j * bs) {
            const T z0 = w(L.Z0 + j), z1 = w(L.Z1 + j);
            if (alpha < (T)0) {
                u0v = z0;
                u1v = z1;
            } else {
                u0v = clampv(z0 + alpha * (w(L.U0 + j) - z0), w(L.LO0 + j), w(L.HI0 + j));
                u1v = clampv(z1 + alpha * (w(L.U1 + j) - z1), w(L.LO1 + j), w(L.HI1 + j));
                gdd += w(L.G0 + j) * (u0v - z0) + w(L.G1 + j) * (u1v - z1);
                if (commit) { w(L.Z0 + j) = u0v; w(L.Z1 + j) = u1v; }
            }
        }
        w(L.X0 + k) = x0s;
        w(L.X1 + k) = x1s;
        w(L.X2 + k) = x2s;
        const T e0 = x0s - w(L.XS0 + k), e1 = x1s - w(L.XS1 + k), e2 = x2s - w(L.XS2 + k);
        F += (T)p.Q[0] * e0 * e0 + (T)p.Q[1] * e1 * e1 + (T)p.Q[2] * e2 * e2;
        const T uu0 = u0v + w(L.US0 + k), uu1 = u1v + w(L.US1 + k);
        F += (T)p.R[0] * uu0 * uu0 + (T)p.R[1] * uu1 * uu1;
        for (int o = 0; o < no; o++) {
            const int idx = k * no + o;
            const T r = w(L.HB + idx) - w(L.HN0 + idx) * x0s - w(L.HN1 + idx) * x1s;
            if (r > (T)0) F += rho * r * r;
        }
        const T n0 = x0s + w(L.A0 + k) * x2s + w(L.B0 + k) * u0v;
        const T n1 = x1s + w(L.A1 + k) * x2s + w(L.B1 + k) * u0v;
        const T n2 = x2s + dt * u1v;
        x0s = n0; x1s = n1; x2s = n2;
    }
    w(L.X0 + N) = x0s;
    w(L.X1 + N) = x1s;
    w(L.X2 + N) = x2s;
    const T e0 = x0s - w(L.XS0 + N), e1 = x1s - w(L.XS1 + N), e2 = x2s - w(L.XS2 + N);
    F += (T)p.P[0] * e0 * e0 + (T)p.P[1] * e1 * e1 + (T)p.P[2] * e2 * e2;
    if (gd) *gd = gdd;
    return F;
}

// adjoint gradient dF/du at (Z, X) into G
template <typename T>
__device__ void gradient(const MpcDevParams &p, const MpcLayout &L, const WaveTile<T> &w) {
    const int N = L.N, no = L.no, bs = L.bs;
    const T rho = (T)p.rho;
    T l0 = (T)2 * (T)p.P[0] * (w(L.X0 + N) - w(L.XS0 + N));
    T l1 = (T)2 * (T)p.P[1] * (w(L.X1 + N) - w(L.XS1 + N));
    T l2 = (T)2 * (T)p.P[2] * (w(L.X2 + N) - w(L.XS2 + N));
    T g0 = 0, g1 = 0;
    for (int k = N - 1; k >= 0; k--) {
        const int j = k / bs;
        g0 += (T)2 * (T)p.R[0] * (w(L.Z0 + j) + w(L.US0 + k)) + w(L.B0 + k) * l0 + w(L.B1 + k) * l1;
        g1 += (T)2 * (T)p.R[1] * (w(L.Z1 + j) + w(L.US1 + k)) + (T)p.dt * l2;
        if (k == j * bs) {
            w(L.G0 + j) = g0;
            w(L.G1 + j) = g1;
            g0 = 0;
            g1 = 0;
        }
        const T x0s = w(L.X0 + k), x1s = w(L.X1 + k), x2s = w(L.X2 + k);
        T d0 = (T)2 * (T)p.Q[0] * (x0s - w(L.XS0 + k));
        T d1 = (T)2 * (T)p.Q[1] * (x1s - w(L.XS1 + k));
        const T d2 = (T)2 * (T)p.Q[2] * (x2s - w(L.XS2 + k));
        for (int o = 0; o < no; o++) {
            const int idx = k * no + o;
            const T n0 = w(L.HN0 + idx), n1 = w(L.HN1 + idx);
            const T r = w(L.HB + idx) - n0 * x0s - n1 * x1s;
            if (r > (T)0) {
                d0 -= (T)2 * rho * r * n0;
                d1 -= (T)2 * rho * r * n1;
            }
        }
        const T nl2 = d2 + w(L.A0 + k) * l0 + w(L.A1 + k) * l1 + l2;
        l0 = d0 + l0;
        l1 = d1 + l1;
        l2 = nl2;
    }
}

// signature of the active sets (PDAS cycle detection; same hash as the fast kernel)
template <typename T>
__device__ uint64_t set_signature(const MpcLayout &L, const WaveTile<T> &w) {
    uint64_t h = 1469598103934665603ull;
    for (int k = 0; k < L.N; k++) {
        uint32_t word = 0;
        for (int o = 0; o < L.no; o++) word |= (uint32_t)(w(L.HACT + k * L.no + o) != (T)0) << o;
        h = (h ^ (uint64_t)word) * 1099511628211ull;
    }
    for (int j = 0; j < L.nb; j++)
        h = (h ^ (uint64_t)((int)w(L.BF0 + j) | ((int)w(L.BF1 + j) << 2))) * 1099511628211ull;
    return h;
}

// One solve of the (soft, or shifted-hard) piecewise-quadratic problem for the robot's
// current record: PDAS from the stored active sets, then projected Newton + Armijo.
// `it` counts Riccati solves; stops at `max_iter`.  Returns 1 if certified (exact KKT).
template <typename T>
__device__ int solve_inner(const MpcDevParams &p, const MpcLayout &L, const WaveTile<T> &w,
                           const T x0[3], int &it, const int max_iter) {
    int cert = 0;
    const int it0 = it;
    // ---- phase 1: primal-dual active set (capped; a repeated signature = cycling)
    uint64_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    for (; it < max_iter && it - it0 < RMPC_PDAS_ITERS;) {
        it++;
        if (!riccati_pass(p, L, w, x0, 0)) { cert = 1; break; }
        const uint64_t sig = set_signature(L, w);
        if (sig == h0 || sig == h1 || sig == h2 || sig == h3) break;
        h3 = h2; h2 = h1; h1 = h0; h0 = sig;
    }
    if (!cert && it < max_iter) {
        // ---- phase 2: projected Newton + Armijo from the projected last iterate
        for (int j = 0; j < L.nb; j++) {
            w(L.Z0 + j) = clampv(w(L.U0 + j), w(L.LO0 + j), w(L.HI0 + j));
            w(L.Z1 + j) = clampv(w(L.U1 + j), w(L.LO1 + j), w(L.HI1 + j));
        }
        T F = simulate_F(p, L, w, x0, (T)-1, (T *)nullptr, 0);
        int stalled = 0;
        while (it < max_iter) {
            gradient(p, L, w);
            T wmax = 0;
            for (int j = 0; j < L.nb; j++) {
                const T z0 = w(L.Z0 + j), z1 = w(L.Z1 + j);
                wmax = fmax(wmax, fabs(z0 - clampv(z0 - w(L.G0 + j), w(L.LO0 + j), w(L.HI0 + j))));
                wmax = fmax(wmax, fabs(z1 - clampv(z1 - w(L.G1 + j), w(L.LO1 + j), w(L.HI1 + j))));
            }
            const T eps = fmin(SetTol<T>::pn, wmax);
            for (int k = 1; k < L.N; k++)
                for (int o = 0; o < L.no; o++) {
                    const int idx = k * L.no + o;
                    const T r = w(L.HB + idx) - w(L.HN0 + idx) * w(L.X0 + k) - w(L.HN1 + idx) * w(L.X1 + k);
                    w(L.HACT + idx) = r > (T)0 ? (T)1 : (T)0;
                }
            for (int j = 0; j < L.nb; j++) {
                const T z0 = w(L.Z0 + j), z1 = w(L.Z1 + j), g0 = w(L.G0 + j), g1 = w(L.G1 + j);
                w(L.BF0 + j) = (z0 <= w(L.LO0 + j) + eps && g0 > 0) ? (T)1
                               : ((z0 >= w(L.HI0 + j) - eps && g0 < 0) ? (T)2 : (T)0);
                w(L.BF1 + j) = (z1 <= w(L.LO1 + j) + eps && g1 > 0) ? (T)1
                               : ((z1 >= w(L.HI1 + j) - eps && g1 < 0) ? (T)2 : (T)0);
            }
            it++;
            if (!riccati_pass(p, L, w, x0, 1)) { cert = 1; break; }
            T alpha = 1, Ft = F, gd = 0;
            int acc = 0;
            for (int ls = 0; ls < 40; ls++) {
                Ft = simulate_F(p, L, w, x0, alpha, &gd, 0);
                if (Ft <= F + (T)1e-4 * gd) { acc = 1; break; }
                alpha *= (T)0.5;
            }
            if (!acc) { stalled = 1; break; }
            simulate_F(p, L, w, x0, alpha, &gd, 1);   // commit Z, X
            F = Ft;
        }
        if (!cert) {
            // best box-feasible point: Z (re-simulate so X matches)
            simulate_F(p, L, w, x0, (T)-1, (T *)nullptr, 0);
            for (int j = 0; j < L.nb; j++) { w(L.U0 + j) = w(L.Z0 + j); w(L.U1 + j) = w(L.Z1 + j); }
        }
        (void)stalled;
    }
    return cert;
}

// Hard half-spaces (use_soft_constraints=False, mpc_controller.py:383-386 / :197-200 with the
// rows of :439-468 / :238-270 as plain inequalities): augmented Lagrangian over the same
// solver.  Each outer round solves the soft problem with penalty rho_h and the rows shifted
// by s_i >= 0 (HB = HBO + s), then s_i <- max(0, r_i + s_i).  A fixed point is exactly the
// KKT point of the hard QP (multipliers 2 rho_h s_i); rows at k = 0 act on the fixed dx_0
// and, when violated, make the QP infeasible -- the reference's solver then reports
// infeasibility and the fallback law applies (:521-522), as it does here when the shifts
// do not converge.
template <typename T> struct HardAlm;
template <> struct HardAlm<double> {
    static constexpr double rho = 1e6, tol = 1e-12, k0_tol = 1e-9;
    static constexpr int outer = 60;
};
template <> struct HardAlm<float> {
    static constexpr float rho = 1e3f, tol = 1e-5f, k0_tol = 1e-5f;
    static constexpr int outer = 60;
};

template <typename T>
__device__ int solve_hard(const MpcDevParams &p, const MpcLayout &L, const WaveTile<T> &w,
                          const T x0[3], int &it, const int max_iter) {
    for (int o = 0; o < L.no; o++)        // k = 0 rows: fixed state, feasibility is decided
        if (w(L.HB + o) - w(L.HN0 + o) * x0[0] - w(L.HN1 + o) * x0[1] > HardAlm<T>::k0_tol) return 0;
    MpcDevParams ph = p;
    ph.rho = HardAlm<T>::rho;
    for (int round = 0; round < HardAlm<T>::outer; round++) {
        if (!solve_inner(ph, L, w, x0, it, it + max_iter)) return 0;
        T viol = 0;
        for (int k = 1; k < L.N; k++)
            for (int o = 0; o < L.no; o++) {
                const int idx = k * L.no + o;
                const T hbo = w(L.HBO + idx);
                if (hbo < (T)-1e29) continue;                   // row absent (dist <= 0.01)
                const T sh = w(L.HB + idx) - hbo;
                const T rs = w(L.HB + idx) - w(L.HN0 + idx) * w(L.X0 + k) - w(L.HN1 + idx) * w(L.X1 + k);
                const T ns = rs > (T)0 ? rs : (T)0;
                viol = fmax(viol, fabs(ns - sh));
                w(L.HB + idx) = hbo + ns;
            }
        if (viol <= HardAlm<T>::tol) return 1;
    }
    return 0;
}

// USE_LDS: the whole robot record lives in LDS (workgroup = blockDim lanes, sized by the
// host so the records fit in 160 KiB) -- used for the small retry lists, where latency
// per robot, not occupancy, decides the launch time.
template <typename T, bool USE_LDS>
__device__ __forceinline__ void mpc_solve_one(const MpcArgs<T> &a, int64_t t) {
    const int64_t b = a.index ? (int64_t)a.index[t] : t;
    const MpcLayout &L = a.L;
    const MpcDevParams &p = a.prm;
    extern __shared__ double lds_ws[];
    WaveTile<T> w = USE_LDS
        ? WaveTile<T>{(T *)lds_ws, (int)threadIdx.x, (int)blockDim.x}
        : WaveTile<T>{a.ws + (size_t)(t / RMPC_WAVE) * (size_t)L.REC * RMPC_WAVE, (int)(t % RMPC_WAVE),
                      RMPC_WAVE};
    const int ltv = p.ltv;
    T x0[3];
    if (ltv) setup_ltv(a, w, b, x0);
    else setup_lti(a, w, b, x0);
    int finite = isfinite((double)(x0[0] + x0[1] + x0[2]));
    for (int k = 0; k < L.N && finite; k++)
        finite = isfinite((double)(w(L.A0 + k) + w(L.A1 + k) + w(L.US0 + k) + w(L.US1 + k) +
                                   w(L.XS0 + k) + w(L.XS1 + k) + w(L.XS2 + k)));
    int cert = 0, it = 0;
    const int max_iter = p.max_iter;
    if (finite) {
        if (!p.soft && L.no > 0) cert = solve_hard(p, L, w, x0, it, max_iter);
        else cert = solve_inner(p, L, w, x0, it, max_iter);
        if (!p.soft && L.no > 0 && !cert) finite = 0;        // infeasible / unconverged -> fallback
    }
    // ---- outputs
    const int N = L.N;
    const double *xr = a.x_refs + ref_row0(a.prm.ref_off, b, a.ref_rows) * 3;
    const double *ur = a.u_refs + ref_row0(a.prm.ref_off, b, a.uref_rows) * 2;
    double J = 0;
    int used = 0;
    if (finite && it > 0) {
        for (int k = 0; k <= N; k++) {
            const double *Wd = k < N ? p.Q : p.P;
            const double e0 = (double)(w(L.X0 + k) - w(L.XS0 + k));
            const double e1 = (double)(w(L.X1 + k) - w(L.XS1 + k));
            const double e2 = (double)(w(L.X2 + k) - w(L.XS2 + k));
            J += Wd[0] * e0 * e0 + Wd[1] * e1 * e1 + Wd[2] * e2 * e2;
            if (k < N) {
                const int j = k / L.bs;
                const double uu0 = (double)(w(L.U0 + j) + w(L.US0 + k));
                const double uu1 = (double)(w(L.U1 + j) + w(L.US1 + k));
                J += p.R[0] * uu0 * uu0 + p.R[1] * uu1 * uu1;
                for (int o = 0; o < L.no; o++) {
                    const int idx = k * L.no + o;
                    const double r = (double)(w(L.HB + idx) - w(L.HN0 + idx) * w(L.X0 + k) -
                                              w(L.HN1 + idx) * w(L.X1 + k));
                    if (r > 0 && p.soft) {                  // hard rows carry no slack term
                        J += p.rho * r * r;
                        if (r > 1e-6) used = 1;             // :485 slack.value > 1e-6
                    }
                }
            }
        }
    }
    const int ok = finite && it > 0 && isfinite(J);
    if (ok) {
        // ltv: x_pred = x_refs + dx (NOT unwrapped, :497), u = u_refs + du (:498)
        double uc0 = 0, uc1 = 0;
        for (int k = 0; k < N; k++) {
            const int j = k / L.bs;
            double v0 = (double)w(L.U0 + j) + (ltv ? ur[2 * k] : 0.0);
            double v1 = (double)w(L.U1 + j) + (ltv ? ur[2 * k + 1] : 0.0);
            if (k == 0) {
                if (ltv) {
                    const int sc = a.step_count ? a.step_count[b] : 0;
                    if (sc < p.ramp_up_steps) {                    // :502-505
                        const double lim = p.omega_max * ((double)(sc + 1) / (double)p.ramp_up_steps);
                        v1 = clampv(v1, -lim, lim);
                    }
                    if (a.step_count) a.step_count[b] = sc + 1;    // :507
                }
                uc0 = v0;
                uc1 = v1;
            }
            if (a.u_seq) {
                a.u_seq[((size_t)b * N + k) * 2] = v0;
                a.u_seq[((size_t)b * N + k) * 2 + 1] = v1;
            }
        }
        if (a.x_pred)
            for (int k = 0; k <= N; k++) {
                double *xp = a.x_pred + ((size_t)b * (N + 1) + k) * 3;
                xp[0] = (double)w(L.X0 + k) + (ltv ? xr[3 * k] : 0.0);
                xp[1] = (double)w(L.X1 + k) + (ltv ? xr[3 * k + 1] : 0.0);
                xp[2] = (double)w(L.X2 + k) + (ltv ? xr[3 * k + 2] : 0.0);
            }
        a.u0[2 * b] = uc0;
        a.u0[2 * b + 1] = uc1;
        if (a.cost) a.cost[b] = J;
        if (a.slack_used) a.slack_used[b] = (uint8_t)used;
        a.status[b] = cert ? RMPC_OPTIMAL : RMPC_OPTIMAL_INACCURATE;
    } else {
        // fallback law mpc_controller.py:316-343 (LTI: padded row 0 == row 0)
        const double *x0p = a.x0 + 3 * b;
        const double e0 = x0p[0] - xr[0], e2 = wrap_pi(x0p[2] - xr[2]);
        const double v0 = clampv(ur[0] - e0, -p.v_max, p.v_max);
        const double v1 = clampv(ur[1] - 0.5 * e2, -p.omega_max, p.omega_max);
        a.u0[2 * b] = v0;
        a.u0[2 * b + 1] = v1;
        if (a.u_seq)
            for (int k = 0; k < N; k++) {
                a.u_seq[((size_t)b * N + k) * 2] = v0;
                a.u_seq[((size_t)b * N + k) * 2 + 1] = v1;
            }
        if (a.x_pred)
            for (int k = 0; k <= N; k++)
                for (int i = 0; i < 3; i++) a.x_pred[((size_t)b * (N + 1) + k) * 3 + i] = x0p[i];
        if (a.cost) a.cost[b] = INFINITY;
        if (a.slack_used) a.slack_used[b] = 0;
        a.status[b] = RMPC_FALLBACK;
    }
    if (a.iters) a.iters[b] = it;
}

#define GENERIC_GRID_MIN 16
// USE_LDS (the leftover lists after the tails): a grid sized from the list lengths this launch
// site saw before, at least GENERIC_GRID_MIN workgroups, looping over the list -- an empty or
// short list (the usual few robots) does not dispatch capacity / lanes workgroups that each
// hold an LDS slot only to exit, and a long one (non-finite inputs, many cycling robots) is not
// left to a few workgroups
template <typename T, bool USE_LDS>
__global__ __launch_bounds__(256) void mpc_solve_kernel(MpcArgs<T> a) {
    RMPC_WLOG_BEGIN
    const int64_t nrob = a.index ? (int64_t)*a.count : a.B;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a.zero_next && t0 == 0)
        for (int i = 0; i < RMPC_COUNT_WORDS; i++) a.zero_next[i] = 0;
    if (a.count_out && t0 == 0) __hip_atomic_store(a.count_out, (int32_t)nrob, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if constexpr (USE_LDS) {
        for (int64_t t = t0; t < nrob; t += (int64_t)gridDim.x * blockDim.x) mpc_solve_one<T, true>(a, t);
    } else {
        if (t0 < nrob) mpc_solve_one<T, false>(a, t0);
    }
    RMPC_WLOG_END(WL_SOLVE)
}

}  // namespace rmpc

// ------------------------------------------------------------------------------ launcher
using namespace rmpc;
RMPC_WLOG_SETTER(rmpc_wlog_set_solve)

MpcLayout rmpc_mpc_layout(int N, int bs, int no) {
    MpcLayout L;
    L.N = N;
    L.bs = bs;
    L.nb = (N + bs - 1) / bs;
    L.no = no;
    int o = 0;
    auto take = [&](int n) { int r = o; o += n; return r; };
    L.A0 = take(N); L.A1 = take(N); L.B0 = take(N); L.B1 = take(N);
    L.US0 = take(N); L.US1 = take(N);
    L.XS0 = take(N + 1); L.XS1 = take(N + 1); L.XS2 = take(N + 1);
    L.LO0 = take(L.nb); L.LO1 = take(L.nb); L.HI0 = take(L.nb); L.HI1 = take(L.nb);
    L.BF0 = take(L.nb); L.BF1 = take(L.nb);
    L.HN0 = take(N * no); L.HN1 = take(N * no); L.HB = take(N * no); L.HACT = take(N * no);
    L.HBO = take(N * no);
    L.K = take(8 * L.nb);
    L.X0 = take(N + 1); L.X1 = take(N + 1); L.X2 = take(N + 1);
    L.U0 = take(L.nb); L.U1 = take(L.nb);
    L.Z0 = take(L.nb); L.Z1 = take(L.nb);
    L.G0 = take(L.nb); L.G1 = take(L.nb);
    L.REC = o;
    return L;
}

// Lanes per workgroup of the LDS generic kernel (the leftover list after the tails): as many
// robots as fit one LDS slot (RMPC_LDS_SLOT) -- the list is short, and a workgroup that needs a
// whole CU's LDS starts only where every other workgroup has left (RMPC_LDS_SLOT) -- else as
// many as fit the CU.
int rmpc_mpc_lds_lanes(const MpcLayout &L) {
    const size_t per_lane = (size_t)L.REC * sizeof(double);
    int lanes = 64;
    while (lanes > 0 && (size_t)lanes * per_lane > RMPC_LDS_SLOT) lanes >>= 1;
    if (lanes > 0) return lanes;
    lanes = 64;
    while (lanes > 0 && (size_t)lanes * per_lane > 160 * 1024) lanes >>= 1;
    return lanes;
}

template <typename T>
static hipError_t launch_generic(const MpcDevParams &prm, const MpcLayout &L, int64_t B,
                               const double *x0, const double *x_refs, int ref_rows,
                               const double *u_refs, int uref_rows, const double *obstacles,
                               int n_obs, int32_t *step_count, double *u0, double *u_seq,
                               double *x_pred, double *cost, int32_t *status, uint8_t *slack_used,
                               int32_t *iters, void *ws, const int32_t *index,
                               const int32_t *count, hipStream_t stream, int lds_lanes, int32_t *zero_next,
                               int32_t *count_out, int prev_count) {
    MpcArgs<T> a;
    a.prm = prm;
    a.L = L;
    a.B = B;
    a.x0 = x0; a.x_refs = x_refs; a.u_refs = u_refs; a.obstacles = obstacles;
    a.ref_rows = ref_rows; a.uref_rows = uref_rows; a.n_obs = n_obs;
    a.step_count = step_count;
    a.u0 = u0; a.u_seq = u_seq; a.x_pred = x_pred; a.cost = cost;
    a.status = status; a.iters = iters; a.slack_used = slack_used;
    a.ws = (T *)ws;
    a.index = index;
    a.count = count;
    a.zero_next = zero_next;
    a.count_out = index ? count_out : nullptr;
    if (B <= 0) return hipSuccess;
    if (lds_lanes > 0) {
        const size_t lds = rmpc_lds_slot_pad((const void *)mpc_solve_kernel<T, true>, (size_t)L.REC * lds_lanes * sizeof(T));
        // the attribute is per device: one bit per device that has it (contexts on several
        // GPUs may share a process)
        static std::atomic<unsigned long long> attr_set{0};
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
        const unsigned long long bit = 1ull << (dev & 63);
        if (!(attr_set.load() & bit)) {
            hipError_t e = hipFuncSetAttribute((const void *)mpc_solve_kernel<T, true>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) return e;
            attr_set.fetch_or(bit);
        }
        static std::atomic<int> n_cu{0};
        if (!n_cu.load()) {
            int v = 0;
            if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
            n_cu.store(v);
        }
        // workgroups looping over the list, each of which has to find a free LDS slot in flight:
        // 1.5x the rounds of the longest recent list (prev_count: a decaying maximum of the
        // lengths this site's launches wrote; -1 unknown), at least GENERIC_GRID_MIN, at most
        // four per CU (RMPC_GENERIC_GRID=<workgroups>: a fixed cap, A/B).  A short guess costs
        // rounds, never results.
        int64_t blocks = (B + lds_lanes - 1) / lds_lanes, cap = GENERIC_GRID_MIN;
        if (prev_count > 0) {
            const int64_t rounds = ((int64_t)prev_count + lds_lanes - 1) / lds_lanes;
            const int64_t want = rounds + rounds / 2;
            cap = want > cap ? want : cap;
        }
        if (cap > 4 * (int64_t)n_cu.load()) cap = 4 * (int64_t)n_cu.load();
        if (const char *g = rmpc_knob("RMPC_GENERIC_GRID")) cap = atoll(g) > 0 ? atoll(g) : cap;
        if (blocks > cap) blocks = cap;
        hipLaunchKernelGGL((mpc_solve_kernel<T, true>), dim3((unsigned)blocks), dim3(lds_lanes), lds,
                           stream, a);
    } else {
        const int threads = 256;
        const int64_t blocks = (B + threads - 1) / threads;
        hipLaunchKernelGGL((mpc_solve_kernel<T, false>), dim3((unsigned)blocks), dim3(threads), 0,
                           stream, a);
    }
    return hipGetLastError();
}

hipError_t rmpc_launch_mpc_f64(const MpcDevParams &prm, const MpcLayout &L, int64_t B,
                               const double *x0, const double *x_refs, int ref_rows,
                               const double *u_refs, int uref_rows, const double *obstacles,
                               int n_obs, int32_t *step_count, double *u0, double *u_seq,
                               double *x_pred, double *cost, int32_t *status, uint8_t *slack_used,
                               int32_t *iters, void *ws, const int32_t *index,
                               const int32_t *count, hipStream_t stream, int lds_lanes, int32_t *zero_next,
                               int32_t *count_out, int prev_count) {
    return launch_generic<double>(prm, L, B, x0, x_refs, ref_rows, u_refs, uref_rows, obstacles, n_obs,
                                  step_count, u0, u_seq, x_pred, cost, status, slack_used, iters, ws, index,
                                  count, stream, lds_lanes, zero_next, count_out, prev_count);
}

// fp32 arithmetic (BASELINE config 4): same algorithm, float workspace; inputs/outputs stay fp64
hipError_t rmpc_launch_mpc_f32(const MpcDevParams &prm, const MpcLayout &L, int64_t B,
                               const double *x0, const double *x_refs, int ref_rows,
                               const double *u_refs, int uref_rows, const double *obstacles,
                               int n_obs, int32_t *step_count, double *u0, double *u_seq,
                               double *x_pred, double *cost, int32_t *status, uint8_t *slack_used,
                               int32_t *iters, void *ws, const int32_t *index,
                               const int32_t *count, hipStream_t stream, int lds_lanes, int32_t *zero_next,
                               int32_t *count_out, int prev_count) {
    return launch_generic<float>(prm, L, B, x0, x_refs, ref_rows, u_refs, uref_rows, obstacles, n_obs,
                                 step_count, u0, u_seq, x_pred, cost, status, slack_used, iters, ws, index,
                                 count, stream, lds_lanes, zero_next, count_out, prev_count);
}
