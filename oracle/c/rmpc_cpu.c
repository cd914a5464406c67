/*
 * rmpc_cpu.c -- plain-C, OpenMP restatement of the batched MPC / LQR solve path.
 *
 * TEST INFRASTRUCTURE ONLY: this is the timed CPU baseline ("port") of bench.py and
 * a second, independent check in tests/.  The product path (librmpc.so, HIP) never
 * links or calls it.
 *
 * It restates the reference's QPs (mpc_controller.py:150-314 LTI, :345-522 LTV) and
 * solves them EXACTLY with the same mathematics the GPU kernel uses:
 *   - slacks eliminated:  min_{s>=0} rho s^2  s.t. s >= r  ==  rho*max(0,r)^2
 *   - box on the (blocked) input, squared hinge on the obstacle rows
 *   - primal-dual active set iterations; each iteration solves the equality-
 *     constrained LQ problem of the current active sets with a block Riccati
 *     recursion (move blocking = a no-input propagation inside the block)
 *   - the loop stops when the active sets reproduce themselves, i.e. the KKT
 *     conditions hold exactly (to rounding).
 * The LQR gain restates lqr_controller.py:92-147 with a structure-preserving
 * doubling algorithm (SDA) for the DARE in place of SciPy's QZ method.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../../include/rmpc.h"

#define NM RMPC_MAX_HORIZON
#define OM RMPC_MAX_OBSTACLES
#define PI_D 3.141592653589793

static double wrap_pi(double a) {           /* mpc_controller.py:540-546 (while loops) */
    while (a > PI_D) a -= 2.0 * PI_D;
    while (a < -PI_D) a += 2.0 * PI_D;
    return a;
}

static double np_mod(double a, double b) {  /* numpy float mod (npy_divmod) */
    double m = fmod(a, b);
    if (m != 0.0) {
        if ((b < 0) != (m < 0)) m += b;
    } else {
        m = copysign(0.0, b);
    }
    return m;
}

static double clampd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }


/* ------------------------------------------------------------------ problem data */
typedef struct {
    int N, bs, nb, no;
    double dt, rho;
    double Qd[3], Rd[2], Pd[3];
    double a0[NM], a1[NM], b0[NM], b1[NM];   /* A_k = I + (a0,a1,0) e_theta^T, B_k = [[b0,0],[b1,0],[0,dt]] */
    double xs[NM + 1][3];                    /* state offset: cost (x - xs)'Q(x - xs)        */
    double us[NM][2];                        /* input offset: cost (u + us)'R(u + us)         */
    double lo[NM][2], hi[NM][2];             /* box on the decision input, per block          */
    double hn0[NM][OM], hn1[NM][OM], hb[NM][OM];   /* hinge row: r = hb - hn . pos(x_k)      */
    uint8_t hk[NM][OM];                      /* row kept (dist > 0.01)                         */
    double x0[3];
} Prob;

typedef struct {
    double u[NM][2];       /* decision inputs per block */
    double x[NM + 1][3];   /* state trajectory          */
    int iters, converged;
} Sol;

/* ------------------------------------------------------------------ block Riccati solve
 * hact[k][o]: hinge row active; bfix[j][c]: 0 free, 1 at lower, 2 at upper.
 * Writes u, x; lam[j][c] = d(objective)/d(u_j,c) for fixed components.                 */
static void riccati_solve(const Prob *pr, const uint8_t hact[NM][OM], const uint8_t bfix[NM][2],
                          Sol *s, double lam[NM][2]) {
    const int N = pr->N, bs = pr->bs, nb = pr->nb, no = pr->no;
    const double dt = pr->dt, rho = pr->rho;
    double K[NM][2][3], kk[NM][2], LK[NM][2][3], Lk[NM][2];
    /* value function V(x) = x'Px + 2p'x */
    double P[3][3] = {{pr->Pd[0], 0, 0}, {0, pr->Pd[1], 0}, {0, 0, pr->Pd[2]}};
    double p[3];
    for (int i = 0; i < 3; i++) p[i] = -pr->Pd[i] * pr->xs[N][i];
    for (int j = nb - 1; j >= 0; j--) {
        int k0 = j * bs, k1 = k0 + bs;
        if (k1 > N) k1 = N;
        double Wxx[3][3], Wxu[3][2] = {{0}}, Wuu[2][2] = {{0}}, wx[3], wu[2] = {0, 0};
        memcpy(Wxx, P, sizeof(Wxx));
        memcpy(wx, p, sizeof(wx));
        for (int k = k1 - 1; k >= k0; k--) {
            /* stage cost of step k in (x_k, u) */
            double Qk[3][3] = {{pr->Qd[0], 0, 0}, {0, pr->Qd[1], 0}, {0, 0, pr->Qd[2]}};
            double qk[3];
            for (int i = 0; i < 3; i++) qk[i] = -pr->Qd[i] * pr->xs[k][i];
            if (k > 0) {
                for (int o = 0; o < no; o++) {
                    if (!hact[k][o]) continue;
                    double n0 = pr->hn0[k][o], n1 = pr->hn1[k][o], b = pr->hb[k][o];
                    Qk[0][0] += rho * n0 * n0;
                    Qk[0][1] += rho * n0 * n1;
                    Qk[1][0] += rho * n0 * n1;
                    Qk[1][1] += rho * n1 * n1;
                    qk[0] -= rho * b * n0;
                    qk[1] -= rho * b * n1;
                }
            }
            double A[3][3] = {{1, 0, pr->a0[k]}, {0, 1, pr->a1[k]}, {0, 0, 1}};
            double Bm[3][2] = {{pr->b0[k], 0}, {pr->b1[k], 0}, {0, dt}};
            double WB[3][2], AtWA[3][3], nWxu[3][2], nWuu[2][2], nwx[3], nwu[2];
            for (int i = 0; i < 3; i++)
                for (int c = 0; c < 2; c++) {
                    double acc = 0;
                    for (int l = 0; l < 3; l++) acc += Wxx[i][l] * Bm[l][c];
                    WB[i][c] = acc + Wxu[i][c];          /* Wxx B + Wxu */
                }
            for (int i = 0; i < 3; i++)
                for (int l = 0; l < 3; l++) {
                    double acc = 0;
                    for (int m = 0; m < 3; m++)
                        for (int n = 0; n < 3; n++) acc += A[m][i] * Wxx[m][n] * A[n][l];
                    AtWA[i][l] = acc;
                }
            for (int i = 0; i < 3; i++)
                for (int c = 0; c < 2; c++) {
                    double acc = 0;
                    for (int m = 0; m < 3; m++) acc += A[m][i] * WB[m][c];
                    nWxu[i][c] = acc;
                }
            for (int c = 0; c < 2; c++)
                for (int d = 0; d < 2; d++) {
                    double acc = Wuu[c][d];
                    for (int m = 0; m < 3; m++)   /* R + B'(Wxx B + Wxu) + Wxu'B + Wuu */
                        acc += Bm[m][c] * WB[m][d] + Wxu[m][c] * Bm[m][d];
                    nWuu[c][d] = acc;
                }
            nWuu[0][0] += pr->Rd[0];
            nWuu[1][1] += pr->Rd[1];
            for (int i = 0; i < 3; i++) {
                double acc = 0;
                for (int m = 0; m < 3; m++) acc += A[m][i] * wx[m];
                nwx[i] = qk[i] + acc;
            }
            for (int c = 0; c < 2; c++) {
                double acc = wu[c] + pr->Rd[c] * pr->us[k][c];
                for (int m = 0; m < 3; m++) acc += Bm[m][c] * wx[m];
                nwu[c] = acc;
            }
            for (int i = 0; i < 3; i++)
                for (int l = 0; l < 3; l++) Wxx[i][l] = Qk[i][l] + AtWA[i][l];
            memcpy(Wxu, nWxu, sizeof(Wxu));
            memcpy(Wuu, nWuu, sizeof(Wuu));
            memcpy(wx, nwx, sizeof(wx));
            memcpy(wu, nwu, sizeof(wu));
        }
        /* minimise u'Mu + 2u'(Lx + g) over the free components */
        double M[2][2] = {{Wuu[0][0], 0.5 * (Wuu[0][1] + Wuu[1][0])},
                          {0.5 * (Wuu[0][1] + Wuu[1][0]), Wuu[1][1]}};
        double L[2][3], g[2] = {wu[0], wu[1]};
        for (int c = 0; c < 2; c++)
            for (int i = 0; i < 3; i++) L[c][i] = Wxu[i][c];
        int f0 = bfix[j][0] == 0, f1 = bfix[j][1] == 0;
        double uc0 = bfix[j][0] == 1 ? pr->lo[j][0] : pr->hi[j][0];
        double uc1 = bfix[j][1] == 1 ? pr->lo[j][1] : pr->hi[j][1];
        double Kj[2][3], kj[2];
        if (f0 && f1) {
            double det = M[0][0] * M[1][1] - M[0][1] * M[1][0];
            double i00 = M[1][1] / det, i01 = -M[0][1] / det, i11 = M[0][0] / det;
            for (int i = 0; i < 3; i++) {
                Kj[0][i] = -(i00 * L[0][i] + i01 * L[1][i]);
                Kj[1][i] = -(i01 * L[0][i] + i11 * L[1][i]);
            }
            kj[0] = -(i00 * g[0] + i01 * g[1]);
            kj[1] = -(i01 * g[0] + i11 * g[1]);
        } else if (f0) {
            for (int i = 0; i < 3; i++) { Kj[0][i] = -L[0][i] / M[0][0]; Kj[1][i] = 0; }
            kj[0] = -(g[0] + M[0][1] * uc1) / M[0][0];
            kj[1] = uc1;
        } else if (f1) {
            for (int i = 0; i < 3; i++) { Kj[1][i] = -L[1][i] / M[1][1]; Kj[0][i] = 0; }
            kj[1] = -(g[1] + M[1][0] * uc0) / M[1][1];
            kj[0] = uc0;
        } else {
            for (int i = 0; i < 3; i++) { Kj[0][i] = 0; Kj[1][i] = 0; }
            kj[0] = uc0;
            kj[1] = uc1;
        }
        /* multiplier maps d/du_c = 2[(MK + L)_c x + (Mk + g)_c] */
        for (int c = 0; c < 2; c++) {
            for (int i = 0; i < 3; i++)
                LK[j][c][i] = 2.0 * (M[c][0] * Kj[0][i] + M[c][1] * Kj[1][i] + L[c][i]);
            Lk[j][c] = 2.0 * (M[c][0] * kj[0] + M[c][1] * kj[1] + g[c]);
        }
        memcpy(K[j], Kj, sizeof(Kj));
        kk[j][0] = kj[0];
        kk[j][1] = kj[1];
        /* value function: P = Wxx + K'MK + Wxu K + K'Wxu' ; p = wx + K'Mk + K'g + Wxu k */
        double MK[2][3];
        for (int c = 0; c < 2; c++)
            for (int i = 0; i < 3; i++) MK[c][i] = M[c][0] * Kj[0][i] + M[c][1] * Kj[1][i];
        for (int i = 0; i < 3; i++)
            for (int l = 0; l < 3; l++) {
                double v = Wxx[i][l];
                for (int c = 0; c < 2; c++)
                    v += Kj[c][i] * MK[c][l] + Wxu[i][c] * Kj[c][l] + Kj[c][i] * Wxu[l][c];
                P[i][l] = v;
            }
        for (int i = 0; i < 3; i++) {
            double v = wx[i];
            for (int c = 0; c < 2; c++) {
                double Mk_c = M[c][0] * kj[0] + M[c][1] * kj[1];
                v += Kj[c][i] * (Mk_c + g[c]) + Wxu[i][c] * kj[c];
            }
            p[i] = v;
        }
        for (int i = 0; i < 3; i++)            /* symmetrise */
            for (int l = i + 1; l < 3; l++) {
                double m = 0.5 * (P[i][l] + P[l][i]);
                P[i][l] = m;
                P[l][i] = m;
            }
    }
    /* forward pass */
    double x[3] = {pr->x0[0], pr->x0[1], pr->x0[2]};
    for (int j = 0; j < nb; j++) {
        int k0 = j * bs, k1 = k0 + bs;
        if (k1 > N) k1 = N;
        double u0 = K[j][0][0] * x[0] + K[j][0][1] * x[1] + K[j][0][2] * x[2] + kk[j][0];
        double u1 = K[j][1][0] * x[0] + K[j][1][1] * x[1] + K[j][1][2] * x[2] + kk[j][1];
        for (int c = 0; c < 2; c++)
            lam[j][c] = LK[j][c][0] * x[0] + LK[j][c][1] * x[1] + LK[j][c][2] * x[2] + Lk[j][c];
        s->u[j][0] = u0;
        s->u[j][1] = u1;
        for (int k = k0; k < k1; k++) {
            s->x[k][0] = x[0];
            s->x[k][1] = x[1];
            s->x[k][2] = x[2];
            double nx0 = x[0] + pr->a0[k] * x[2] + pr->b0[k] * u0;
            double nx1 = x[1] + pr->a1[k] * x[2] + pr->b1[k] * u0;
            double nx2 = x[2] + dt * u1;
            x[0] = nx0;
            x[1] = nx1;
            x[2] = nx2;
        }
    }
    s->x[N][0] = x[0];
    s->x[N][1] = x[1];
    s->x[N][2] = x[2];
}

/* forward simulation of the decision u (per block) from x0; objective F and, optionally,
 * the hinge residual signs.  F is the full (slack-eliminated) QP objective.             */
static double simulate_F(const Prob *pr, const double u[NM][2], double x[NM + 1][3]) {
    const int N = pr->N;
    double xc[3] = {pr->x0[0], pr->x0[1], pr->x0[2]};
    double F = 0.0;
    for (int k = 0; k < N; k++) {
        const int j = k / pr->bs;
        x[k][0] = xc[0];
        x[k][1] = xc[1];
        x[k][2] = xc[2];
        for (int i = 0; i < 3; i++) {
            double e = xc[i] - pr->xs[k][i];
            F += pr->Qd[i] * e * e;
        }
        for (int c = 0; c < 2; c++) {
            double uu = u[j][c] + pr->us[k][c];
            F += pr->Rd[c] * uu * uu;
        }
        for (int o = 0; o < pr->no; o++) {
            if (!pr->hk[k][o]) continue;
            double r = pr->hb[k][o] - pr->hn0[k][o] * xc[0] - pr->hn1[k][o] * xc[1];
            if (r > 0) F += pr->rho * r * r;
        }
        double n0 = xc[0] + pr->a0[k] * xc[2] + pr->b0[k] * u[j][0];
        double n1 = xc[1] + pr->a1[k] * xc[2] + pr->b1[k] * u[j][0];
        double n2 = xc[2] + pr->dt * u[j][1];
        xc[0] = n0;
        xc[1] = n1;
        xc[2] = n2;
    }
    x[N][0] = xc[0];
    x[N][1] = xc[1];
    x[N][2] = xc[2];
    for (int i = 0; i < 3; i++) {
        double e = xc[i] - pr->xs[N][i];
        F += pr->Pd[i] * e * e;
    }
    return F;
}

/* adjoint gradient dF/du (per block) at the trajectory x of u */
static void gradient(const Prob *pr, const double u[NM][2], const double x[NM + 1][3],
                     double g[NM][2]) {
    const int N = pr->N;
    double lam[3];
    for (int i = 0; i < 3; i++) lam[i] = 2.0 * pr->Pd[i] * (x[N][i] - pr->xs[N][i]);
    for (int j = 0; j < pr->nb; j++) g[j][0] = g[j][1] = 0.0;
    for (int k = N - 1; k >= 0; k--) {
        const int j = k / pr->bs;
        /* du: 2R(u+us) + B' lam_{k+1} */
        g[j][0] += 2.0 * pr->Rd[0] * (u[j][0] + pr->us[k][0]) + pr->b0[k] * lam[0] + pr->b1[k] * lam[1];
        g[j][1] += 2.0 * pr->Rd[1] * (u[j][1] + pr->us[k][1]) + pr->dt * lam[2];
        /* lam_k = dl_k/dx + A' lam_{k+1} */
        double l0 = lam[0], l1 = lam[1], l2 = lam[2];
        double d0 = 2.0 * pr->Qd[0] * (x[k][0] - pr->xs[k][0]);
        double d1 = 2.0 * pr->Qd[1] * (x[k][1] - pr->xs[k][1]);
        double d2 = 2.0 * pr->Qd[2] * (x[k][2] - pr->xs[k][2]);
        for (int o = 0; o < pr->no; o++) {
            if (!pr->hk[k][o]) continue;
            double r = pr->hb[k][o] - pr->hn0[k][o] * x[k][0] - pr->hn1[k][o] * x[k][1];
            if (r > 0) {
                d0 -= 2.0 * pr->rho * r * pr->hn0[k][o];
                d1 -= 2.0 * pr->rho * r * pr->hn1[k][o];
            }
        }
        lam[0] = d0 + l0;
        lam[1] = d1 + l1;
        lam[2] = d2 + pr->a0[k] * l0 + pr->a1[k] * l1 + l2;
    }
}

#ifndef RMPC_KMAX_STUDY
#define RMPC_KMAX_STUDY 0
#endif
#if RMPC_KMAX_STUDY
/* (study builds only, scripts/study_gain_reuse.py: histogram of the last step whose sets a
 * stage-1 PDAS update changed -- the backward sweep's gains beyond it repeat the last sweep's) */
static long g_kmax_hist[NM + 2];
static _Thread_local int g_in_stage1;
void rmpc_cpu_kmax_hist(long *out) { memcpy(out, g_kmax_hist, sizeof(g_kmax_hist)); }
void rmpc_cpu_kmax_reset(void) { memset(g_kmax_hist, 0, sizeof(g_kmax_hist)); }
#endif
/* PDAS set update from a Riccati solution; returns 1 if any set changed */
static int update_sets(const Prob *pr, const Sol *s, const double lam[NM][2], uint8_t hact[NM][OM],
                       uint8_t bfix[NM][2]) {
    const double eps_h = 1e-14, eps_b = 1e-13;
    int changed = 0;
#if RMPC_KMAX_STUDY
    int kmax = -1;
#define KMAX_NOTE(k) do { if ((k) > kmax) kmax = (k); } while (0)
#else
#define KMAX_NOTE(k) do { } while (0)
#endif
    for (int k = 1; k < pr->N; k++)
        for (int o = 0; o < pr->no; o++) {
            if (!pr->hk[k][o]) continue;
            double r = pr->hb[k][o] - pr->hn0[k][o] * s->x[k][0] - pr->hn1[k][o] * s->x[k][1];
            uint8_t na = hact[k][o] ? (r > -eps_h) : (r > eps_h);
            if (na != hact[k][o]) { changed = 1; hact[k][o] = na; KMAX_NOTE(k); }
        }
    for (int j = 0; j < pr->nb; j++)
        for (int c = 0; c < 2; c++) {
            uint8_t st = bfix[j][c], ns = st;
            double u = s->u[j][c];
            if (st == 0) {
                if (u < pr->lo[j][c] - eps_b) ns = 1;
                else if (u > pr->hi[j][c] + eps_b) ns = 2;
            } else if (st == 1) {
                if (lam[j][c] < 0) ns = 0;
            } else {
                if (lam[j][c] > 0) ns = 0;
            }
            if (ns != st) { changed = 1; bfix[j][c] = ns; KMAX_NOTE(j * pr->bs); }
        }
#if RMPC_KMAX_STUDY
    if (changed && g_in_stage1) {
#pragma omp atomic
        g_kmax_hist[kmax + 1]++;
    }
#endif
#undef KMAX_NOTE
    return changed;
}

/* signature of the active sets (cycle detection) */
static uint64_t set_signature(const Prob *pr, const uint8_t hact[NM][OM], const uint8_t bfix[NM][2]) {
    uint64_t h = 1469598103934665603ull;
    for (int k = 0; k < pr->N; k++) {
        uint32_t w = 0;
        for (int o = 0; o < pr->no; o++) w |= (uint32_t)(hact[k][o] != 0) << o;
        h = (h ^ w) * 1099511628211ull;
    }
    for (int j = 0; j < pr->nb; j++) h = (h ^ (uint64_t)(bfix[j][0] | (bfix[j][1] << 2))) * 1099511628211ull;
    return h;
}

/* Active-set solver; returns 1 if the KKT conditions were certified.
 * Phase 1: primal-dual active set (semismooth Newton, full steps) -- 1 Riccati solve for
 *          ~70% of config-3 robots, <= 10 for 99%; on robots starting inside an obstacle's
 *          margin the actuator bounds activate in a monotone cascade over several solves.
 *          Capped at PDAS_ITERS solves, and left as soon as an active-set signature
 *          repeats (PDAS cycling, ~1e-3 of instances).
 * Phase 2: projected Newton with Armijo backtracking on F over the box (Bertsekas 1982)
 *          from the projected last iterate, with the same Riccati solve as its Newton step;
 *          it certifies with the same set-reproduction test.                           */
#define PDAS_ITERS 32
static long g_cnt[4];
/* Stage caps of the GPU pipeline (rmpc_api.cpp): fast_cap PDAS solves with cycle detection (the
 * lane-per-robot kernel), then tail_cap more from the same sets (the lane-group tail; cycle
 * detection only for caps > 4, as there), then projected Newton.  0, 0 (the default): one
 * PDAS phase of up to PDAS_ITERS solves.  Set with rmpc_cpu_set_pdas_caps to restate the
 * device's iterate path (and iteration counts) for one configuration. */
static int g_fast_cap = 0, g_tail_cap = 0;
void rmpc_cpu_set_pdas_caps(int fast_cap, int tail_cap) { g_fast_cap = fast_cap; g_tail_cap = tail_cap; }
           /* diagnostics: phase-2 entries, phase-2 iterations, F evaluations */
long rmpc_cpu_counter(int i) { return (i >= 0 && i < 4) ? g_cnt[i] : 0; }
void rmpc_cpu_reset_counters(void) { memset(g_cnt, 0, sizeof(g_cnt)); }
#ifndef RMPC_LS_STUDY
#define RMPC_LS_STUDY 0
#endif
#if RMPC_LS_STUDY > 0
/* trial step lengths of the study modes: 1 = {1, 1/2, 1/4, 1/8}, 2 = {2, 1, 1/2, 1/4},
 * 3 = {1.5, 1, 0.7, 0.45}, 4 = 200 points on (0, 2] (the ceiling) */
static int ls_study_pick(const Prob *pr, double z[NM][2], const Sol *s, double g[NM][2], double F,
                         double zbest[NM][2], double xbest[NM + 1][3], double *Fbest) {
    static const double a1[] = {1, .5, .25, .125}, a2[] = {2, 1, .5, .25}, a3[] = {1.5, 1, .7, .45};
    const int mode = RMPC_LS_STUDY, n = mode == 4 ? 200 : 4;
    int found = 0;
    double zt[NM][2], xt[NM + 1][3];
    for (int i = 0; i < n; i++) {
        const double alpha = mode == 1 ? a1[i] : mode == 2 ? a2[i] : mode == 3 ? a3[i] : 2.0 * (i + 1) / n;
        double gd = 0.0;
        for (int j = 0; j < pr->nb; j++)
            for (int c = 0; c < 2; c++) {
                zt[j][c] = clampd(z[j][c] + alpha * (s->u[j][c] - z[j][c]), pr->lo[j][c], pr->hi[j][c]);
                gd += g[j][c] * (zt[j][c] - z[j][c]);
            }
        const double Ft = simulate_F(pr, (const double(*)[2])zt, xt);
        if (Ft <= F + 1e-4 * gd && (!found || Ft < *Fbest)) {
            found = 1;
            *Fbest = Ft;
            memcpy(zbest, zt, sizeof(zt));
            memcpy(xbest, xt, sizeof(xt));
        }
    }
    return found;
}
#endif
static int pdas_solve(const Prob *pr, int max_iter, Sol *s) {
    uint8_t hact[NM][OM];
    uint8_t bfix[NM][2];
    double lam[NM][2];
    memset(hact, 0, sizeof(hact));
    memset(bfix, 0, sizeof(bfix));
    s->converged = 0;
    int it = 0;
    uint64_t hist[4] = {0, 0, 0, 0};
    double xt[NM + 1][3];
    const int staged = g_fast_cap > 0;
    const int cap1 = staged ? g_fast_cap : PDAS_ITERS;
    for (; it < max_iter && it < cap1;) {
        riccati_solve(pr, (const uint8_t(*)[OM])hact, (const uint8_t(*)[2])bfix, s, lam);
        s->iters = ++it;
#if RMPC_KMAX_STUDY
        g_in_stage1 = it < cap1;      /* an update that the next stage-1 sweep consumes */
#endif
        if (!update_sets(pr, s, (const double(*)[2])lam, hact, bfix)) {
            s->converged = 1;
            return 1;
        }
        const uint64_t sig = set_signature(pr, (const uint8_t(*)[OM])hact, (const uint8_t(*)[2])bfix);
        if (sig == hist[0] || sig == hist[1] || sig == hist[2] || sig == hist[3]) break;   /* cycle */
        hist[it & 3] = sig;
    }
    if (staged) {     /* the tail's PDAS phase: tail_cap more solves from the same sets */
        uint64_t h2[4] = {0, 0, 0, 0};
        for (int t = 0; t < g_tail_cap && it < max_iter; t++) {
            riccati_solve(pr, (const uint8_t(*)[OM])hact, (const uint8_t(*)[2])bfix, s, lam);
            s->iters = ++it;
            if (!update_sets(pr, s, (const double(*)[2])lam, hact, bfix)) {
                s->converged = 1;
                return 1;
            }
            if (g_tail_cap > 4) {
                const uint64_t sig = set_signature(pr, (const uint8_t(*)[OM])hact, (const uint8_t(*)[2])bfix);
                if (sig == h2[0] || sig == h2[1] || sig == h2[2] || sig == h2[3]) break;
                h2[3] = h2[2]; h2[2] = h2[1]; h2[1] = h2[0]; h2[0] = sig;
            }
        }
    }
    if (it >= max_iter) {
        for (int j = 0; j < pr->nb; j++)
            for (int c = 0; c < 2; c++) s->u[j][c] = clampd(s->u[j][c], pr->lo[j][c], pr->hi[j][c]);
        simulate_F(pr, (const double(*)[2])s->u, s->x);
        return 0;
    }
    /* ---- phase 2: globalised projected Newton from the projected last iterate */
    g_cnt[0]++;
    double z[NM][2], g[NM][2], x[NM + 1][3];
    for (int j = 0; j < pr->nb; j++)
        for (int c = 0; c < 2; c++) z[j][c] = clampd(s->u[j][c], pr->lo[j][c], pr->hi[j][c]);
    double F = simulate_F(pr, (const double(*)[2])z, x);
    for (; it < max_iter;) {
        gradient(pr, (const double(*)[2])z, (const double(*)[3])x, g);
        double w = 0.0;
        for (int j = 0; j < pr->nb; j++)
            for (int c = 0; c < 2; c++)
                w = fmax(w, fabs(z[j][c] - clampd(z[j][c] - g[j][c], pr->lo[j][c], pr->hi[j][c])));
        const double eps = fmin(1e-6, w);
        for (int k = 1; k < pr->N; k++)
            for (int o = 0; o < pr->no; o++) {
                if (!pr->hk[k][o]) { hact[k][o] = 0; continue; }
                double r = pr->hb[k][o] - pr->hn0[k][o] * x[k][0] - pr->hn1[k][o] * x[k][1];
                hact[k][o] = r > 0;
            }
        for (int j = 0; j < pr->nb; j++)
            for (int c = 0; c < 2; c++) {
                bfix[j][c] = 0;
                if (z[j][c] <= pr->lo[j][c] + eps && g[j][c] > 0) bfix[j][c] = 1;
                else if (z[j][c] >= pr->hi[j][c] - eps && g[j][c] < 0) bfix[j][c] = 2;
            }
        riccati_solve(pr, (const uint8_t(*)[OM])hact, (const uint8_t(*)[2])bfix, s, lam);
        s->iters = ++it;
        g_cnt[1]++;
        uint8_t h2[NM][OM], b2[NM][2];
        memcpy(h2, hact, sizeof(h2));
        memcpy(b2, bfix, sizeof(b2));
        if (!update_sets(pr, s, (const double(*)[2])lam, h2, b2)) {
            s->converged = 1;                 /* the Newton point is the exact optimum */
            return 1;
        }
        /* Armijo backtracking along the projection arc */
        double alpha = 1.0, zt[NM][2], Ft = F;
        int acc = 0;
#if RMPC_LS_STUDY > 0
        /* (line-search study builds only, scripts/study_linesearch.py: several trial points
         * along the arc evaluated up front, the lowest F among those passing Armijo taken) */
        if (ls_study_pick(pr, z, s, g, F, zt, xt, &Ft)) {
            memcpy(z, zt, sizeof(z));
            memcpy(x, xt, sizeof(x));
            F = Ft;
            continue;
        }
#endif
        for (int ls = 0; ls < 40; ls++) {
            double gd = 0.0;
            for (int j = 0; j < pr->nb; j++)
                for (int c = 0; c < 2; c++) {
                    zt[j][c] = clampd(z[j][c] + alpha * (s->u[j][c] - z[j][c]), pr->lo[j][c], pr->hi[j][c]);
                    gd += g[j][c] * (zt[j][c] - z[j][c]);
                }
            Ft = simulate_F(pr, (const double(*)[2])zt, xt);
            g_cnt[2]++;
            if (Ft <= F + 1e-4 * gd) { acc = 1; break; }
            {   /* safeguarded quadratic interpolation, as the lane-group tail's default
                 * (rmpc_mpc_group.hip, ls_beta = 0): q(a) = F + (gd/alpha) a + c a^2 through
                 * the failed trial, next alpha = argmin q clamped to [0.1, 0.5] alpha */
                const double gdn = gd / alpha, c = (Ft - F - gdn * alpha) / (alpha * alpha);
                double an = c > 0.0 ? -gdn / (2.0 * c) : 0.5 * alpha;
                if (!(an >= 0.1 * alpha)) an = 0.1 * alpha;
                if (!(an <= 0.5 * alpha)) an = 0.5 * alpha;
                alpha = an;
            }
        }
        if (!acc) break;                      /* no progress possible at this precision */
        memcpy(z, zt, sizeof(z));
        memcpy(x, xt, sizeof(x));
        F = Ft;
    }
    /* not certified: leave the best box-feasible iterate in s (OPTIMAL_INACCURATE) */
    for (int j = 0; j < pr->nb; j++) { s->u[j][0] = z[j][0]; s->u[j][1] = z[j][1]; }
    memcpy(s->x, x, sizeof(x));
    return 0;
}

/* ------------------------------------------------------------------ LTV / LTI setup */
static void setup_ltv(const RmpcMpcParams *p, const double *x0, const double *xr, int ref_rows,
                      const double *ur, const double *obs, int no, Prob *pr, double *th_unw) {
    const int N = p->horizon;
    int bs = p->block_size < 1 ? 1 : p->block_size;
    pr->N = N;
    pr->bs = bs;
    pr->nb = (N + bs - 1) / bs;
    pr->no = no;
    pr->dt = p->dt;
    pr->rho = p->slack_penalty;
    memcpy(pr->Qd, p->Q, sizeof(pr->Qd));
    memcpy(pr->Rd, p->R, sizeof(pr->Rd));
    memcpy(pr->Pd, p->P, sizeof(pr->Pd));
    /* np.unwrap of x_refs[:,2] (mpc_controller.py:392-393); only the prefix is needed */
    double corr = 0.0;
    th_unw[0] = xr[2];
    for (int k = 1; k <= N && k < ref_rows; k++) {
        double dd = xr[3 * k + 2] - xr[3 * (k - 1) + 2];
        double ddmod = np_mod(dd + PI_D, 2.0 * PI_D) - PI_D;
        if (ddmod == -PI_D && dd > 0) ddmod = PI_D;
        double ph = ddmod - dd;
        if (fabs(dd) < PI_D) ph = 0.0;
        corr += ph;
        th_unw[k] = xr[3 * k + 2] + corr;
    }
    (void)ref_rows;
    /* x0 heading moved into the reference branch (:397-401) */
    double th0 = th_unw[0];
    double x0a = th0 + wrap_pi(x0[2] - th0);
    pr->x0[0] = x0[0] - xr[0];
    pr->x0[1] = x0[1] - xr[1];
    pr->x0[2] = x0a - th0;
    for (int k = 0; k <= N; k++) pr->xs[k][0] = pr->xs[k][1] = pr->xs[k][2] = 0.0;
    for (int k = 0; k < N; k++) {
        double v = ur[2 * k];
        double vr = fabs(v) > 0.01 ? v : 0.1;                      /* :425 */
        double s = sin(th_unw[k]), c = cos(th_unw[k]);
        pr->a0[k] = -vr * s * p->dt;
        pr->a1[k] = vr * c * p->dt;
        pr->b0[k] = c * p->dt;
        pr->b1[k] = s * p->dt;
        pr->us[k][0] = ur[2 * k];
        pr->us[k][1] = ur[2 * k + 1];
    }
    for (int j = 0; j < pr->nb; j++) {                              /* :431-436 */
        double lo0 = -1e300, hi0 = 1e300, lo1 = -1e300, hi1 = 1e300;
        for (int k = j * bs; k < (j + 1) * bs && k < N; k++) {
            lo0 = fmax(lo0, -p->v_max - ur[2 * k]);
            hi0 = fmin(hi0, p->v_max - ur[2 * k]);
            lo1 = fmax(lo1, -p->omega_max - ur[2 * k + 1]);
            hi1 = fmin(hi1, p->omega_max - ur[2 * k + 1]);
        }
        pr->lo[j][0] = lo0;
        pr->hi[j][0] = hi0;
        pr->lo[j][1] = lo1;
        pr->hi[j][1] = hi1;
    }
    for (int k = 0; k < N; k++)                                     /* :439-468 */
        for (int o = 0; o < no; o++) {
            double ddx = xr[3 * k] - obs[3 * o], ddy = xr[3 * k + 1] - obs[3 * o + 1];
            double dist = sqrt(ddx * ddx + ddy * ddy);
            pr->hk[k][o] = (p->soft && dist > 0.01) ? 1 : 0;
            if (pr->hk[k][o]) {
                double nx = ddx / dist, ny = ddy / dist;
                double safe = p->d_safe + obs[3 * o + 2];
                pr->hn0[k][o] = nx;
                pr->hn1[k][o] = ny;
                pr->hb[k][o] = safe - (nx * (xr[3 * k] - obs[3 * o]) + ny * (xr[3 * k + 1] - obs[3 * o + 1]));
            }
        }
}

static void setup_lti(const RmpcMpcParams *p, const double *x0, const double *xr_in, int ref_rows,
                      const double *ur_in, int uref_rows, const double *obs, int no, Prob *pr,
                      double *xr_pad, double *ur_pad) {
    const int N = p->horizon;
    for (int k = 0; k <= N; k++) {                                  /* :172-177 */
        int kk = k < ref_rows ? k : ref_rows - 1;
        for (int i = 0; i < 3; i++) xr_pad[3 * k + i] = xr_in[3 * kk + i];
    }
    for (int k = 0; k < N; k++) {                                   /* :179-183 */
        int kk = k < uref_rows ? k : uref_rows - 1;
        ur_pad[2 * k] = ur_in[2 * kk];
        ur_pad[2 * k + 1] = ur_in[2 * kk + 1];
    }
    pr->N = N;
    pr->bs = 1;
    pr->nb = N;
    pr->no = no;
    pr->dt = p->dt;
    pr->rho = p->slack_penalty;
    memcpy(pr->Qd, p->Q, sizeof(pr->Qd));
    memcpy(pr->Rd, p->R, sizeof(pr->Rd));
    memcpy(pr->Pd, p->P, sizeof(pr->Pd));
    double v = ur_pad[0];
    double vr = fabs(v) > 0.01 ? v : 0.1;                          /* :186 */
    double s = sin(xr_pad[2]), c = cos(xr_pad[2]);
    for (int k = 0; k < N; k++) {
        pr->a0[k] = -vr * s * p->dt;
        pr->a1[k] = vr * c * p->dt;
        pr->b0[k] = c * p->dt;
        pr->b1[k] = s * p->dt;
        pr->us[k][0] = pr->us[k][1] = 0.0;
        pr->lo[k][0] = -p->v_max;
        pr->hi[k][0] = p->v_max;
        pr->lo[k][1] = -p->omega_max;
        pr->hi[k][1] = p->omega_max;
    }
    for (int k = 0; k <= N; k++)
        for (int i = 0; i < 3; i++) pr->xs[k][i] = xr_pad[3 * k + i];
    for (int i = 0; i < 3; i++) pr->x0[i] = x0[i];
    for (int k = 0; k < N; k++)                                     /* :237-270 */
        for (int o = 0; o < no; o++) {
            double ddx = xr_pad[3 * k] - obs[3 * o], ddy = xr_pad[3 * k + 1] - obs[3 * o + 1];
            double dist = sqrt(ddx * ddx + ddy * ddy);
            pr->hk[k][o] = (p->soft && dist > 0.01) ? 1 : 0;
            if (pr->hk[k][o]) {
                double nx = ddx / dist, ny = ddy / dist;
                pr->hn0[k][o] = nx;
                pr->hn1[k][o] = ny;
                pr->hb[k][o] = p->d_safe + obs[3 * o + 2] + nx * obs[3 * o] + ny * obs[3 * o + 1];
            }
        }
}

/* objective value (problem.value) and slack usage at the solution */
static double objective(const Prob *pr, const Sol *s, int *slack_used) {
    double J = 0.0;
    int used = 0;
    for (int k = 0; k <= pr->N; k++) {
        const double *W = k < pr->N ? pr->Qd : pr->Pd;
        for (int i = 0; i < 3; i++) {
            double e = s->x[k][i] - pr->xs[k][i];
            J += W[i] * e * e;
        }
        if (k < pr->N) {
            int j = k / pr->bs;
            for (int c = 0; c < 2; c++) {
                double u = s->u[j][c] + pr->us[k][c];
                J += pr->Rd[c] * u * u;
            }
            for (int o = 0; o < pr->no; o++) {
                if (!pr->hk[k][o]) continue;
                double r = pr->hb[k][o] - pr->hn0[k][o] * s->x[k][0] - pr->hn1[k][o] * s->x[k][1];
                if (r > 0) {
                    J += pr->rho * r * r;
                    if (r > 1e-6) used = 1;
                }
            }
        }
    }
    *slack_used = used;
    return J;
}

static int finite_prob(const Prob *pr) {
    double acc = pr->x0[0] + pr->x0[1] + pr->x0[2];
    for (int k = 0; k < pr->N; k++) acc += pr->a0[k] + pr->a1[k] + pr->us[k][0] + pr->us[k][1];
    for (int k = 0; k <= pr->N; k++) acc += pr->xs[k][0] + pr->xs[k][1] + pr->xs[k][2];
    return isfinite(acc);
}

static void mpc_one(const RmpcMpcParams *p, const double *x0, const double *xr, int ref_rows,
                    const double *ur, int uref_rows, const double *obs, int no, int32_t *step_count,
                    double *u0, double *useq, double *xpred, double *cost, int32_t *status,
                    uint8_t *slack, int32_t *iters) {
    Prob pr;
    Sol s;
    s.iters = 0;
    double th[NM + 1], xr_pad[3 * (NM + 1)], ur_pad[2 * NM];
    const int N = p->horizon;
    const int ltv = p->formulation == RMPC_LTV;
    const double *xrr = xr, *urr = ur;
    if (ltv) {
        setup_ltv(p, x0, xr, ref_rows, ur, obs, no, &pr, th);
    } else {
        setup_lti(p, x0, xr, ref_rows, ur, uref_rows, obs, no, &pr, xr_pad, ur_pad);
        xrr = xr_pad;
        urr = ur_pad;
    }
    int fin = finite_prob(&pr);
    int cert = fin && pdas_solve(&pr, p->max_iter > 0 ? p->max_iter : 64, &s);
    int ok = fin;
    double ucur[2] = {0.0, 0.0};
    if (ok) {
        int su;
        double J = objective(&pr, &s, &su);
        ok = isfinite(J);
        if (ok) {
            if (cost) *cost = J;
            if (slack) *slack = (uint8_t)su;
            for (int k = 0; k < N; k++) {
                int j = k / pr.bs;
                double a = s.u[j][0] + (ltv ? urr[2 * k] : 0.0);
                double b = s.u[j][1] + (ltv ? urr[2 * k + 1] : 0.0);
                if (useq) { useq[2 * k] = a; useq[2 * k + 1] = b; }
                if (k == 0) { ucur[0] = a; ucur[1] = b; }
            }
            for (int k = 0; k <= N; k++)
                for (int i = 0; i < 3; i++)
                    if (xpred) xpred[3 * k + i] = s.x[k][i] + (ltv ? xrr[3 * k + i] : 0.0);
            if (ltv) {
                int sc = step_count ? *step_count : 0;
                int ramp = p->ramp_up_steps;
                if (sc < ramp) {                                            /* :502-505 */
                    double lim = p->omega_max * ((double)(sc + 1) / (double)ramp);
                    ucur[1] = clampd(ucur[1], -lim, lim);
                    if (useq) useq[1] = ucur[1];
                }
                if (step_count) *step_count = sc + 1;                       /* :507 */
            }
            u0[0] = ucur[0];
            u0[1] = ucur[1];
            *status = cert ? RMPC_OPTIMAL : RMPC_OPTIMAL_INACCURATE;
            if (iters) *iters = s.iters;
            return;
        }
    }
    /* fallback law mpc_controller.py:316-343 (x_refs / u_refs as passed, padded for LTI) */
    double e0 = x0[0] - xrr[0], e2 = wrap_pi(x0[2] - xrr[2]);
    double a = clampd(urr[0] - e0, -p->v_max, p->v_max);
    double b = clampd(urr[1] - 0.5 * e2, -p->omega_max, p->omega_max);
    u0[0] = a;
    u0[1] = b;
    if (useq)
        for (int k = 0; k < N; k++) { useq[2 * k] = a; useq[2 * k + 1] = b; }
    if (xpred)
        for (int k = 0; k <= N; k++)
            for (int i = 0; i < 3; i++) xpred[3 * k + i] = x0[i];
    if (cost) *cost = INFINITY;
    if (slack) *slack = 0;
    if (iters) *iters = s.iters;
    *status = RMPC_FALLBACK;
}

int rmpc_cpu_mpc_solve_batch(const RmpcMpcParams *p, int64_t B, const double *x0,
                             const double *x_refs, int32_t ref_rows, const double *u_refs,
                             int32_t uref_rows, const double *obstacles, int32_t n_obs,
                             int32_t *step_count, double *u0, double *u_seq, double *x_pred,
                             double *cost, int32_t *status, uint8_t *slack_used, int32_t *iters,
                             int32_t n_threads) {
    const int N = p->horizon;
    if (N < 1 || N > NM || n_obs < 0 || n_obs > OM) return RMPC_EINVAL;
    if (p->formulation == RMPC_LTV && (ref_rows < N + 1 || uref_rows < N)) return RMPC_EINVAL;
    if (ref_rows < 1 || uref_rows < 1) return RMPC_EINVAL;
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1)
    for (int64_t b = 0; b < B; b++) {
        mpc_one(p, x0 + 3 * b, x_refs + (int64_t)3 * ref_rows * b, ref_rows,
                u_refs + (int64_t)2 * uref_rows * b, uref_rows, obstacles, n_obs,
                step_count ? step_count + b : NULL, u0 + 2 * b,
                u_seq ? u_seq + (int64_t)2 * N * b : NULL,
                x_pred ? x_pred + (int64_t)3 * (N + 1) * b : NULL, cost ? cost + b : NULL,
                status + b, slack_used ? slack_used + b : NULL, iters ? iters + b : NULL);
    }
    return RMPC_OK;
}

/* ------------------------------------------------------------------ LQR (SDA DARE) */
static int inv3(const double M[3][3], double I[3][3]) {
    double c00 = M[1][1] * M[2][2] - M[1][2] * M[2][1];
    double c01 = M[1][2] * M[2][0] - M[1][0] * M[2][2];
    double c02 = M[1][0] * M[2][1] - M[1][1] * M[2][0];
    double det = M[0][0] * c00 + M[0][1] * c01 + M[0][2] * c02;
    if (!(fabs(det) > 0) || !isfinite(det)) return 0;
    double id = 1.0 / det;
    I[0][0] = c00 * id;
    I[1][0] = c01 * id;
    I[2][0] = c02 * id;
    I[0][1] = (M[0][2] * M[2][1] - M[0][1] * M[2][2]) * id;
    I[1][1] = (M[0][0] * M[2][2] - M[0][2] * M[2][0]) * id;
    I[2][1] = (M[0][1] * M[2][0] - M[0][0] * M[2][1]) * id;
    I[0][2] = (M[0][1] * M[1][2] - M[0][2] * M[1][1]) * id;
    I[1][2] = (M[0][2] * M[1][0] - M[0][0] * M[1][2]) * id;
    I[2][2] = (M[0][0] * M[1][1] - M[0][1] * M[1][0]) * id;
    return 1;
}

static void mm3(const double A[3][3], const double B[3][3], double C[3][3]) {
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C[i][j] = A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j];
}

/* DARE by SDA: A_{k+1} = A W^-1 A, G_{k+1} = G + A W^-1 G A', H_{k+1} = H + A' H W^-1 A, W = I + G H */
static int lqr_gain_one(const RmpcLqrParams *p, double v_r, double th, int guard, double K[6],
                        double Pout[9]) {
    if (guard && fabs(v_r) < 1e-6) v_r = 0.01;                       /* :120-122 */
    double s = sin(th), c = cos(th), dt = p->dt;
    double A[3][3] = {{1, 0, -v_r * s * dt}, {0, 1, v_r * c * dt}, {0, 0, 1}};
    double Bm[3][2] = {{c * dt, 0}, {s * dt, 0}, {0, dt}};
    double G[3][3], H[3][3] = {{p->Q[0], 0, 0}, {0, p->Q[1], 0}, {0, 0, p->Q[2]}}, Ak[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            G[i][j] = Bm[i][0] * Bm[j][0] / p->R[0] + Bm[i][1] * Bm[j][1] / p->R[1];
    memcpy(Ak, A, sizeof(Ak));
    int maxit = p->max_iter > 0 ? p->max_iter : 64, conv = 0, last = 0;
    for (int it = 0; it < maxit; it++) {
        double W[3][3], Wi[3][3], T[3][3], WiA[3][3], WiG[3][3], nA[3][3], nG[3][3], nH[3][3];
        mm3(G, H, T);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) W[i][j] = (i == j) + T[i][j];
        if (!inv3(W, Wi)) return 0;
        mm3(Wi, Ak, WiA);
        mm3(Wi, G, WiG);
        mm3(Ak, WiA, nA);
        double AWG[3][3], HWA[3][3];
        mm3(Ak, WiG, AWG);
        mm3(H, WiA, HWA);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                double g = G[i][j], h = H[i][j];
                for (int l = 0; l < 3; l++) {
                    g += AWG[i][l] * Ak[j][l];
                    h += Ak[l][i] * HWA[l][j];
                }
                nG[i][j] = g;
                nH[i][j] = h;
            }
        double dH = 0, nrm = 0;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                dH = fmax(dH, fabs(nH[i][j] - H[i][j]));
                nrm = fmax(nrm, fabs(nH[i][j]));
            }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                Ak[i][j] = nA[i][j];
                G[i][j] = 0.5 * (nG[i][j] + nG[j][i]);
                H[i][j] = 0.5 * (nH[i][j] + nH[j][i]);
            }
        if (!isfinite(nrm)) return 0;
        if (last) { conv = 1; break; }
        if (dH <= 1e-10 * nrm) last = 1;   /* quadratic convergence: one more step */
    }
    if (!conv) return 0;
    /* K = (R + B'PB)^-1 B'PA  (:130-132) */
    double PB[3][2], M[2][2], N2[2][3];
    for (int i = 0; i < 3; i++)
        for (int c2 = 0; c2 < 2; c2++)
            PB[i][c2] = H[i][0] * Bm[0][c2] + H[i][1] * Bm[1][c2] + H[i][2] * Bm[2][c2];
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < 2; b++)
            M[a][b] = (a == b ? p->R[a] : 0.0) + Bm[0][a] * PB[0][b] + Bm[1][a] * PB[1][b] + Bm[2][a] * PB[2][b];
    for (int a = 0; a < 2; a++)
        for (int j = 0; j < 3; j++) {
            double acc = 0;
            for (int l = 0; l < 3; l++) acc += PB[l][a] * A[l][j];
            N2[a][j] = acc;
        }
    double det = M[0][0] * M[1][1] - M[0][1] * M[1][0];
    for (int j = 0; j < 3; j++) {
        K[j] = (M[1][1] * N2[0][j] - M[0][1] * N2[1][j]) / det;
        K[3 + j] = (M[0][0] * N2[1][j] - M[1][0] * N2[0][j]) / det;
    }
    if (Pout)
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) Pout[3 * i + j] = H[i][j];
    if (!isfinite(K[0] + K[1] + K[2] + K[3] + K[4] + K[5])) return 0;
    /* stabilising solution: A - BK strictly stable (Jury test), as the device kernel */
    double Mc[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Mc[i][j] = A[i][j] - Bm[i][0] * K[j] - Bm[i][1] * K[3 + j];
    const double tr = Mc[0][0] + Mc[1][1] + Mc[2][2];
    const double c2 = Mc[0][0] * Mc[1][1] - Mc[0][1] * Mc[1][0] + Mc[0][0] * Mc[2][2] - Mc[0][2] * Mc[2][0] +
                      Mc[1][1] * Mc[2][2] - Mc[1][2] * Mc[2][1];
    const double dd = Mc[0][0] * (Mc[1][1] * Mc[2][2] - Mc[1][2] * Mc[2][1]) -
                      Mc[0][1] * (Mc[1][0] * Mc[2][2] - Mc[1][2] * Mc[2][0]) +
                      Mc[0][2] * (Mc[1][0] * Mc[2][1] - Mc[1][1] * Mc[2][0]);
    const double a2 = -tr, a1 = c2, a0 = -dd, eps = 1e-12;
    return (1.0 + a2 + a1 + a0 > eps) && (1.0 - a2 + a1 - a0 > eps) && (fabs(a0) < 1.0 - eps) &&
           (1.0 - a0 * a0 - fabs(a1 - a0 * a2) > eps);
}

int rmpc_cpu_lqr_gain_batch(const RmpcLqrParams *p, int64_t B, const double *v_r,
                            const double *theta_r, int32_t guard_v, double *K_out, double *P_out,
                            int32_t *status, int32_t n_threads) {
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1)
    for (int64_t b = 0; b < B; b++) {
        double K[6];
        int ok = lqr_gain_one(p, v_r[b], theta_r[b], guard_v, K, P_out ? P_out + 9 * b : NULL);
        if (!ok) {
            static const double FB[6] = {1, 0, 0, 0, 0, 1};              /* :137-140 */
            memcpy(K, FB, sizeof(K));
        }
        memcpy(K_out + 6 * b, K, sizeof(K));
        if (status) status[b] = ok ? RMPC_OPTIMAL : RMPC_DARE_FALLBACK;
    }
    return RMPC_OK;
}

int rmpc_cpu_lqr_control_batch(const RmpcLqrParams *p, int64_t B, const double *x,
                               const double *x_ref, const double *u_ref, RmpcLqrCache *cache,
                               double *u_out, double *err_out, int32_t n_threads) {
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1)
    for (int64_t b = 0; b < B; b++) {
        const double *xb = x + 3 * b, *xr = x_ref + 3 * b, *ur = u_ref + 2 * b;
        double K[6];
        double v = ur[0], th = xr[2];
        RmpcLqrCache *cb = cache ? cache + b : NULL;
        if (cb && p->use_cache && cb->valid && fabs(v - cb->last_v) < 1e-6 &&
            fabs(th - cb->last_theta) < 1e-6) {
            memcpy(K, cb->K, sizeof(K));
        } else {
            if (!lqr_gain_one(p, v, th, 1, K, NULL)) {
                static const double FB[6] = {1, 0, 0, 0, 0, 1};
                memcpy(K, FB, sizeof(K));
            }
            if (cb) {
                memcpy(cb->K, K, sizeof(K));
                cb->last_v = v;
                cb->last_theta = th;
                cb->valid = 1;
            }
        }
        double e0 = xb[0] - xr[0], e1 = xb[1] - xr[1], e2 = wrap_pi(xb[2] - xr[2]);
        double u0 = ur[0] + -(K[0] * e0 + K[1] * e1 + K[2] * e2);
        double u1 = ur[1] + -(K[3] * e0 + K[4] * e1 + K[5] * e2);
        u_out[2 * b] = clampd(u0, -p->v_max, p->v_max);
        u_out[2 * b + 1] = clampd(u1, -p->omega_max, p->omega_max);
        if (err_out) {
            err_out[3 * b] = e0;
            err_out[3 * b + 1] = e1;
            err_out[3 * b + 2] = e2;
        }
    }
    return RMPC_OK;
}
