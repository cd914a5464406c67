// rmpc_lqr.hip -- batched LQR gain + control on CDNA4 (gfx950).
//
// Replaces LQRController.compute_control_at_operating_point (lqr_controller.py:191-215),
// i.e. compute_gain (92-147: linearise at (v_r, theta_r), |v_r| < 1e-6 -> 0.01 guard,
// DARE, K = (R + B'PB)^-1 B'PA, fallback K on failure, 1e-6 operating-point cache) and
// compute_control (149-189: wrapped error, u = clip(u_ref - K e)).
//
// One lane per robot; the 3x3 DARE is solved in registers with the structure-preserving
// doubling algorithm (SDA): A_{k+1} = A_k W^-1 A_k, G_{k+1} = G_k + A_k W^-1 G_k A_k',
// H_{k+1} = H_k + A_k' H_k W^-1 A_k, W = I + G_k H_k, H_k -> P quadratically
// (10-17 doubling steps on the Figure-8 operating range versus 350-42000 plain Riccati
// fixed-point steps).  SciPy's solve_discrete_are (QZ) is the reference's
// arithmetic; both return the unique stabilising solution.
#include "rmpc_device.h"
#include "rmpc_internal.h"

namespace rmpc {

struct M3 {
    double m[3][3];
};

__device__ __forceinline__ M3 mul3(const M3 &A, const M3 &B) {
    M3 C;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) C.m[i][j] = A.m[i][0] * B.m[0][j] + A.m[i][1] * B.m[1][j] + A.m[i][2] * B.m[2][j];
    return C;
}

__device__ __forceinline__ bool inv3(const M3 &M, M3 &I) {
    const double c00 = M.m[1][1] * M.m[2][2] - M.m[1][2] * M.m[2][1];
    const double c01 = M.m[1][2] * M.m[2][0] - M.m[1][0] * M.m[2][2];
    const double c02 = M.m[1][0] * M.m[2][1] - M.m[1][1] * M.m[2][0];
    const double det = M.m[0][0] * c00 + M.m[0][1] * c01 + M.m[0][2] * c02;
    if (!(fabs(det) > 0.0) || !isfinite(det)) return false;
    const double id = 1.0 / det;
    I.m[0][0] = c00 * id;
    I.m[1][0] = c01 * id;
    I.m[2][0] = c02 * id;
    I.m[0][1] = (M.m[0][2] * M.m[2][1] - M.m[0][1] * M.m[2][2]) * id;
    I.m[1][1] = (M.m[0][0] * M.m[2][2] - M.m[0][2] * M.m[2][0]) * id;
    I.m[2][1] = (M.m[0][1] * M.m[2][0] - M.m[0][0] * M.m[2][1]) * id;
    I.m[0][2] = (M.m[0][1] * M.m[1][2] - M.m[0][2] * M.m[1][1]) * id;
    I.m[1][2] = (M.m[0][2] * M.m[1][0] - M.m[0][0] * M.m[1][2]) * id;
    I.m[2][2] = (M.m[0][0] * M.m[1][1] - M.m[0][1] * M.m[1][0]) * id;
    return true;
}

// Strict stability of a 3x3 discrete-time system matrix (all eigenvalues inside the unit
// circle, margin 1e-12) by the Jury criterion on its characteristic polynomial.
__device__ __forceinline__ bool jury3_stable(const double M[3][3]) {
    const double tr = M[0][0] + M[1][1] + M[2][2];
    const double c2 = M[0][0] * M[1][1] - M[0][1] * M[1][0] + M[0][0] * M[2][2] - M[0][2] * M[2][0] +
                      M[1][1] * M[2][2] - M[1][2] * M[2][1];
    const double dt = M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) -
                      M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
                      M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
    const double a2 = -tr, a1 = c2, a0 = -dt, eps = 1e-12;
    return (1.0 + a2 + a1 + a0 > eps) && (1.0 - a2 + a1 - a0 > eps) && (fabs(a0) < 1.0 - eps) &&
           (1.0 - a0 * a0 - fabs(a1 - a0 * a2) > eps);
}

// Equal position weights (Q[0] == Q[1]: the reference's defaults [10,10,1] and config 2's
// [15,15,8]) make the DARE rotation-invariant.  In path coordinates z = T'e, T = diag(R(theta), 1),
// the linearisation is A~ = [[1,0,0],[0,1,v dt],[0,0,1]], B~ = [[dt,0],[0,0],[0,dt]] and Q~ = Q:
// the speed channel is a scalar DARE with a closed-form root, the lateral/heading channel a
// 2x2 DARE (SDA on 2x2 blocks, a third of the 3x3 flops).  P = T P~ T', K = K~ T'.
__device__ bool lqr_gain_rotated(const LqrDevParams &p, double v_r, double s, double c, double K[6], M3 *Pout) {
    const double dt = p.dt, q0 = p.Q[0], r0 = p.R[0], r1 = p.R[1];
    // speed channel: p0 = q + p0 - p0^2 dt^2 / (r + p0 dt^2)  ->  p0 = q/2 + sqrt(q^2/4 + q r / dt^2)
    const double p0 = 0.5 * q0 + sqrt(0.25 * q0 * q0 + q0 * r0 / (dt * dt));
    const double k0 = p0 * dt / (r0 + p0 * dt * dt);
    // lateral offset / heading: A2 = [[1, a], [0, 1]], B2 = (0, dt)', Q2 = diag(Q[1], Q[2])
    const double a = v_r * dt;
    double A00 = 1, A01 = a, A10 = 0, A11 = 1;
    double G00 = 0, G01 = 0, G11 = dt * dt / r1;
    double H00 = p.Q[1], H01 = 0, H11 = p.Q[2];
    bool conv = false, last = false;
    for (int it = 0; it < p.max_iter; it++) {
        // W = I + G H, Wi = W^-1
        const double W00 = 1 + G00 * H00 + G01 * H01, W01 = G00 * H01 + G01 * H11;
        const double W10 = G01 * H00 + G11 * H01, W11 = 1 + G01 * H01 + G11 * H11;
        const double det = W00 * W11 - W01 * W10;
        if (!(fabs(det) > 0.0) || !isfinite(det)) return false;
        const double id = 1.0 / det;
        const double I00 = W11 * id, I01 = -W01 * id, I10 = -W10 * id, I11 = W00 * id;
        // WiA = Wi A, WiG = Wi G
        const double X00 = I00 * A00 + I01 * A10, X01 = I00 * A01 + I01 * A11;
        const double X10 = I10 * A00 + I11 * A10, X11 = I10 * A01 + I11 * A11;
        const double Y00 = I00 * G00 + I01 * G01, Y01 = I00 * G01 + I01 * G11;
        const double Y10 = I10 * G00 + I11 * G01, Y11 = I10 * G01 + I11 * G11;
        // A_{k+1} = A WiA; G_{k+1} = G + A WiG A'; H_{k+1} = H + A' H WiA
        const double nA00 = A00 * X00 + A01 * X10, nA01 = A00 * X01 + A01 * X11;
        const double nA10 = A10 * X00 + A11 * X10, nA11 = A10 * X01 + A11 * X11;
        const double Z00 = A00 * Y00 + A01 * Y10, Z01 = A00 * Y01 + A01 * Y11;   // A WiG
        const double Z10 = A10 * Y00 + A11 * Y10, Z11 = A10 * Y01 + A11 * Y11;
        const double U00 = H00 * X00 + H01 * X10, U01 = H00 * X01 + H01 * X11;   // H WiA
        const double U10 = H01 * X00 + H11 * X10, U11 = H01 * X01 + H11 * X11;
        const double g00 = G00 + Z00 * A00 + Z01 * A01, g01 = G01 + Z00 * A10 + Z01 * A11;
        const double g10 = G01 + Z10 * A00 + Z11 * A01, g11 = G11 + Z10 * A10 + Z11 * A11;
        const double h00 = H00 + A00 * U00 + A10 * U10, h01 = H01 + A00 * U01 + A10 * U11;
        const double h10 = H01 + A01 * U00 + A11 * U10, h11 = H11 + A01 * U01 + A11 * U11;
        const double nh01 = 0.5 * (h01 + h10);
        const double dH = fmax(fmax(fabs(h00 - H00), fabs(nh01 - H01)), fabs(h11 - H11));
        const double nrm = fmax(fmax(fabs(h00), fabs(nh01)), fabs(h11));
        A00 = nA00; A01 = nA01; A10 = nA10; A11 = nA11;
        G00 = g00; G01 = 0.5 * (g01 + g10); G11 = g11;
        H00 = h00; H01 = nh01; H11 = h11;
        if (!isfinite(nrm)) return false;
        if (last) { conv = true; break; }
        if (dH <= 1e-10 * nrm) last = true;      // (as the 3x3 SDA below)
    }
    if (!conv) return false;
    // K2 = (r1 + B2'P2B2)^-1 B2'P2A2
    const double den = r1 + dt * dt * H11;
    const double k1 = dt * H01 / den, k2 = dt * (a * H01 + H11) / den;
    // back to the error coordinates: u = -K~ T'e
    K[0] = k0 * c; K[1] = k0 * s; K[2] = 0;
    K[3] = -k1 * s; K[4] = k1 * c; K[5] = k2;
    if (Pout) {
        const double d = p0 - H00;
        Pout->m[0][0] = c * c * p0 + s * s * H00;
        Pout->m[0][1] = Pout->m[1][0] = c * s * d;
        Pout->m[1][1] = s * s * p0 + c * c * H00;
        Pout->m[0][2] = Pout->m[2][0] = -s * H01;
        Pout->m[1][2] = Pout->m[2][1] = c * H01;
        Pout->m[2][2] = H11;
    }
    return isfinite(K[0] + K[1] + K[3] + K[4] + K[5]);
}

// DARE + gain at one operating point; returns false when the DARE fails (fallback K).
__device__ bool lqr_gain(const LqrDevParams &p, double v_r, double th, double K[6], M3 *Pout) {
    double s, c;
    sincos(th, &s, &c);
    const double dt = p.dt;
#ifndef RMPC_LQR_ROTATED
#define RMPC_LQR_ROTATED 1
#endif
    if (RMPC_LQR_ROTATED && p.Q[0] == p.Q[1]) {
        if (!lqr_gain_rotated(p, v_r, s, c, K, Pout)) return false;
        // the same strict-stability test of A - BK as the general path (below)
        const double B[3][2] = {{c * dt, 0}, {s * dt, 0}, {0, dt}};
        const double A2[3] = {-v_r * s * dt, v_r * c * dt, 1};
        double Mc[3][3];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++)
                Mc[i][j] = (j == 2 ? A2[i] : (i == j ? 1.0 : 0.0)) - B[i][0] * K[j] - B[i][1] * K[3 + j];
        return jury3_stable(Mc);
    }
    M3 A = {{{1, 0, -v_r * s * dt}, {0, 1, v_r * c * dt}, {0, 0, 1}}};
    const double B[3][2] = {{c * dt, 0}, {s * dt, 0}, {0, dt}};
    M3 G, H = {{{p.Q[0], 0, 0}, {0, p.Q[1], 0}, {0, 0, p.Q[2]}}};
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) G.m[i][j] = B[i][0] * B[j][0] / p.R[0] + B[i][1] * B[j][1] / p.R[1];
    M3 Ak = A;
    bool conv = false, last = false;
    for (int it = 0; it < p.max_iter; it++) {
        M3 T = mul3(G, H), W, Wi;
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) W.m[i][j] = (i == j ? 1.0 : 0.0) + T.m[i][j];
        if (!inv3(W, Wi)) return false;
        const M3 WiA = mul3(Wi, Ak), WiG = mul3(Wi, G);
        const M3 nA = mul3(Ak, WiA), AWG = mul3(Ak, WiG), HWA = mul3(H, WiA);
        double dH = 0, nrm = 0;
        M3 nG, nH;
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) {
                double g = G.m[i][j], h = H.m[i][j];
#pragma unroll
                for (int l = 0; l < 3; l++) {
                    g += AWG.m[i][l] * Ak.m[j][l];
                    h += Ak.m[l][i] * HWA.m[l][j];
                }
                nG.m[i][j] = g;
                nH.m[i][j] = h;
            }
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) {
                dH = fmax(dH, fabs(nH.m[i][j] - H.m[i][j]));
                nrm = fmax(nrm, fabs(nH.m[i][j]));
                Ak.m[i][j] = nA.m[i][j];
            }
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) {
                G.m[i][j] = 0.5 * (nG.m[i][j] + nG.m[j][i]);
                H.m[i][j] = 0.5 * (nH.m[i][j] + nH.m[j][i]);
            }
        if (!isfinite(nrm)) return false;
        if (last) { conv = true; break; }
        // quadratic convergence: once the update is below 1e-10 relative, one more
        // doubling step lands at rounding level
        if (dH <= 1e-10 * nrm) last = true;
    }
    if (!conv) return false;
    // K = (R + B'PB)^-1 B'PA   (lqr_controller.py:130-132)
    double PB[3][2];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) PB[i][j] = H.m[i][0] * B[0][j] + H.m[i][1] * B[1][j] + H.m[i][2] * B[2][j];
    double M[2][2], Nm[2][3];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
            M[a][b] = (a == b ? p.R[a] : 0.0) + B[0][a] * PB[0][b] + B[1][a] * PB[1][b] + B[2][a] * PB[2][b];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int j = 0; j < 3; j++) Nm[a][j] = PB[0][a] * A.m[0][j] + PB[1][a] * A.m[1][j] + PB[2][a] * A.m[2][j];
    const double id = 1.0 / (M[0][0] * M[1][1] - M[0][1] * M[1][0]);
#pragma unroll
    for (int j = 0; j < 3; j++) {
        K[j] = (M[1][1] * Nm[0][j] - M[0][1] * Nm[1][j]) * id;
        K[3 + j] = (M[0][0] * Nm[1][j] - M[1][0] * Nm[0][j]) * id;
    }
    if (Pout) *Pout = H;
    if (!isfinite(K[0] + K[1] + K[2] + K[3] + K[4] + K[5])) return false;
    // A stabilising solution must leave A - BK strictly stable (SciPy's solve_discrete_are
    // fails otherwise, lqr_controller.py:126 -> fallback :134-141).  Without it, an exactly
    // uncontrollable marginal mode (|v_r| = 0 unguarded at theta_r = 0) lets the doubling
    // "converge" on rounding (A_k -> 0 through W^-1 = 1 - eps) to ||P|| ~ 1e18.
    // Jury test on det(zI - M) = z^3 + a2 z^2 + a1 z + a0, M = A - BK.
    double Mc[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) Mc[i][j] = A.m[i][j] - B[i][0] * K[j] - B[i][1] * K[3 + j];
    return jury3_stable(Mc);
}

// Workgroup size: one wave (RMPC_LQR_BLK=64), so a small batch (config 2: 4096 robots, 64
// waves) spreads over 64 CUs instead of sharing 16
#ifndef RMPC_LQR_BLK
#define RMPC_LQR_BLK 64
#endif
__global__ __launch_bounds__(RMPC_LQR_BLK) void lqr_control_kernel(LqrDevParams p, int64_t B, const double *x,
                                                          const double *x_ref, int xref_stride,
                                                          const double *u_ref, int uref_stride,
                                                          RmpcLqrCache *cache, double *u_out,
                                                          double *err_out, double *K_out,
                                                          double *P_out, int32_t *status,
                                                          const int32_t *index, const int32_t *count) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = index ? (int64_t)*count : B;
    if (t >= n) return;
    const int64_t b = index ? (int64_t)index[t] : t;
    const double *xb = x + 3 * b;
    const double *xr = x_ref + (p.ref_off ? (size_t)p.ref_off[b] * 3 : (size_t)xref_stride * b);
    const double *ur = u_ref + (p.ref_off ? (size_t)p.ref_off[b] * 2 : (size_t)uref_stride * b);
    const double v = ur[0], th = xr[2];
    // every load before the first store (the cache update): one in-order vmcnt
    const double x0 = xb[0], x1 = xb[1], x2 = xb[2], xr0 = xr[0], xr1 = xr[1], u1r = ur[1];
    double K[6];
    int st = RMPC_OPTIMAL;
    bool hit = false;
    if (cache && p.use_cache) {                      // lqr_controller.py:112-114
        const RmpcLqrCache &cb = cache[b];
        if (cb.valid && fabs(v - cb.last_v) < 1e-6 && fabs(th - cb.last_theta) < 1e-6) {
#pragma unroll
            for (int i = 0; i < 6; i++) K[i] = cb.K[i];
            hit = true;
        }
    }
    if (!hit) {
        const double vg = fabs(v) < 1e-6 ? 0.01 : v;  // :120-122
        M3 P;
        if (!lqr_gain(p, vg, th, K, P_out ? &P : nullptr)) {
            K[0] = 1; K[1] = 0; K[2] = 0; K[3] = 0; K[4] = 0; K[5] = 1;   // :137-140
            st = RMPC_DARE_FALLBACK;
        } else if (P_out) {
#pragma unroll
            for (int i = 0; i < 3; i++)
#pragma unroll
                for (int j = 0; j < 3; j++) P_out[9 * b + 3 * i + j] = P.m[i][j];
        }
        if (cache) {
            RmpcLqrCache &cb = cache[b];
#pragma unroll
            for (int i = 0; i < 6; i++) cb.K[i] = K[i];
            cb.last_v = v;
            cb.last_theta = th;
            cb.valid = 1;
        }
    }
    // compute_control (:175-187)
    const double e0 = x0 - xr0, e1 = x1 - xr1, e2 = wrap_pi(x2 - th);
    const double u0 = v + -(K[0] * e0 + K[1] * e1 + K[2] * e2);
    const double u1 = u1r + -(K[3] * e0 + K[4] * e1 + K[5] * e2);
    u_out[2 * b] = clampv(u0, -p.v_max, p.v_max);
    u_out[2 * b + 1] = clampv(u1, -p.omega_max, p.omega_max);
    if (err_out) {
        err_out[3 * b] = e0;
        err_out[3 * b + 1] = e1;
        err_out[3 * b + 2] = e2;
    }
    if (K_out)
#pragma unroll
        for (int i = 0; i < 6; i++) K_out[6 * b + i] = K[i];
    if (status) status[b] = st;
}

__global__ __launch_bounds__(256) void lqr_gain_kernel(LqrDevParams p, int64_t B, const double *v_r,
                                                       const double *theta_r, int guard,
                                                       double *K_out, double *P_out, int32_t *status) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double v = v_r[b];
    if (guard && fabs(v) < 1e-6) v = 0.01;
    double K[6];
    M3 P;
    const bool ok = lqr_gain(p, v, theta_r[b], K, &P);
    if (!ok) { K[0] = 1; K[1] = 0; K[2] = 0; K[3] = 0; K[4] = 0; K[5] = 1; }
#pragma unroll
    for (int i = 0; i < 6; i++) K_out[6 * b + i] = K[i];
    if (P_out)
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) P_out[9 * b + 3 * i + j] = ok ? P.m[i][j] : NAN;
    if (status) status[b] = ok ? RMPC_OPTIMAL : RMPC_DARE_FALLBACK;
}

}  // namespace rmpc

using namespace rmpc;

hipError_t rmpc_launch_lqr_control(const LqrDevParams &p, int64_t B, const double *x,
                                   const double *x_ref, int xref_stride, const double *u_ref,
                                   int uref_stride, RmpcLqrCache *cache, double *u_out,
                                   double *err_out, double *K_out, double *P_out, int32_t *status,
                                   const int32_t *index, const int32_t *count, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    const int threads = RMPC_LQR_BLK;
    hipLaunchKernelGGL(lqr_control_kernel, dim3((unsigned)((B + threads - 1) / threads)), dim3(threads), 0,
                       stream, p, B, x, x_ref, xref_stride, u_ref, uref_stride, cache, u_out, err_out,
                       K_out, P_out, status, index, count);
    return hipGetLastError();
}

hipError_t rmpc_launch_lqr_gain(const LqrDevParams &p, int64_t B, const double *v_r,
                                const double *theta_r, int guard, double *K_out, double *P_out,
                                int32_t *status, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    const int threads = 256;
    hipLaunchKernelGGL(lqr_gain_kernel, dim3((unsigned)((B + threads - 1) / threads)), dim3(threads), 0,
                       stream, p, B, v_r, theta_r, guard, K_out, P_out, status);
    return hipGetLastError();
}
